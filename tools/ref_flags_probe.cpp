// Compiled with the REFERENCE's own flags (CMakeLists.txt:10-11,18: -O3 -march=native -std=c++11; on an
// FMA-capable x86-64 host), this translation unit restates the float expressions of the path exactly as
// the reference writes them, so that GCC makes the same contraction decisions it makes for
// src/ORBextractor.cc and src/ORBmatcher.cc.  tools/ref_flags_check.cpp (built -ffp-contract=off)
// compares the results with the explicit forms the oracle and the kernels use.  Test infrastructure
// (tests/test_trig_pin.py); nothing here is linked into the product or the oracle.
#include <cmath>
#include <xmmintrin.h>

using namespace std;

namespace probe {

// OpenCV 3.2 cvRound(float) on x86-64 SSE2 (core/fast_math.hpp)
static inline int cvRound(float value) { return _mm_cvtss_si32(_mm_set_ss(value)); }

struct Point { int x, y; };

// computeOrbDescriptor's trigonometry and sample offsets (ORBextractor.cc:112-120): for keypoint angle
// `kpt_angle` (degrees), the (dx, dy) of each of the 512 pattern points
void orb_offsets(float kpt_angle, const Point* pattern, int* out) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = (float)kpt_angle * factorPI;
    float a = (float)cos(angle), b = (float)sin(angle);
    for (int i = 0; i < 512; ++i) {
        out[2 * i] = cvRound(pattern[i].x * a - pattern[i].y * b);
        out[2 * i + 1] = cvRound(pattern[i].x * b + pattern[i].y * a);
    }
}

// computeOrbDescriptor itself on a blurred patch (centre pointer, row step), the GET_VALUE form of
// ORBextractor.cc:118-144
void orb_descriptor(float kpt_angle, const unsigned char* center, int step, const Point* pattern,
                    unsigned char* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = (float)kpt_angle * factorPI;
    float a = (float)cos(angle), b = (float)sin(angle);
#define PROBE_GET(idx) \
    center[cvRound(pattern[idx].x * b + pattern[idx].y * a) * step + cvRound(pattern[idx].x * a - pattern[idx].y * b)]
    for (int i = 0; i < 32; ++i, pattern += 16) {
        int t0, t1, val;
        t0 = PROBE_GET(0); t1 = PROBE_GET(1); val = t0 < t1;
        t0 = PROBE_GET(2); t1 = PROBE_GET(3); val |= (t0 < t1) << 1;
        t0 = PROBE_GET(4); t1 = PROBE_GET(5); val |= (t0 < t1) << 2;
        t0 = PROBE_GET(6); t1 = PROBE_GET(7); val |= (t0 < t1) << 3;
        t0 = PROBE_GET(8); t1 = PROBE_GET(9); val |= (t0 < t1) << 4;
        t0 = PROBE_GET(10); t1 = PROBE_GET(11); val |= (t0 < t1) << 5;
        t0 = PROBE_GET(12); t1 = PROBE_GET(13); val |= (t0 < t1) << 6;
        t0 = PROBE_GET(14); t1 = PROBE_GET(15); val |= (t0 < t1) << 7;
        desc[i] = (unsigned char)val;
    }
#undef PROBE_GET
}

// CheckDistEpipolarLine (ORBmatcher.cc:140-157) with F12 row-major; returns dsqr and the verdict
bool epipolar(float x1, float y1, float x2, float y2, const float* F, double sigma2, float* dsqr_out) {
    const float a = x1 * F[0] + y1 * F[3] + F[6];
    const float b = x1 * F[1] + y1 * F[4] + F[7];
    const float c = x1 * F[2] + y1 * F[5] + F[8];
    const float num = a * x2 + b * y2 + c;
    const float den = a * a + b * b;
    if (den == 0) {
        *dsqr_out = -1;
        return false;
    }
    const float dsqr = num * num / den;
    *dsqr_out = dsqr;
    return dsqr < 3.84 * sigma2;
}

// SearchForTriangulation's epipole gate (ORBmatcher.cc:743-749)
bool epipole_near(float ex, float ey, float x2, float y2, float scale) {
    const float distex = ex - x2;
    const float distey = ey - y2;
    return distex * distex + distey * distey < 100 * scale;
}

}  // namespace probe
