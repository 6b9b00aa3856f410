// Built with -ffp-contract=off and linked with tools/ref_flags_probe.cpp (built with the reference's
// -O3 -march=native -std=c++11).  Checks that the explicit float forms the oracle and the kernels use
// (oracle/orb_oracle.cpp, csrc/extract_kernels.hip, csrc/hamming_kernels.hip) are the ones GCC produces
// for the reference's expressions, and how often the uncontracted forms would differ.  Prints one JSON
// object; exit status 1 on any mismatch.  Test infrastructure (tests/test_trig_pin.py).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../oracle/glibc_sincosf.inc"
#include "../oracle/pattern31_data.inc"

namespace probe {
struct Point { int x, y; };
void orb_offsets(float kpt_angle, const Point* pattern, int* out);
void orb_descriptor(float kpt_angle, const unsigned char* center, int step, const Point* pattern, unsigned char* desc);
bool epipolar(float x1, float y1, float x2, float y2, const float* F, double sigma2, float* dsqr_out);
bool epipole_near(float ex, float ey, float x2, float y2, float scale);
}  // namespace probe

static const int kPatternInts[1024] = {ORACLE_PATTERN31_VALUES};

static float from_bits(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// the oracle's forms (orb_oracle.cpp computeOrbDescriptor): y offset fma(x, b, y*a), x offset
// fma(x, a, -(y*b)); `fused` = 0 gives the uncontracted forms
static void offsets(float deg, int fused, int* out) {
    const float factorPI = (float)(M_PI / 180.f);
    const float ang = deg * factorPI;
    const float a = glibc_sincosf::cosf_(ang), b = glibc_sincosf::sinf_(ang);
    for (int i = 0; i < 512; i++) {
        const float x = (float)kPatternInts[2 * i], y = (float)kPatternInts[2 * i + 1];
        const float fx = fused ? std::fmaf(x, a, -(y * b)) : x * a - y * b;
        const float fy = fused ? std::fmaf(x, b, y * a) : x * b + y * a;
        out[2 * i] = (int)std::nearbyint(fx);
        out[2 * i + 1] = (int)std::nearbyint(fy);
    }
}

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 997;
    probe::Point pts[512];
    for (int i = 0; i < 512; i++) pts[i] = {kPatternInts[2 * i], kPatternInts[2 * i + 1]};
    long nang = 0, bad_off = 0, sep_differs = 0;
    std::vector<int> got(1024), want(1024), sep(1024);
    std::vector<float> sensitive;
    for (uint32_t u = 0;; u += stride) {
        const float deg = from_bits(u);
        if (!(deg < 360.f)) break;
        nang++;
        probe::orb_offsets(deg, pts, got.data());
        offsets(deg, 1, want.data());
        offsets(deg, 0, sep.data());
        if (got != want) bad_off++;
        if (sep != want) {
            sep_differs++;
            if (sensitive.size() < 4096) sensitive.push_back(deg);
        }
    }
    // descriptors at the angles where contraction matters, on random 37x37 patches
    std::mt19937 rng(12345);
    long ndesc = 0, bad_desc = 0;
    std::vector<unsigned char> patch(37 * 37);
    for (float deg : sensitive) {
        for (auto& p : patch) p = (unsigned char)(rng() & 255);
        const unsigned char* center = patch.data() + 18 * 37 + 18;
        unsigned char d1[32], d2[32];
        probe::orb_descriptor(deg, center, 37, pts, d1);
        offsets(deg, 1, want.data());
        for (int i = 0; i < 32; i++) {
            int val = 0;
            for (int k = 0; k < 8; k++) {
                const int p0 = 16 * i + 2 * k, p1 = p0 + 1;
                const int t0 = center[want[2 * p0 + 1] * 37 + want[2 * p0]];
                const int t1 = center[want[2 * p1 + 1] * 37 + want[2 * p1]];
                val |= (t0 < t1) << k;
            }
            d2[i] = (unsigned char)val;
        }
        ndesc++;
        bad_desc += std::memcmp(d1, d2, 32) != 0;
    }
    // CheckDistEpipolarLine / epipole gate: the fused forms vs the probe, on random geometry
    std::uniform_real_distribution<float> U(-1.f, 1.f), P(0.f, 1280.f);
    long nepi = 0, bad_epi = 0, sep_epi = 0, bad_gate = 0, sep_gate = 0;
    for (int it = 0; it < 1000000; it++) {
        float F[9];
        for (float& f : F) f = U(rng) * (it & 1 ? 1e-3f : 1.f);
        const float x1 = P(rng), y1 = P(rng) * 0.6f, x2 = P(rng), y2 = P(rng) * 0.6f;
        float dq;
        probe::epipolar(x1, y1, x2, y2, F, 1.44, &dq);
        const float a = std::fmaf(x1, F[0], y1 * F[3]) + F[6];
        const float b = std::fmaf(x1, F[1], y1 * F[4]) + F[7];
        const float c = std::fmaf(y1, F[5], x1 * F[2]) + F[8];
        const float num = std::fmaf(b, y2, a * x2) + c;
        const float den = std::fmaf(a, a, b * b);
        const float dsqr = den == 0 ? -1.f : num * num / den;
        const float as = x1 * F[0] + y1 * F[3] + F[6], bs = x1 * F[1] + y1 * F[4] + F[7];
        const float cs = x1 * F[2] + y1 * F[5] + F[8];
        const float nums = as * x2 + bs * y2 + cs, dens = as * as + bs * bs;
        const float dsqs = dens == 0 ? -1.f : nums * nums / dens;
        nepi++;
        bad_epi += bits(dq) != bits(dsqr);
        sep_epi += bits(dsqs) != bits(dsqr);
        const float ex = P(rng), ey = P(rng) * 0.6f, sc = 1.f + (float)(it % 8) * 0.2f;
        const float dx = ex - x2, dy = ey - y2;
        const bool g = probe::epipole_near(ex, ey, x2, y2, sc);
        bad_gate += g != (std::fmaf(dx, dx, dy * dy) < 100 * sc);
        sep_gate += (dx * dx + dy * dy < 100 * sc) != (std::fmaf(dx, dx, dy * dy) < 100 * sc);
    }
    std::printf("{\"angles\": %ld, \"angle_stride\": %u, \"offsets_mismatch_vs_fused_form\": %ld, "
                "\"angles_where_uncontracted_differs\": %ld, \"descriptors\": %ld, \"descriptor_mismatch\": %ld, "
                "\"epipolar_cases\": %ld, \"epipolar_dsqr_mismatch\": %ld, \"epipolar_uncontracted_differs\": %ld, "
                "\"epipole_gate_mismatch\": %ld, \"epipole_gate_uncontracted_differs\": %ld}\n",
                nang, stride, bad_off, sep_differs, ndesc, bad_desc, nepi, bad_epi, sep_epi, bad_gate, sep_gate);
    return (bad_off || bad_desc || bad_epi || bad_gate) ? 1 : 0;
}
