// glibc's single-precision sinf/cosf (sysdeps/ieee754/flt-32: sincosf.h, sincosf_data.c; glibc 2.28-2.35,
// the x86-64 FMA ifunc variant an AVX2 host runs) as device code.  The reference computes the BRIEF
// rotation as `(float)cos(angle), (float)sin(angle)` on a float angle (ORBextractor.cc:113) — glibc
// cosf/sinf, merged by GCC -O3 into one sincosf — and cv::ORB does the same inside OpenCV (the birdview
// stream, Frame.cc:329-342).  glibc does not round correctly (a double polynomial rounded once), so the
// kernels evaluate its exact operation sequence: double arithmetic, every `a + b*c` of the FMA build one
// fused multiply-add.  Valid for 0 <= |x| < 120 (the path's angles are in [0, 2*pi]).  Pinned on the host
// against libm over every float in [0, 2*pi] (tools/trig_pin.cpp, tests/test_trig_pin.py, which also
// checks this file's table against the oracle's).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbgpu {

// sincosf_data.c, as constants: __sincosf_table[1] is entry 0 with the cosine polynomial negated
// (quadrants 2 and 3), expressed here as a sign applied to c0..c4 (multiplying by -1 is exact).  No table
// in memory: a dynamically indexed one lands in scratch.
constexpr double kTrigHpiInv = 0x1.45F306DC9C883p+23;   // 2/pi * 2^24 (x86-64: no TOINT_INTRINSICS)
constexpr double kTrigHpi = 0x1.921FB54442D18p0;
constexpr double kTrigC0 = 0x1p0, kTrigC1 = -0x1.ffffffd0c621cp-2, kTrigC2 = 0x1.55553e1068f19p-5,
                 kTrigC3 = -0x1.6c087e89a359dp-10, kTrigC4 = 0x1.99343027bf8c3p-16;
constexpr double kTrigS1 = -0x1.555545995a603p-3, kTrigS2 = 0x1.1107605230bc4p-7, kTrigS3 = -0x1.994eb3774cf24p-13;

__device__ __forceinline__ uint32_t trig_abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

// sinf_poly: n even -> sine polynomial, odd -> cosine polynomial scaled by cs (+-1: the table entry);
// every a + b*c of the FMA build is one fused multiply-add
__device__ __forceinline__ float glibc_sinf_poly(double x, double x2, double cs, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = __builtin_fma(x2, kTrigS3, kTrigS2);
        const double x7 = x3 * x2;
        const double s = __builtin_fma(x3, kTrigS1, x);
        return (float)__builtin_fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = __builtin_fma(x2, cs * kTrigC4, cs * kTrigC3);
    const double c1 = __builtin_fma(x2, cs * kTrigC1, cs * kTrigC0);
    const double x6 = x4 * x2;
    const double c = __builtin_fma(x4, cs * kTrigC2, c1);
    return (float)__builtin_fma(x6, c2, c);
}

// sincosf(y) for |y| < 120: *s = sinf(y), *c = cosf(y), bit-identical to glibc's FMA variant
__device__ __forceinline__ void glibc_sincosf(float y, float* s, float* c) {
    double x = y;
    if (trig_abstop12(y) < trig_abstop12(0x1.921FB6p-1f)) {   // |y| < pi/4 (top 12 bits)
        const double x2 = x * x;
        if (trig_abstop12(y) < trig_abstop12(0x1p-12f)) {
            *s = y;
            *c = 1.0f;
            return;
        }
        *s = glibc_sinf_poly(x, x2, 1.0, 0);
        *c = glibc_sinf_poly(x, x2, 1.0, 1);
        return;
    }
    // reduce_fast (!TOINT_INTRINSICS): n = round(x * 2/pi) by the shift trick, x - n*pi/2 fused
    const double r = x * kTrigHpiInv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = __builtin_fma(-(double)n, kTrigHpi, x);
    const double sg = ((n + 1) & 2) ? -1.0 : 1.0;   // sign[n & 3] = {1, -1, -1, 1}
    const double cs = (n & 2) ? -1.0 : 1.0;         // table entry 1 for quadrants 2, 3
    *s = glibc_sinf_poly(x * sg, x * x, cs, n);
    *c = glibc_sinf_poly(x * sg, x * x, cs, n ^ 1);
}

}  // namespace orbgpu
