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

struct SinCosTable {
    double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

// sincosf_data.c: entry 1 negates the cosine polynomial (quadrants 2, 3)
__device__ __forceinline__ SinCosTable glibc_sincos_table(int neg) {
    SinCosTable t;
    t.sign[0] = 1.0; t.sign[1] = -1.0; t.sign[2] = -1.0; t.sign[3] = 1.0;
    t.hpi_inv = 0x1.45F306DC9C883p+23;
    t.hpi = 0x1.921FB54442D18p0;
    const double sg = neg ? -1.0 : 1.0;
    t.c0 = sg * 0x1p0;
    t.c1 = sg * -0x1.ffffffd0c621cp-2;
    t.c2 = sg * 0x1.55553e1068f19p-5;
    t.c3 = sg * -0x1.6c087e89a359dp-10;
    t.c4 = sg * 0x1.99343027bf8c3p-16;
    t.s1 = -0x1.555545995a603p-3;
    t.s2 = 0x1.1107605230bc4p-7;
    t.s3 = -0x1.994eb3774cf24p-13;
    return t;
}

__device__ __forceinline__ uint32_t trig_abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

// sinf_poly: n even -> sine polynomial, odd -> cosine polynomial (fma = the FMA build's contractions)
__device__ __forceinline__ float glibc_sinf_poly(double x, double x2, const SinCosTable& p, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = __builtin_fma(x2, p.s3, p.s2);
        const double x7 = x3 * x2;
        const double s = __builtin_fma(x3, p.s1, x);
        return (float)__builtin_fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = __builtin_fma(x2, p.c4, p.c3);
    const double c1 = __builtin_fma(x2, p.c1, p.c0);
    const double x6 = x4 * x2;
    const double c = __builtin_fma(x4, p.c2, c1);
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
        const SinCosTable p = glibc_sincos_table(0);
        *s = glibc_sinf_poly(x, x2, p, 0);
        *c = glibc_sinf_poly(x, x2, p, 1);
        return;
    }
    // reduce_fast (!TOINT_INTRINSICS): n = round(x * 2/pi) by the shift trick, x - n*pi/2 fused
    const double r = x * 0x1.45F306DC9C883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = __builtin_fma(-(double)n, 0x1.921FB54442D18p0, x);
    const SinCosTable p = glibc_sincos_table((n & 2) != 0);
    const double sg = p.sign[n & 3];
    *s = glibc_sinf_poly(x * sg, x * x, p, n);
    *c = glibc_sinf_poly(x * sg, x * x, p, n ^ 1);
}

}  // namespace orbgpu
