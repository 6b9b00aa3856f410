// Pins the oracle's glibc sinf/cosf restatement (oracle/glibc_sincosf.inc) against this machine's libm,
// and measures what the round-1 "correctly rounded" pin would have changed in rBRIEF.
//
//   trig_pin exhaustive   every float x in [0, 2*pi]: restatement vs libm sinf / cosf / sincosf; also
//                         counts the x where libm differs from (float)cos((double)x) (the round-1 pin)
//   trig_pin angles       every float degree value d in [0, 360) (a superset of what fastAtan2 can
//                         return, ORBextractor.cc:103): at angle = d * factorPI (:112) where libm and the
//                         round-1 pin differ, does any of the 512 pattern offsets
//                         cvRound(x*b + y*a), cvRound(x*a - y*b) (:119-120) move?
//
// Output: one JSON object per mode on stdout.  Test infrastructure (tests/test_trig_pin.py).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../oracle/glibc_sincosf.inc"
#include "../oracle/pattern31_data.inc"

static const int kPattern[1024] = {ORACLE_PATTERN31_VALUES};

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
static float from_bits(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// libm through volatile function pointers: no constant folding, no builtin expansion
static float (*volatile p_sinf)(float) = sinf;
static float (*volatile p_cosf)(float) = cosf;
static void (*volatile p_sincosf)(float, float*, float*) = sincosf;

static int exhaustive() {
    const float two_pi = (float)(2 * M_PI);
    long n = 0, bad_sin = 0, bad_cos = 0, bad_sc = 0, cr_sin = 0, cr_cos = 0;
    for (uint32_t u = 0;; u++) {
        const float x = from_bits(u);
        if (!(x <= two_pi)) break;
        n++;
        const float s = p_sinf(x), c = p_cosf(x);
        float ss, cc;
        p_sincosf(x, &ss, &cc);
        if (bits(glibc_sincosf::sinf_(x)) != bits(s)) bad_sin++;
        if (bits(glibc_sincosf::cosf_(x)) != bits(c)) bad_cos++;
        if (bits(ss) != bits(s) || bits(cc) != bits(c)) bad_sc++;
        if (bits((float)std::sin((double)x)) != bits(s)) cr_sin++;
        if (bits((float)std::cos((double)x)) != bits(c)) cr_cos++;
    }
    std::printf("{\"mode\": \"exhaustive\", \"floats\": %ld, \"restatement_vs_libm_sinf\": %ld, "
                "\"restatement_vs_libm_cosf\": %ld, \"sincosf_vs_sinf_cosf\": %ld, "
                "\"libm_vs_correctly_rounded_sinf\": %ld, \"libm_vs_correctly_rounded_cosf\": %ld}\n",
                n, bad_sin, bad_cos, bad_sc, cr_sin, cr_cos);
    return (bad_sin || bad_cos || bad_sc) ? 1 : 0;
}

// the 512 pattern-point offsets under (a, b): cvRound (half-even) of the reference's expressions in the
// contraction form `fma_form` selects (0: separate multiply and add; 1: GCC -march=native FMA)
static void offsets(float a, float b, int fma_form, int* out) {
    for (int i = 0; i < 512; i++) {
        const float x = (float)kPattern[2 * i], y = (float)kPattern[2 * i + 1];
        float fy, fx;
        if (fma_form) {
            fy = std::fmaf(x, b, y * a);
            fx = std::fmaf(x, a, -(y * b));
        } else {
            fy = x * b + y * a;
            fx = x * a - y * b;
        }
        out[2 * i] = (int)std::nearbyint(fx);
        out[2 * i + 1] = (int)std::nearbyint(fy);
    }
}

static int angles() {
    const float factorPI = (float)(M_PI / 180.f);
    long ndeg = 0, ndiff = 0, moved[2] = {0, 0}, moved_pts[2] = {0, 0};
    std::vector<int> o1(1024), o2(1024);
    for (uint32_t u = 0;; u++) {
        const float deg = from_bits(u);
        if (!(deg < 360.f)) break;
        ndeg++;
        const float ang = deg * factorPI;
        const float c = p_cosf(ang), s = p_sinf(ang);
        const float ccr = (float)std::cos((double)ang), scr = (float)std::sin((double)ang);
        if (bits(c) == bits(ccr) && bits(s) == bits(scr)) continue;
        ndiff++;
        for (int form = 0; form < 2; form++) {
            offsets(c, s, form, o1.data());
            offsets(ccr, scr, form, o2.data());
            int np = 0;
            for (int i = 0; i < 512; i++) np += o1[2 * i] != o2[2 * i] || o1[2 * i + 1] != o2[2 * i + 1];
            if (np) {
                moved[form]++;
                moved_pts[form] += np;
            }
        }
    }
    std::printf("{\"mode\": \"angles\", \"degree_floats\": %ld, \"libm_ne_correctly_rounded\": %ld, "
                "\"angles_with_moved_offsets_uncontracted\": %ld, \"moved_points_uncontracted\": %ld, "
                "\"angles_with_moved_offsets_fma\": %ld, \"moved_points_fma\": %ld}\n",
                ndeg, ndiff, moved[0], moved_pts[0], moved[1], moved_pts[1]);
    return 0;
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "exhaustive";
    if (!std::strcmp(mode, "exhaustive")) return exhaustive();
    if (!std::strcmp(mode, "angles")) return angles();
    std::fprintf(stderr, "usage: trig_pin exhaustive|angles\n");
    return 2;
}
