// Birdview ORB stream of Frame::Frame (reference src/Frame.cc:318-342) on gfx950 — SURVEY §8(f) row 3.
//
// The reference runs OpenCV's own cv::ORB (not ORBextractor) on the birdview image:
//     mask = birdviewMask with the vehicle footprint zeroed          Frame.cc:320-327
//     cv::ORB::create(2000)->detect(img, kps, mask)                  Frame.cc:329-330
//     cv::cornerSubPix(img, pts, (5,5), (-1,-1), EPS|ITER 40 0.001)  Frame.cc:331-341
//     cv::ORB::compute(img, kps, desc)                               Frame.cc:342
// restated from OpenCV 3.2 orb.cpp / keypoint.cpp / cornersubpix.cpp / samplers.cpp (the oracle's
// oracle/cvorb_oracle.inc states each detail).
//
// Device side: pyramid (+ mask pyramid) by per-level resize launches, one FAST score-map launch over
// all levels, a count / scan / emit pass that writes the masked, border-filtered, non-max-suppressed
// candidates of every level in raster order together with their Harris responses, the 7x7 blurred
// pyramid, and per-keypoint IC angle, cornerSubPix and rBRIEF kernels.
// Host side: KeyPointsFilter::retainBest (std::nth_element + std::partition) — the reference's own
// sequential selection, whose output ORDER is libstdc++'s introselect order, so it runs on the host
// with the same library call the OpenCV build makes.
#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "glibc_trig.h"
#include "orbgpu_ctx.h"

namespace orbgpu {
namespace {

constexpr int kBirdMaxLevels = ORBGPU_MAX_LEVELS;
constexpr int kSubWin = 5;                     // cornerSubPix win (5,5): 11 x 11 window, 13 x 13 patch
constexpr int kSubW = 2 * kSubWin + 1;
constexpr int kSubP = kSubW + 2;

struct BirdLevel {
    int w, h, pitch;
    int pad;
    long long off;     // byte offset of the level in a pyramid buffer
    float scale;       // getScale(level) = (float)pow(scaleFactor, level)
    int nfeat;         // nfeaturesPerLevel
};

struct BirdGeom {
    int nlevels, W, H, edge, fastTh;
    int variant;           // ORB_VARIANT_RESIZE_GENERIC / ORB_VARIANT_BLUR_HALFUP (orb_bird_params.variant)
    float harris_scale4;   // (1 / (4 * 7 * 255.f))^4
    int gk[8];             // 7-tap Gaussian sigma 2, 8-bit fixed point
    int umax[16];          // orb.cpp computeKeyPoints u_max (halfPatchSize 15)
    BirdLevel L[kBirdMaxLevels];
};

// candidate record of the emit pass
struct BirdCand {
    int xy;          // x | y << 16 (level coordinates)
    int level;
    int score;       // FAST score (KeyPoint::response before Harris)
    float harris;    // HarrisResponses(blockSize 7, k 0.04)
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int reflect101_d(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

/* ---------------- pyramid: cv::resize(prev level, INTER_LINEAR) (orb.cpp detectAndCompute) --------
 * plane 1 is the mask pyramid: resize of the previous (thresholded) mask level, then
 * threshold(254, 0, THRESH_TOZERO). */
__global__ __launch_bounds__(256) void k_bird_resize(const BirdGeom* __restrict__ g, int l,
                                                     const ResizeCoef* __restrict__ coef, uint8_t* __restrict__ pyr,
                                                     uint8_t* __restrict__ mpyr) {
    const BirdLevel D = g->L[l], S = g->L[l - 1];
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= D.w) return;
    uint8_t* base = blockIdx.z ? mpyr : pyr;
    const ResizeCoef cx = coef[x], cy = coef[D.w + y];
    const uint8_t* r0 = base + S.off + (long long)cy.s0 * S.pitch;
    const uint8_t* r1 = base + S.off + (long long)cy.s1 * S.pitch;
    const int h0 = r0[cx.s0] * cx.c0 + r0[cx.s1] * cx.c1;
    const int h1 = r1[cx.s0] * cx.c0 + r1[cx.s1] * cx.c1;
    int v = (g->variant & ORB_VARIANT_RESIZE_GENERIC)
                ? min((cy.c0 * h0 + cy.c1 * h1 + (1 << 21)) >> 22, 255)   // generic FixedPtCast
                : (((cy.c0 * (h0 >> 4)) >> 16) + ((cy.c1 * (h1 >> 4)) >> 16) + 2) >> 2;
    if (blockIdx.z) v = v > 254 ? v : 0;
    base[D.off + (long long)y * D.pitch + x] = (uint8_t)v;
}

/* ---------------- FAST 9/16 score map (cv::FAST, threshold fastThreshold, TYPE_9_16) -------------
 * score = (max over 9-arcs of the arc's weakest |v - p|, same sign) - 1 when that exceeds the
 * threshold (OpenCV cornerScore<16>), else 0.  Only rows/columns [edge-1, dim-edge] are scored: every
 * candidate that survives runByImageBorder(edge) lies in [edge, dim-edge) and its NMS neighbours one
 * pixel further out.  rows: (level, y) table. */
__device__ __forceinline__ int fast_score_at(const uint8_t* c, int P, int t) {
    const int v = c[0];
    int d[16];
    d[0] = v - c[3 * P];
    d[1] = v - c[1 + 3 * P];
    d[2] = v - c[2 + 2 * P];
    d[3] = v - c[3 + 1 * P];
    d[4] = v - c[3];
    d[5] = v - c[3 - 1 * P];
    d[6] = v - c[2 - 2 * P];
    d[7] = v - c[1 - 3 * P];
    d[8] = v - c[-3 * P];
    d[9] = v - c[-1 - 3 * P];
    d[10] = v - c[-2 - 2 * P];
    d[11] = v - c[-3 - 1 * P];
    d[12] = v - c[-3];
    d[13] = v - c[-3 + 1 * P];
    d[14] = v - c[-2 + 2 * P];
    d[15] = v - c[-1 + 3 * P];
    int m3[16], x3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        m3[k] = min(min(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
        x3[k] = max(max(d[k], d[(k + 1) & 15]), d[(k + 2) & 15]);
    }
    int A = 0, Bn = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        A = max(A, min(min(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]));
        Bn = min(Bn, max(max(x3[k], x3[(k + 3) & 15]), x3[(k + 6) & 15]));
    }
    const int s = max(A, -Bn);
    return s > t ? s - 1 : 0;
}

__global__ __launch_bounds__(256) void k_bird_fast(const BirdGeom* __restrict__ g, const int2* __restrict__ rows,
                                                   const uint8_t* __restrict__ pyr, uint8_t* __restrict__ score) {
    const int2 r = rows[blockIdx.y];
    const BirdLevel L = g->L[r.x];
    const int x = g->edge - 1 + blockIdx.x * 256 + threadIdx.x;
    if (x > L.w - g->edge) return;
    const long long o = L.off + (long long)r.y * L.pitch + x;
    const uint8_t* c = pyr + o;
    const int P = L.pitch, t = g->fastTh, v = c[0];
    // compass prefilter (a 9-arc holds two cyclically adjacent compass points): necessary for a corner
    const int p0 = c[3 * P], p4 = c[3], p8 = c[-3 * P], p12 = c[-3];
    const int hi = v + t, lo = v - t;
    const int bm = (p0 > hi) | ((p4 > hi) << 1) | ((p8 > hi) << 2) | ((p12 > hi) << 3);
    const int dm = (p0 < lo) | ((p4 < lo) << 1) | ((p8 < lo) << 2) | ((p12 < lo) << 3);
    score[o] = ((0xFAC8 >> bm) | (0xFAC8 >> dm)) & 1 ? (uint8_t)fast_score_at(c, P, t) : (uint8_t)0;
}

/* ---------------- candidates: NMS + runByPixelsMask + runByImageBorder, raster order ------------
 * One wave per (level, y) row of [edge, h-edge); mode 0 counts, mode 1 writes at the scanned
 * offsets with the Harris response (orb.cpp HarrisResponses, blockSize 7, HARRIS_K 0.04f: integer
 * gradient sums, then the float formula in the reference's evaluation order). */
template <int kMode>
__global__ __launch_bounds__(256) void k_bird_cands(const BirdGeom* __restrict__ g, const int2* __restrict__ rows,
                                                    int nrows, const uint8_t* __restrict__ pyr,
                                                    const uint8_t* __restrict__ mpyr, const uint8_t* __restrict__ score,
                                                    int* __restrict__ rowcnt, const int* __restrict__ rowoff,
                                                    BirdCand* __restrict__ out) {
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wid >= nrows) return;
    const int2 r = rows[wid];
    const BirdLevel L = g->L[r.x];
    const int e = g->edge, P = L.pitch;
    int pos = kMode ? rowoff[wid] : 0;
    for (int x0 = e; x0 < L.w - e; x0 += 64) {
        const int x = x0 + lane;
        bool keep = false;
        int s = 0;
        const long long o = L.off + (long long)r.y * P + x;
        if (x < L.w - e) {
            s = score[o];
            if (s) {
                const uint8_t* q = score + o;
                keep = s > q[-1] && s > q[1] && s > q[-P - 1] && s > q[-P] && s > q[-P + 1] && s > q[P - 1] &&
                       s > q[P] && s > q[P + 1];
                if (keep && mpyr) keep = mpyr[o] != 0;
            }
        }
        const unsigned long long m = __ballot(keep);
        if (kMode) {
            // Harris responses, one candidate at a time over the whole wave: lane q < 49 takes pixel
            // (q / 7, q % 7) of the 7x7 block, the integer sums are wave reductions (order-free)
            float hr = 0.f;
            unsigned long long mm = m;
            while (mm) {
                const int src = __ffsll((long long)mm) - 1;
                mm &= mm - 1;
                const long long oc = o - lane + src;   // the candidate's pixel (same row, x0 + src)
                int ixx = 0, iyy = 0, ixy = 0;
                if (lane < 49) {
                    const int i = lane / 7, j = lane - 7 * (lane / 7);
                    const uint8_t* q = pyr + oc + (long long)(i - 3) * P + (j - 3);
                    const int Ix = (q[1] - q[-1]) * 2 + (q[-P + 1] - q[-P - 1]) + (q[P + 1] - q[P - 1]);
                    const int Iy = (q[P] - q[-P]) * 2 + (q[P - 1] - q[-P - 1]) + (q[P + 1] - q[-P + 1]);
                    ixx = Ix * Ix;
                    iyy = Iy * Iy;
                    ixy = Ix * Iy;
                }
#pragma unroll
                for (int sft = 32; sft > 0; sft >>= 1) {
                    ixx += __shfl_xor(ixx, sft);
                    iyy += __shfl_xor(iyy, sft);
                    ixy += __shfl_xor(ixy, sft);
                }
                const float fa = (float)ixx, fb = (float)iyy, fc = (float)ixy;
                const float h = (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * g->harris_scale4;
                if (lane == src) hr = h;
            }
            if (keep) {
                const int rank = __popcll(m & ((1ull << lane) - 1));
                BirdCand c;
                c.xy = x | (r.y << 16);
                c.level = r.x;
                c.score = s;
                c.harris = hr;
                out[pos + rank] = c;
            }
        }
        pos += __popcll(m);
    }
    if (!kMode && lane == 0) rowcnt[wid] = pos;
}

// exclusive scan of the row counts (one block); per-level counts from the level row ranges
__global__ __launch_bounds__(1024) void k_bird_scan(const int* __restrict__ rowcnt, int nrows,
                                                    const int* __restrict__ lvl_row0, int nlevels,
                                                    int* __restrict__ rowoff, int* __restrict__ lvlcnt) {
    __shared__ int s_w[16];
    __shared__ int s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int base = 0; base < nrows; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < nrows ? rowcnt[i] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        int pre = 0;
        for (int k = 0; k < wv; k++) pre += s_w[k];
        const int carry = s_carry;
        if (i < nrows) rowoff[i] = carry + pre + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = carry + pre + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) rowoff[nrows] = s_carry;
    __syncthreads();
    if ((int)threadIdx.x < nlevels) lvlcnt[threadIdx.x] = rowoff[lvl_row0[threadIdx.x + 1]] - rowoff[lvl_row0[threadIdx.x]];
}

/* ---------------- GaussianBlur(7x7, sigma 2, REFLECT_101) of every level ROI ----------------------
 * Integer separable filter; the column pass rounds half-to-even on columns x < (w & ~3) (OpenCV's SSE2
 * SymmColumnVec_32s8u) and half-up on the tail (FixedPtCastEx) — the oracle's gauss7_blur. */
__global__ __launch_bounds__(256) void k_bird_blur(const BirdGeom* __restrict__ g, const int2* __restrict__ rows,
                                                   const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur) {
    const int2 r = rows[blockIdx.y];
    const BirdLevel L = g->L[r.x];
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= L.w) return;
    const uint8_t* src = pyr + L.off;
    int xs[7];
#pragma unroll
    for (int j = 0; j < 7; j++) xs[j] = reflect101_d(x + j - 3, L.w);
    int S = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const uint8_t* row = src + (long long)reflect101_d(r.y + i - 3, L.h) * L.pitch;
        int acc = 0;
#pragma unroll
        for (int j = 0; j < 7; j++) acc += g->gk[j] * row[xs[j]];
        S += g->gk[i] * acc;
    }
    const int q = S >> 16, rem = S & 0xFFFF;
    int v;
    // ORB_VARIANT_BLUR_HALFUP: half-up everywhere (no SSE2 body)
    if (x < ((g->variant & ORB_VARIANT_BLUR_HALFUP) ? 0 : (L.w & ~3))) v = rem > 32768 ? q + 1 : (rem < 32768 ? q : q + (q & 1));
    else v = (S + 32768) >> 16;
    blur[L.off + (long long)r.y * L.pitch + x] = (uint8_t)min(max(v, 0), 255);
}

/* ---------------- ICAngles + pt *= layerScale (orb.cpp computeKeyPoints tail) ----------------------
 * One wave per keypoint: lane v in [0, 31) sums row v-15 of the circular patch (integer moments,
 * order-free), then cv::fastAtan2. */
constexpr float kAtanScale = (float)(180 / 3.14159265358979323846);
constexpr float kP1 = 0.9997878412794807f * kAtanScale;
constexpr float kP3 = -0.3258083974640975f * kAtanScale;
constexpr float kP5 = 0.1555786518463281f * kAtanScale;
constexpr float kP7 = -0.04432655554792128f * kAtanScale;
constexpr float kFactorPI = (float)(3.14159265358979323846 / 180.f);

__device__ __forceinline__ float cv_fast_atan2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((kP7 * c2 + kP5) * c2 + kP3) * c2 + kP1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((kP7 * c2 + kP5) * c2 + kP3) * c2 + kP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__global__ __launch_bounds__(256) void k_bird_angle(const BirdGeom* __restrict__ g, const uint8_t* __restrict__ pyr,
                                                    orb_keypoint* __restrict__ kps, int n) {
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (k >= n) return;
    orb_keypoint kp = kps[k];
    const BirdLevel L = g->L[kp.octave];
    const uint8_t* center = pyr + L.off + (long long)(int)rintf(kp.y) * L.pitch + (int)rintf(kp.x);
    int m10 = 0, m01 = 0;
    if (lane < 31) {
        const int v = lane - 15, av = v < 0 ? -v : v;
        const int d = g->umax[av];
        const uint8_t* row = center + v * L.pitch;
        int sum = 0, mom = 0;
        for (int u = -d; u <= d; u++) {
            const int val = row[u];
            sum += val;
            mom += u * val;
        }
        m10 = mom;
        m01 = v * sum;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m10 += __shfl_xor(m10, o);
        m01 += __shfl_xor(m01, o);
    }
    if (lane == 0) {
        kp.angle = cv_fast_atan2((float)m01, (float)m10);
        kp.x = kp.x * L.scale;
        kp.y = kp.y * L.scale;
        kps[k] = kp;
    }
}

/* ---------------- cv::cornerSubPix(win (5,5), zeroZone (-1,-1)) --------------------------------------
 * One wavefront per point.  Per iteration: lanes 0..12 generate the 13 rows of the getRectSubPix_8u32f
 * patch (each row is a 13-step float recurrence) into LDS; lanes then compute the 121 per-pixel terms
 * (gxx, gxy, gyy, gxx*px + gxy*py, gxy*px + gyy*py, in double) into LDS; lanes 0..4 each run ONE of the
 * five accumulations sequentially in the reference's (i, j) order, so every double sum is bit-identical
 * to the sequential code; the sums are broadcast and every lane updates the point identically. */
struct SubpixSrc {
    const uint8_t* img;
    int pitch, W, H;
};

constexpr int kSubE = kSubW * kSubW;   // 121 window pixels

// one patch row r of getRectSubPix(img, (13, 13), (cx, cy)) into out[13]; interior windows read the
// point's cached neighbourhood (`cache`, pitch kSubC, origin (cx0, cy0)) when they lie inside it
constexpr int kSubC = 32;
__device__ __forceinline__ void subpix_row(const SubpixSrc& s, bool inside, int ipx, int ipy, float a, float b,
                                           double sd, int r, float (&out)[kSubP], const uint8_t* cache, int cx0,
                                           int cy0) {
    if (inside) {
        const float a12 = a * (1.f - b), a22 = a * b, b1 = 1.f - b, b2 = b;
        const bool cached = cache && ipx >= cx0 && ipx + kSubP < cx0 + kSubC && ipy >= cy0 &&
                            ipy + kSubP < cy0 + kSubC;
        const uint8_t* s0 = cached ? cache + (ipy + r - cy0) * kSubC + (ipx - cx0)
                                   : s.img + (long long)(ipy + r) * s.pitch + ipx;
        const uint8_t* s1 = s0 + (cached ? kSubC : s.pitch);
        float prev = (1 - a) * (b1 * s0[0] + b2 * s1[0]);
#pragma unroll
        for (int j = 0; j < kSubP; j++) {
            const float t = a12 * s0[j + 1] + a22 * s1[j + 1];
            out[j] = prev + t;
            prev = (float)(t * sd);
        }
    } else {
        const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
        const int y0 = min(max(ipy + r, 0), s.H - 1), y1 = min(max(ipy + r + 1, 0), s.H - 1);
        const uint8_t* s0 = s.img + (long long)y0 * s.pitch;
        const uint8_t* s1 = s.img + (long long)y1 * s.pitch;
#pragma unroll
        for (int j = 0; j < kSubP; j++) {
            const int x0 = min(max(ipx + j, 0), s.W - 1), x1 = min(max(ipx + j + 1, 0), s.W - 1);
            out[j] = (float)s0[x0] * a11 + (float)s0[x1] * a12 + (float)s1[x0] * a21 + (float)s1[x1] * a22;
        }
    }
}

__global__ __launch_bounds__(256) void k_bird_subpix(SubpixSrc s, const float* __restrict__ wmask, float* pts,
                                                     int stride, int n, int max_iters, double eps2, int edge,
                                                     int* __restrict__ keep) {
    __shared__ float s_patch[4][kSubP * kSubP + 3];
    __shared__ double s_terms[4][5 * kSubE + 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_cache[4][kSubC * kSubC];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int k = blockIdx.x * 4 + wv;
    if (k >= n) return;
    float* patch = s_patch[wv];
    double* terms = s_terms[wv];
    float* pt = pts + (long long)k * stride;
    const float cTx = pt[0], cTy = pt[1];
    // the 32 x 32 neighbourhood of the start point, staged once (windows within +-9 px of it read LDS)
    const int cx0 = (int)floorf(cTx) - 15, cy0 = (int)floorf(cTy) - 15;
    const uint8_t* cache = nullptr;
    if (cx0 >= 0 && cy0 >= 0 && cx0 + kSubC <= s.W && cy0 + kSubC <= s.H && (cTx == cTx) && (cTy == cTy)) {
        uint8_t* c = s_cache[wv];
#pragma unroll
        for (int q = 0; q < kSubC * kSubC / 64 / 4; q++) {   // 4 bytes per lane per step
            const int i = (q * 64 + lane) * 4, yy = i / kSubC, xx = i - yy * kSubC;
            const uint8_t* src = s.img + (long long)(cy0 + yy) * s.pitch + cx0 + xx;
            c[i] = src[0];
            c[i + 1] = src[1];
            c[i + 2] = src[2];
            c[i + 3] = src[3];
        }
        cache = c;
        wave_lds_sync();
    }
    float cIx = cTx, cIy = cTy;
    int iter = 0;
    double err = 0;
    do {
        const float centx = cIx - (kSubP - 1) * 0.5f, centy = cIy - (kSubP - 1) * 0.5f;
        const int ipx = (int)floorf(centx), ipy = (int)floorf(centy);
        const bool inside = 0 <= ipx && ipx + kSubP < s.W && 0 <= ipy && ipy + kSubP < s.H;
        float fa = centx - ipx, fb = centy - ipy;
        double sd = 0;
        if (inside) {
            fa = fmaxf(fa, 0.0001f);
            sd = (1. - fa) / fa;
        }
        if (lane < kSubP) {
            float row[kSubP];
            subpix_row(s, inside, ipx, ipy, fa, fb, sd, lane, row, cache, cx0, cy0);
#pragma unroll
            for (int j = 0; j < kSubP; j++) patch[lane * kSubP + j] = row[j];
        }
        wave_lds_sync();
        for (int e = lane; e < kSubE; e += 64) {
            const int i = e / kSubW, j = e - i * kSubW;
            const float* sp = patch + (i + 1) * kSubP + (j + 1);
            const double m = wmask[e];
            const double tgx = sp[1] - sp[-1];
            const double tgy = sp[kSubP] - sp[-kSubP];
            const double gxx = tgx * tgx * m, gxy = tgx * tgy * m, gyy = tgy * tgy * m;
            const double px = j - kSubWin, py = i - kSubWin;
            terms[e] = gxx;
            terms[kSubE + e] = gxy;
            terms[2 * kSubE + e] = gyy;
            terms[3 * kSubE + e] = gxx * px + gxy * py;
            terms[4 * kSubE + e] = gxy * px + gyy * py;
        }
        wave_lds_sync();
        double acc = 0;
        if (lane < 5) {   // in order; row g+1's loads are in flight while row g is added
            const double* t = terms + lane * kSubE;
            double v[kSubW], w[kSubW];
#pragma unroll
            for (int j = 0; j < kSubW; j++) v[j] = t[j];
#pragma unroll
            for (int g = 0; g < kSubW; g++) {
                if (g + 1 < kSubW) {
#pragma unroll
                    for (int j = 0; j < kSubW; j++) w[j] = t[(g + 1) * kSubW + j];
                }
#pragma unroll
                for (int j = 0; j < kSubW; j++) acc += v[j];
#pragma unroll
                for (int j = 0; j < kSubW; j++) v[j] = w[j];
            }
        }
        const double a = __shfl(acc, 0), b = __shfl(acc, 1), c = __shfl(acc, 2), bb1 = __shfl(acc, 3),
                     bb2 = __shfl(acc, 4);
        wave_lds_sync();   // this iteration's LDS reads precede the next iteration's patch stores
        const double det = a * c - b * b;
        if (fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
        const double sc = 1.0 / det;
        const float nx = (float)(cIx + c * sc * bb1 - b * sc * bb2);
        const float ny = (float)(cIy - b * sc * bb1 + a * sc * bb2);
        err = (nx - cIx) * (nx - cIx) + (ny - cIy) * (ny - cIy);
        cIx = nx;
        cIy = ny;
        if (cIx < 0 || cIx >= s.W || cIy < 0 || cIy >= s.H) break;
    } while (++iter < max_iters && err > eps2);
    if (fabsf(cIx - cTx) > kSubWin || fabsf(cIy - cTy) > kSubWin) {
        cIx = cTx;
        cIy = cTy;
    }
    if (lane == 0) {
        pt[0] = cIx;
        pt[1] = cIy;
        if (keep) {   // ORB::compute -> runByImageBorder(image.size(), edgeThreshold): Rect::contains(cvRound(pt))
            const int px = (int)rintf(cIx), py = (int)rintf(cIy);
            keep[k] = s.W > 2 * edge && s.H > 2 * edge && edge <= px && px < s.W - edge && edge <= py &&
                      py < s.H - edge;
        }
    }
}

/* ---------------- computeOrbDescriptors (WTA_K 2) on the blurred pyramid ----------------------------
 * One wave per keypoint, 4 ballots of 64 pair tests = 32 bytes.  Samples outside the level ROI read the
 * unblurred REFLECT_101 frame the reference's pyramid buffer holds around each (blurred) ROI. */
__global__ __launch_bounds__(256) void k_bird_desc(const BirdGeom* __restrict__ g, const uint8_t* __restrict__ pyr,
                                                   const uint8_t* __restrict__ blur, const int* __restrict__ pattern,
                                                   const orb_keypoint* __restrict__ kps, const int* __restrict__ keep,
                                                   int n, uint8_t* __restrict__ desc) {
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (k >= n) return;
    const orb_keypoint kp = kps[k];
    unsigned long long* out = reinterpret_cast<unsigned long long*>(desc + (long long)k * 32);
    if (keep && !keep[k]) {
        if (lane < 4) out[lane] = 0;
        return;
    }
    const BirdLevel L = g->L[kp.octave];
    const float scale = 1.f / L.scale;
    const int cy = (int)rintf(kp.y * scale), cx = (int)rintf(kp.x * scale);
    const float angle = kp.angle * kFactorPI;
    float a, b;
    glibc_sincosf(angle, &b, &a);   // cv::ORB's (float)cos / (float)sin of a float: glibc cosf / sinf
#pragma unroll
    for (int rnd = 0; rnd < 4; rnd++) {
        const int p = rnd * 64 + lane;   // pair p: points 2p, 2p+1 -> byte p/8, bit p%8
        int val[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int px = pattern[4 * p + 2 * q], py = pattern[4 * p + 2 * q + 1];
            const float x = px * a - py * b, y = px * b + py * a;
            const int sx = cx + (int)rintf(x), sy = cy + (int)rintf(y);
            if ((unsigned)sx < (unsigned)L.w && (unsigned)sy < (unsigned)L.h)
                val[q] = blur[L.off + (long long)sy * L.pitch + sx];
            else
                val[q] = pyr[L.off + (long long)reflect101_d(sy, L.h) * L.pitch + reflect101_d(sx, L.w)];
        }
        const unsigned long long m = __ballot(val[0] < val[1]);
        if (lane == 0) out[rnd] = m;
    }
}

#include "pattern31_data.inc"
const int kPattern31[1024] = {ORBGPU_PATTERN31_VALUES};

inline int cv_round(float v) { return (int)std::nearbyint(v); }
inline int cv_round(double v) { return (int)std::nearbyint(v); }

struct HostKP {   // cv::KeyPoint + the candidate it came from (payload only: the comparisons read response)
    float x, y, size, angle, response;
    int octave, class_id;
    int cand;
};

struct SelKey {   // (KeyPoint::response, candidate index)
    float response;
    int cand;
};

// KeyPointsFilter::retainBest (keypoint.cpp): nth_element + partition of the boundary ties
void retain_best(std::vector<SelKey>& kps, int n_points) {
    if (n_points >= 0 && kps.size() > (size_t)n_points) {
        if (n_points == 0) {
            kps.clear();
            return;
        }
        std::nth_element(kps.begin(), kps.begin() + n_points, kps.end(),
                         [](const SelKey& a, const SelKey& b) { return a.response > b.response; });
        const float amb = kps[n_points - 1].response;
        auto e = std::partition(kps.begin() + n_points, kps.end(),
                                [amb](const SelKey& k) { return k.response >= amb; });
        kps.resize(e - kps.begin());
    }
}

}  // namespace

struct Bird {
    int device = 0;
    hipStream_t stream = nullptr;
    int nfeatures = 2000, nlevels = 8, edge = 31, fastTh = 20, variant = 0;
    double scaleFactor = 1.2f;
    float wmask[kSubW * kSubW]{};

    bool have_geom = false;
    BirdGeom g{};
    long long pyr_bytes = 0;
    std::vector<int2> frows, crows, brows;   // FAST score rows, candidate rows, blur rows
    std::vector<int> lvl_row0;               // candidate-row range per level (nlevels + 1)
    std::vector<int> brow0;                  // blur-row range per level
    std::vector<int> rcoef_off;
    int max_w = 0;

    // device
    BirdGeom* d_geom = nullptr;
    int2* d_rows = nullptr;         // frows | crows | brows
    int* d_lvlrow0 = nullptr;
    ResizeCoef* d_rcoef = nullptr;
    int* d_pattern = nullptr;
    float* d_wmask = nullptr;
    uint8_t *d_pyr = nullptr, *d_mpyr = nullptr, *d_score = nullptr, *d_blur = nullptr;
    int *d_rowcnt = nullptr, *d_rowoff = nullptr, *d_lvlcnt = nullptr;
    BirdCand* d_cand = nullptr;
    size_t cand_cap = 0;
    size_t cand_guess = 16384;      // candidates downloaded with the counts (next frame: this one's + 1/8)
    orb_keypoint* d_kps = nullptr;
    int* d_keep = nullptr;
    uint8_t* d_desc = nullptr;
    size_t kp_cap = 0;
    float* d_pts = nullptr;
    size_t pts_cap = 0;
    void* h_pin = nullptr;
    size_t pin_cap = 0;

    // last detect (debug view): candidates per level
    std::vector<BirdCand> last_cands;
    std::vector<int> last_lvlcnt;

    ~Bird();
    void free_geom();
    int ensure_geometry(int W, int H, int nl);
    int ensure_kp(size_t n);
    int ensure_pin(size_t bytes);
    int upload(const uint8_t* img, size_t stride, const uint8_t* mask, size_t mstride, bool footprint, bool device_src);
    int build_pyramid(int nl, bool with_mask);
    int detect_select(bool with_mask, std::vector<HostKP>& sel, int blur_levels);
    int launch_angle(int n);
    int launch_subpix(int n, bool keep);
    int launch_blur(int nl);
    int launch_desc(int n, bool keep);
};

void Bird::free_geom() {
    for (void* p : {(void*)d_geom, (void*)d_rows, (void*)d_lvlrow0, (void*)d_rcoef, (void*)d_pyr, (void*)d_mpyr,
                    (void*)d_score, (void*)d_blur, (void*)d_rowcnt, (void*)d_rowoff, (void*)d_lvlcnt})
        if (p) (void)hipFree(p);
    d_geom = nullptr;
    d_rows = nullptr;
    d_lvlrow0 = nullptr;
    d_rcoef = nullptr;
    d_pyr = d_mpyr = d_score = d_blur = nullptr;
    d_rowcnt = d_rowoff = d_lvlcnt = nullptr;
    have_geom = false;
}

Bird::~Bird() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    free_geom();
    for (void* p : {(void*)d_pattern, (void*)d_wmask, (void*)d_cand, (void*)d_kps, (void*)d_keep, (void*)d_desc,
                    (void*)d_pts})
        if (p) (void)hipFree(p);
    if (h_pin) (void)hipHostFree(h_pin);
    if (stream) (void)hipStreamDestroy(stream);
}

// orb.cpp detectAndCompute: level sizes cvRound(cols / getScale(level)); nfeaturesPerLevel
int Bird::ensure_geometry(int W, int H, int nl) {
    if (have_geom && g.W == W && g.H == H && g.nlevels == nl) return ORB_OK;
    hipError_t e;
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return set_error("sync", e), ORB_ERR_HIP;
    free_geom();
    BirdGeom G{};
    G.nlevels = nl;
    G.W = W;
    G.H = H;
    G.edge = edge;
    G.fastTh = std::min(std::max(fastTh, 0), 255);
    G.variant = variant;
    const float sc = 1.f / ((1 << 2) * 7 * 255.f);
    G.harris_scale4 = sc * sc * sc * sc;
    {   // getGaussianKernel(7, 2, CV_32F) -> 8-bit fixed point
        float cf[7];
        double s = 0;
        for (int i = 0; i < 7; i++) {
            const double x = i - 3.0;
            cf[i] = (float)std::exp(-0.5 / (2.0 * 2.0) * x * x);
            s += cf[i];
        }
        s = 1. / s;
        for (int i = 0; i < 7; i++) G.gk[i] = cv_round((float)(cf[i] * s) * 256.f);
    }
    {   // u_max (halfPatchSize 15)
        const int hp = 15;
        int umax[17];
        int v, v0, vmax = (int)std::floor(hp * std::sqrt(2.f) / 2 + 1), vmin = (int)std::ceil(hp * std::sqrt(2.f) / 2);
        for (v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt((double)hp * hp - v * v));
        for (v = hp, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
        for (int i = 0; i < 16; i++) G.umax[i] = umax[i];
    }
    {   // nfeaturesPerLevel
        const float factor = (float)(1.0 / scaleFactor);
        float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; l++) {
            G.L[l].nfeat = cv_round(nd);
            sum += G.L[l].nfeat;
            nd *= factor;
        }
        G.L[nl - 1].nfeat = std::max(nfeatures - sum, 0);
    }
    long long off = 0;
    frows.clear();
    crows.clear();
    brows.clear();
    lvl_row0.assign(nl + 1, 0);
    brow0.assign(nl + 1, 0);
    std::vector<ResizeCoef> coefs;
    rcoef_off.assign(nl, 0);
    max_w = 0;
    for (int l = 0; l < nl; l++) {
        BirdLevel& L = G.L[l];
        L.scale = (float)std::pow(scaleFactor, (double)l);
        L.w = cv_round((float)W / L.scale);
        L.h = cv_round((float)H / L.scale);
        if (L.w < 1 || L.h < 1) return set_error("birdview image too small for the pyramid", hipSuccess), ORB_ERR_GEOMETRY;
        L.pitch = (L.w + 63) & ~63;
        L.off = off;
        off += (long long)L.pitch * L.h + 256;
        max_w = std::max(max_w, L.w);
        lvl_row0[l] = (int)crows.size();
        brow0[l] = (int)brows.size();
        // runByImageBorder clears a level with h <= 2e or w <= 2e; FAST needs the 3-pixel ring
        if (L.w > 2 * edge && L.h > 2 * edge && edge >= 4) {
            for (int y = edge - 1; y <= L.h - edge; y++) frows.push_back(make_int2(l, y));
            for (int y = edge; y < L.h - edge; y++) crows.push_back(make_int2(l, y));
        }
        for (int y = 0; y < L.h; y++) brows.push_back(make_int2(l, y));
        if (l > 0) {
            rcoef_off[l] = (int)coefs.size();
            resize_coefs(G.L[l - 1].w, L.w, coefs, false);
            resize_coefs(G.L[l - 1].h, L.h, coefs, true);
        }
    }
    if (edge < 4) return set_error("edgeThreshold < 4 is not supported", hipSuccess), ORB_ERR_ARG;
    lvl_row0[nl] = (int)crows.size();
    brow0[nl] = (int)brows.size();
    pyr_bytes = off;
    g = G;
    std::vector<int2> rows(frows);
    rows.insert(rows.end(), crows.begin(), crows.end());
    rows.insert(rows.end(), brows.begin(), brows.end());
    const size_t nr = crows.size();
    size_t ccap = 0;   // NMS survivors never touch: <= ceil(w/2) * ceil(h/2) per level
    for (int l = 0; l < nl; l++) ccap += (size_t)((G.L[l].w + 1) / 2) * ((G.L[l].h + 1) / 2);
    if ((e = hipMalloc((void**)&d_geom, sizeof(BirdGeom))) != hipSuccess ||
        (e = hipMalloc((void**)&d_rows, std::max<size_t>(rows.size(), 1) * sizeof(int2))) != hipSuccess ||
        (e = hipMalloc((void**)&d_lvlrow0, (nl + 1) * sizeof(int))) != hipSuccess ||
        (e = hipMalloc((void**)&d_rcoef, std::max<size_t>(coefs.size(), 1) * sizeof(ResizeCoef))) != hipSuccess ||
        (e = hipMalloc((void**)&d_pyr, pyr_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&d_mpyr, pyr_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&d_score, pyr_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&d_blur, pyr_bytes)) != hipSuccess ||
        (e = hipMalloc((void**)&d_rowcnt, (nr + 1) * sizeof(int))) != hipSuccess ||
        (e = hipMalloc((void**)&d_rowoff, (nr + 1) * sizeof(int))) != hipSuccess ||
        (e = hipMalloc((void**)&d_lvlcnt, kBirdMaxLevels * sizeof(int))) != hipSuccess)
        return free_geom(), set_error("birdview buffers", e), ORB_ERR_NOMEM;
    if (ccap > cand_cap) {
        if (d_cand) (void)hipFree(d_cand);
        d_cand = nullptr;
        cand_cap = 0;
        if ((e = hipMalloc((void**)&d_cand, ccap * sizeof(BirdCand))) != hipSuccess)
            return free_geom(), set_error("birdview candidates", e), ORB_ERR_NOMEM;
        cand_cap = ccap;
    }
    if ((e = hipMemcpyAsync(d_geom, &g, sizeof(BirdGeom), hipMemcpyHostToDevice, stream)) != hipSuccess ||
        (!rows.empty() &&
         (e = hipMemcpyAsync(d_rows, rows.data(), rows.size() * sizeof(int2), hipMemcpyHostToDevice, stream)) !=
             hipSuccess) ||
        (e = hipMemcpyAsync(d_lvlrow0, lvl_row0.data(), (nl + 1) * sizeof(int), hipMemcpyHostToDevice, stream)) !=
            hipSuccess ||
        (!coefs.empty() && (e = hipMemcpyAsync(d_rcoef, coefs.data(), coefs.size() * sizeof(ResizeCoef),
                                               hipMemcpyHostToDevice, stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
        return free_geom(), set_error("birdview geometry upload", e), ORB_ERR_HIP;
    have_geom = true;
    return ORB_OK;
}

int Bird::ensure_kp(size_t n) {
    if (n <= kp_cap && d_kps) return ORB_OK;
    size_t cap = std::max<size_t>(n, 4096);
    for (void* p : {(void*)d_kps, (void*)d_keep, (void*)d_desc})
        if (p) (void)hipFree(p);
    d_kps = nullptr;
    d_keep = nullptr;
    d_desc = nullptr;
    kp_cap = 0;
    hipError_t e;
    if ((e = hipMalloc((void**)&d_kps, cap * sizeof(orb_keypoint))) != hipSuccess ||
        (e = hipMalloc((void**)&d_keep, cap * sizeof(int))) != hipSuccess ||
        (e = hipMalloc((void**)&d_desc, cap * 32)) != hipSuccess)
        return set_error("birdview keypoint buffers", e), ORB_ERR_NOMEM;
    kp_cap = cap;
    return ORB_OK;
}

int Bird::ensure_pin(size_t bytes) {
    if (bytes <= pin_cap && h_pin) return ORB_OK;
    if (h_pin) (void)hipHostFree(h_pin);
    h_pin = nullptr;
    pin_cap = 0;
    size_t cap = std::max<size_t>(bytes, 1 << 20);
    hipError_t e = hipHostMalloc(&h_pin, cap);
    if (e != hipSuccess) return set_error("pinned staging", e), ORB_ERR_NOMEM;
    pin_cap = cap;
    return ORB_OK;
}

// Frame.cc:320-327 footprint rectangle (doubles truncated into cv::Rect, filled, clipped)
static void footprint_rect(int W, int H, int& x0, int& y0, int& x1, int& y1) {
    const double p2m = 0.03984 * 1.7, len = 4.63, wid = 1.901, boundary = 15.0;
    const double x = W / 2 - (wid / 2 / p2m) - boundary, y = H / 2 - (len / 2 / p2m) - boundary;
    const double width = wid / p2m + 2 * boundary, height = len / p2m + 2 * boundary;
    const int rx = (int)x, ry = (int)y, rw = (int)width, rh = (int)height;
    if (rw <= 0 || rh <= 0) {
        x0 = y0 = x1 = y1 = 0;
        return;
    }
    x0 = std::max(rx, 0);
    y0 = std::max(ry, 0);
    x1 = std::min(rx + rw, W);
    y1 = std::min(ry + rh, H);
}

int Bird::upload(const uint8_t* img, size_t stride, const uint8_t* mask, size_t mstride, bool footprint,
                 bool device_src) {
    const hipMemcpyKind kind = device_src ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const BirdLevel& L0 = g.L[0];
    hipError_t e;
    if ((e = hipMemcpy2DAsync(d_pyr + L0.off, L0.pitch, img, stride, L0.w, L0.h, kind, stream)) != hipSuccess)
        return set_error("birdview image upload", e), ORB_ERR_HIP;
    if (mask) {
        if ((e = hipMemcpy2DAsync(d_mpyr + L0.off, L0.pitch, mask, mstride, L0.w, L0.h, kind, stream)) != hipSuccess)
            return set_error("birdview mask upload", e), ORB_ERR_HIP;
        if (footprint) {
            int x0, y0, x1, y1;
            footprint_rect(L0.w, L0.h, x0, y0, x1, y1);
            if (x1 > x0 && y1 > y0 &&
                (e = hipMemset2DAsync(d_mpyr + L0.off + (long long)y0 * L0.pitch + x0, L0.pitch, 0, x1 - x0, y1 - y0,
                                      stream)) != hipSuccess)
                return set_error("footprint", e), ORB_ERR_HIP;
        }
    }
    return ORB_OK;
}

int Bird::build_pyramid(int nl, bool with_mask) {
    for (int l = 1; l < nl; l++) {
        dim3 grid((g.L[l].w + 255) / 256, g.L[l].h, with_mask ? 2 : 1);
        hipLaunchKernelGGL(k_bird_resize, grid, dim3(256), 0, stream, d_geom, l, d_rcoef + rcoef_off[l], d_pyr, d_mpyr);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error("k_bird_resize", e), ORB_ERR_HIP;
    return ORB_OK;
}

// computeKeyPoints up to the final per-level selection; sel receives the kept keypoints (level coords,
// octave, size, Harris response) in the reference's order.
int Bird::detect_select(bool with_mask, std::vector<HostKP>& sel, int blur_levels) {
    sel.clear();
    const int nl = g.nlevels;
    const int nf = (int)frows.size(), nc = (int)crows.size();
    hipError_t e;
    last_lvlcnt.assign(nl, 0);
    last_cands.clear();
    if (nc > 0) {
        const int2* d_frows = d_rows;
        const int2* d_crows = d_rows + nf;
        const int fx = (max_w - 2 * edge + 2 + 255) / 256;
        hipLaunchKernelGGL(k_bird_fast, dim3(std::max(fx, 1), nf), dim3(256), 0, stream, d_geom, d_frows, d_pyr,
                           d_score);
        const uint8_t* mp = with_mask ? d_mpyr : nullptr;
        hipLaunchKernelGGL(k_bird_cands<0>, dim3((nc + 3) / 4), dim3(256), 0, stream, d_geom, d_crows, nc, d_pyr, mp,
                           d_score, d_rowcnt, (const int*)nullptr, (BirdCand*)nullptr);
        hipLaunchKernelGGL(k_bird_scan, dim3(1), dim3(1024), 0, stream, d_rowcnt, nc, d_lvlrow0, nl, d_rowoff,
                           d_lvlcnt);
        hipLaunchKernelGGL(k_bird_cands<1>, dim3((nc + 3) / 4), dim3(256), 0, stream, d_geom, d_crows, nc, d_pyr, mp,
                           d_score, (int*)nullptr, d_rowoff, d_cand);
        if ((e = hipGetLastError()) != hipSuccess) return set_error("birdview FAST", e), ORB_ERR_HIP;
        int r;
        // the blurred pyramid only needs the pyramid: it runs while the host selects
        if (blur_levels > 0 && (r = launch_blur(blur_levels)) != ORB_OK) return r;
        // one download of the level counts and a speculative prefix of the candidates (sized from the
        // previous frame); a second only if this frame has more
        const size_t hdr = 64, guess = std::min(cand_guess, cand_cap);
        if ((r = ensure_pin(hdr + guess * sizeof(BirdCand))) != ORB_OK) return r;
        uint8_t* hp = (uint8_t*)h_pin;
        if ((e = hipMemcpyAsync(hp, d_lvlcnt, nl * sizeof(int), hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (guess && (e = hipMemcpyAsync(hp + hdr, d_cand, guess * sizeof(BirdCand), hipMemcpyDeviceToHost, stream)) !=
                          hipSuccess) ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)
            return set_error("birdview candidate download", e), ORB_ERR_HIP;
        std::memcpy(last_lvlcnt.data(), hp, nl * sizeof(int));
        size_t total = 0;
        for (int l = 0; l < nl; l++) total += last_lvlcnt[l];
        if (total > cand_cap) return set_error("birdview candidate overflow", hipSuccess), ORB_ERR_INTERNAL;
        last_cands.resize(total);
        std::memcpy(last_cands.data(), hp + hdr, std::min(total, guess) * sizeof(BirdCand));
        if (total > guess) {
            const size_t rest = total - guess;
            if ((r = ensure_pin(rest * sizeof(BirdCand))) != ORB_OK) return r;
            if ((e = hipMemcpyAsync(h_pin, d_cand + guess, rest * sizeof(BirdCand), hipMemcpyDeviceToHost, stream)) !=
                    hipSuccess ||
                (e = hipStreamSynchronize(stream)) != hipSuccess)
                return set_error("birdview candidates download", e), ORB_ERR_HIP;
            std::memcpy(last_cands.data() + guess, h_pin, rest * sizeof(BirdCand));
        }
        cand_guess = total + total / 8 + 256;
    } else if (blur_levels > 0) {
        int r;
        if ((r = launch_blur(blur_levels)) != ORB_OK) return r;
    }
    // KeyPointsFilter::retainBest(2 N) on the FAST response, per level; then Harris, retainBest(N).
    // nth_element / partition see only the responses, so they run on 8-byte (response, candidate)
    // keys: the resulting arrangement is the one a vector<cv::KeyPoint> gets.
    std::vector<std::vector<SelKey>> lv(nl);
    size_t off = 0;
    for (int l = 0; l < nl; l++) {
        auto& k = lv[l];
        k.resize(last_lvlcnt[l]);
        for (int i = 0; i < last_lvlcnt[l]; i++) k[i] = {(float)last_cands[off + i].score, (int)(off + i)};
        off += last_lvlcnt[l];
        retain_best(k, 2 * g.L[l].nfeat);
    }
    size_t any = 0;
    for (int l = 0; l < nl; l++) any += lv[l].size();
    if (!any) return ORB_OK;
    for (int l = 0; l < nl; l++) {
        for (auto& kp : lv[l]) kp.response = last_cands[kp.cand].harris;
        retain_best(lv[l], g.L[l].nfeat);
        const float size = 31 * g.L[l].scale;
        for (const auto& kp : lv[l]) {
            const BirdCand& c = last_cands[kp.cand];
            sel.push_back({(float)(c.xy & 0xFFFF), (float)(c.xy >> 16), size, -1.f, kp.response, l, -1, kp.cand});
        }
    }
    return ORB_OK;
}

int Bird::launch_angle(int n) {
    if (n) hipLaunchKernelGGL(k_bird_angle, dim3((n + 3) / 4), dim3(256), 0, stream, d_geom, d_pyr, d_kps, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ORB_OK : (set_error("k_bird_angle", e), ORB_ERR_HIP);
}

int Bird::launch_subpix(int n, bool keep) {
    SubpixSrc s{d_pyr + g.L[0].off, g.L[0].pitch, g.L[0].w, g.L[0].h};
    if (n)
        hipLaunchKernelGGL(k_bird_subpix, dim3((n + 3) / 4), dim3(256), 0, stream, s, d_wmask,
                           reinterpret_cast<float*>(d_kps), 7, n, 40, 0.001 * 0.001, edge, keep ? d_keep : nullptr);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ORB_OK : (set_error("k_bird_subpix", e), ORB_ERR_HIP);
}

int Bird::launch_blur(int nl) {
    const int2* d_brows = d_rows + frows.size() + crows.size();
    const int nb = brow0[nl];
    if (nb) hipLaunchKernelGGL(k_bird_blur, dim3((max_w + 255) / 256, nb), dim3(256), 0, stream, d_geom, d_brows, d_pyr, d_blur);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ORB_OK : (set_error("k_bird_blur", e), ORB_ERR_HIP);
}

int Bird::launch_desc(int n, bool keep) {
    if (n)
        hipLaunchKernelGGL(k_bird_desc, dim3((n + 3) / 4), dim3(256), 0, stream, d_geom, d_pyr, d_blur, d_pattern, d_kps,
                           keep ? d_keep : nullptr, n, d_desc);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ORB_OK : (set_error("k_bird_desc", e), ORB_ERR_HIP);
}

}  // namespace orbgpu

using namespace orbgpu;

struct orb_bird : Bird {};

static int bird_enter(orb_bird* b) {
    if (!b) return set_error("NULL orb_bird", hipSuccess), ORB_ERR_ARG;
    hipError_t e = hipSetDevice(b->device);
    if (e != hipSuccess) return set_error("hipSetDevice", e), ORB_ERR_HIP;
    return ORB_OK;
}

extern "C" orb_bird* orb_bird_create(const orb_bird_params* p, int* status) {
    auto fail = [&](int st) -> orb_bird* {
        if (status) *status = st;
        return nullptr;
    };
    if (!p || p->nfeatures < 0 || p->nlevels < 1 || p->nlevels > ORBGPU_MAX_LEVELS || !(p->scaleFactor > 1.0f) ||
        p->edgeThreshold < 4 || p->fastThreshold < 0 ||
        (p->variant & ~(ORB_VARIANT_RESIZE_GENERIC | ORB_VARIANT_BLUR_HALFUP))) {
        set_error("invalid orb_bird_params", hipSuccess);
        return fail(ORB_ERR_ARG);
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || p->device < 0 || p->device >= ndev) {
        set_error("no HIP device (liborbgpu has no CPU fallback)", e);
        return fail(ORB_ERR_HIP);
    }
    if ((e = hipSetDevice(p->device)) != hipSuccess) return set_error("hipSetDevice", e), fail(ORB_ERR_HIP);
    orb_bird* b = new (std::nothrow) orb_bird();
    if (!b) return fail(ORB_ERR_NOMEM);
    b->device = p->device;
    b->nfeatures = p->nfeatures;
    b->scaleFactor = p->scaleFactor;
    b->nlevels = p->nlevels;
    b->edge = p->edgeThreshold;
    b->fastTh = p->fastThreshold;
    b->variant = p->variant;
    // cornerSubPix weight mask: exp(-y^2) * exp(-x^2) in float (glibc expf, as the reference's host)
    for (int i = 0; i < kSubW; i++) {
        const float y = (float)(i - kSubWin) / kSubWin;
        const float vy = std::exp(-y * y);
        for (int j = 0; j < kSubW; j++) {
            const float x = (float)(j - kSubWin) / kSubWin;
            b->wmask[i * kSubW + j] = (float)(vy * std::exp(-x * x));
        }
    }
    if ((e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc((void**)&b->d_pattern, sizeof(kPattern31))) != hipSuccess ||
        (e = hipMalloc((void**)&b->d_wmask, sizeof(b->wmask))) != hipSuccess ||
        (e = hipMemcpyAsync(b->d_pattern, kPattern31, sizeof(kPattern31), hipMemcpyHostToDevice, b->stream)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(b->d_wmask, b->wmask, sizeof(b->wmask), hipMemcpyHostToDevice, b->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(b->stream)) != hipSuccess) {
        delete b;
        set_error("orb_bird_create", e);
        return fail(ORB_ERR_HIP);
    }
    if (status) *status = ORB_OK;
    return b;
}

extern "C" void orb_bird_destroy(orb_bird* b) {
    if (b) delete b;
}

extern "C" int orb_bird_footprint_mask(uint8_t* mask, int w, int h, size_t stride) {
    if (!mask || w < 0 || h < 0 || stride < (size_t)w) return set_error("orb_bird_footprint_mask: bad arguments", hipSuccess), ORB_ERR_ARG;
    int x0, y0, x1, y1;
    footprint_rect(w, h, x0, y0, x1, y1);
    for (int y = y0; y < y1; y++) std::memset(mask + (size_t)y * stride + x0, 0, x1 - x0);
    return ORB_OK;
}

static void to_kp(const HostKP& h, orb_keypoint& k) {
    k.x = h.x;
    k.y = h.y;
    k.size = h.size;
    k.angle = h.angle;
    k.response = h.response;
    k.octave = h.octave;
    k.class_id = h.class_id;
}

// detect (+ optional cornerSubPix and compute) on an image already in the level-0 slot
static int bird_run(orb_bird* b, bool with_mask, bool subpix_compute, orb_keypoint* kps, int cap, int* n,
                    uint8_t* desc) {
    int r;
    std::vector<HostKP> sel;
    if ((r = b->build_pyramid(b->g.nlevels, with_mask)) != ORB_OK) return r;
    // the fused call blurs every level while the host selects (compute() would blur max octave + 1 of
    // them; the extra levels are never read)
    if ((r = b->detect_select(with_mask, sel, subpix_compute ? b->g.nlevels : 0)) != ORB_OK) return r;
    const int ns = (int)sel.size();
    if (!subpix_compute && ns > cap) {
        *n = ns;
        return set_error("orb_bird_detect: capacity", hipSuccess), ORB_ERR_CAPACITY;
    }
    if ((r = b->ensure_kp(std::max(ns, 1))) != ORB_OK) return r;
    std::vector<orb_keypoint> hk(ns);
    for (int i = 0; i < ns; i++) to_kp(sel[i], hk[i]);
    hipError_t e;
    if (ns && (e = hipMemcpyAsync(b->d_kps, hk.data(), ns * sizeof(orb_keypoint), hipMemcpyHostToDevice, b->stream)) !=
                  hipSuccess)
        return set_error("birdview keypoint upload", e), ORB_ERR_HIP;
    if ((r = b->launch_angle(ns)) != ORB_OK) return r;
    if (!subpix_compute) {
        if (ns && ((e = hipMemcpyAsync(kps, b->d_kps, ns * sizeof(orb_keypoint), hipMemcpyDeviceToHost, b->stream)) !=
                       hipSuccess ||
                   (e = hipStreamSynchronize(b->stream)) != hipSuccess))
            return set_error("birdview keypoint download", e), ORB_ERR_HIP;
        *n = ns;
        return ORB_OK;
    }
    // cornerSubPix on the level-0 image, border flag, descriptors on the blurred pyramid
    if ((r = b->launch_subpix(ns, true)) != ORB_OK) return r;
    if ((r = b->launch_desc(ns, true)) != ORB_OK) return r;
    const size_t kb = (size_t)ns * sizeof(orb_keypoint), fb = (size_t)ns * sizeof(int), db = (size_t)ns * 32;
    if ((r = b->ensure_pin(kb + fb + db + 64)) != ORB_OK) return r;
    uint8_t* hp = (uint8_t*)b->h_pin;
    if (ns && ((e = hipMemcpyAsync(hp, b->d_kps, kb, hipMemcpyDeviceToHost, b->stream)) != hipSuccess ||
               (e = hipMemcpyAsync(hp + kb, b->d_keep, fb, hipMemcpyDeviceToHost, b->stream)) != hipSuccess ||
               (e = hipMemcpyAsync(hp + kb + fb, b->d_desc, db, hipMemcpyDeviceToHost, b->stream)) != hipSuccess))
        return set_error("birdview result download", e), ORB_ERR_HIP;
    if ((e = hipStreamSynchronize(b->stream)) != hipSuccess) return set_error("birdview sync", e), ORB_ERR_HIP;
    const orb_keypoint* rk = (const orb_keypoint*)hp;
    const int* keep = (const int*)(hp + kb);
    const uint8_t* rd = hp + kb + fb;
    int m = 0;
    for (int i = 0; i < ns; i++) m += keep[i] != 0;
    *n = m;
    if (m > cap) return set_error("orb_bird_extract: capacity", hipSuccess), ORB_ERR_CAPACITY;
    for (int i = 0, j = 0; i < ns; i++)
        if (keep[i]) {
            kps[j] = rk[i];
            if (desc) std::memcpy(desc + (size_t)j * 32, rd + (size_t)i * 32, 32);
            j++;
        }
    return ORB_OK;
}

extern "C" int orb_bird_detect(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, const uint8_t* mask,
                               size_t mask_stride, orb_keypoint* kps, int cap, int* n) {
    int r;
    if ((r = bird_enter(b)) != ORB_OK) return r;
    if (!n || cap < 0 || (cap && !kps)) return set_error("orb_bird_detect: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (!img || w <= 0 || h <= 0) {   // Feature2D::detect: empty image -> keypoints.clear()
        *n = 0;
        return ORB_OK;
    }
    if (stride < (size_t)w || (mask && mask_stride < (size_t)w)) return ORB_ERR_ARG;
    if ((r = b->ensure_geometry(w, h, b->nlevels)) != ORB_OK) return r;
    if ((r = b->upload(img, stride, mask, mask_stride, false, false)) != ORB_OK) return r;
    return bird_run(b, mask != nullptr, false, kps, cap, n, nullptr);
}

static int bird_extract(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, const uint8_t* mask,
                        size_t mask_stride, orb_keypoint* kps, int cap, int* n, uint8_t* desc, bool device_src) {
    int r;
    if ((r = bird_enter(b)) != ORB_OK) return r;
    if (!n || cap < 0 || (cap && (!kps || !desc))) return set_error("orb_bird_extract: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (!img || w <= 0 || h <= 0) {
        *n = 0;
        return ORB_OK;
    }
    if (stride < (size_t)w || (mask && mask_stride < (size_t)w)) return ORB_ERR_ARG;
    if ((r = b->ensure_geometry(w, h, b->nlevels)) != ORB_OK) return r;
    if ((r = b->upload(img, stride, mask, mask_stride, true, device_src)) != ORB_OK) return r;
    return bird_run(b, mask != nullptr, true, kps, cap, n, desc);
}

extern "C" int orb_bird_extract(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, const uint8_t* mask,
                                size_t mask_stride, orb_keypoint* kps, int cap, int* n, uint8_t* desc) {
    return bird_extract(b, img, w, h, stride, mask, mask_stride, kps, cap, n, desc, false);
}

extern "C" int orb_bird_extract_device(orb_bird* b, const uint8_t* d_img, int w, int h, size_t stride,
                                       const uint8_t* d_mask, size_t mask_stride, orb_keypoint* kps, int cap, int* n,
                                       uint8_t* desc) {
    return bird_extract(b, d_img, w, h, stride, d_mask, mask_stride, kps, cap, n, desc, true);
}

extern "C" int orb_bird_compute(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, orb_keypoint* kps,
                                int* n, uint8_t* desc) {
    int r;
    if ((r = bird_enter(b)) != ORB_OK) return r;
    if (!n || *n < 0 || (*n && !kps)) return set_error("orb_bird_compute: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (!img || w <= 0 || h <= 0) return ORB_OK;   // Feature2D::compute: empty image -> descriptors released
    if (stride < (size_t)w) return ORB_ERR_ARG;
    // detectAndCompute(useProvidedKeypoints): nLevels = max octave + 1; border cull; level sort
    const int n0 = *n;
    int nl = 0;
    bool sorted = true;
    for (int i = 0; i < n0; i++) {
        if (kps[i].octave < 0 || kps[i].octave >= ORBGPU_MAX_LEVELS)
            return set_error("orb_bird_compute: octave out of range", hipSuccess), ORB_ERR_ARG;
        if (i > 0 && kps[i].octave < kps[i - 1].octave) sorted = false;
        nl = std::max(nl, kps[i].octave);
    }
    nl++;
    const int e = b->edge;
    std::vector<orb_keypoint> v;
    v.reserve(n0);
    if (!(h <= 2 * e || w <= 2 * e))
        for (int i = 0; i < n0; i++) {
            const int px = cv_round(kps[i].x), py = cv_round(kps[i].y);
            if (e <= px && px < w - e && e <= py && py < h - e) v.push_back(kps[i]);
        }
    if (!sorted) {
        std::vector<orb_keypoint> s;
        s.reserve(v.size());
        for (int l = 0; l < nl; l++)
            for (const auto& k : v)
                if (k.octave == l) s.push_back(k);
        v.swap(s);
    }
    const int m = (int)v.size();
    std::memcpy(kps, v.data(), m * sizeof(orb_keypoint));
    *n = m;
    if (!m) return ORB_OK;
    if (!desc) return set_error("orb_bird_compute: NULL desc", hipSuccess), ORB_ERR_ARG;
    if ((r = b->ensure_geometry(w, h, std::max(nl, b->nlevels))) != ORB_OK) return r;
    if ((r = b->ensure_kp(m)) != ORB_OK) return r;
    if ((r = b->upload(img, stride, nullptr, 0, false, false)) != ORB_OK) return r;
    if ((r = b->build_pyramid(nl, false)) != ORB_OK) return r;
    hipError_t he;
    if ((he = hipMemcpyAsync(b->d_kps, v.data(), m * sizeof(orb_keypoint), hipMemcpyHostToDevice, b->stream)) !=
        hipSuccess)
        return set_error("birdview keypoint upload", he), ORB_ERR_HIP;
    if ((r = b->launch_blur(nl)) != ORB_OK || (r = b->launch_desc(m, false)) != ORB_OK) return r;
    if ((he = hipMemcpyAsync(desc, b->d_desc, (size_t)m * 32, hipMemcpyDeviceToHost, b->stream)) != hipSuccess ||
        (he = hipStreamSynchronize(b->stream)) != hipSuccess)
        return set_error("birdview descriptor download", he), ORB_ERR_HIP;
    return ORB_OK;
}

extern "C" int orb_corner_subpix(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, float* pts, int n,
                                 int win_w, int win_h, int max_iter, double eps) {
    int r;
    if ((r = bird_enter(b)) != ORB_OK) return r;
    if (n < 0 || (n && !pts) || !img || w <= 0 || h <= 0 || stride < (size_t)w)
        return set_error("orb_corner_subpix: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (win_w != kSubWin || win_h != kSubWin)   // the kernel is built for the reference's Size(5,5)
        return set_error("orb_corner_subpix: only win (5,5) is built (Frame.cc:337)", hipSuccess), ORB_ERR_ARG;
    if (w < kSubWin * 2 + 5 || h < kSubWin * 2 + 5) return ORB_ERR_GEOMETRY;   // CV_Assert in cornerSubPix
    if (!n) return ORB_OK;
    if ((r = b->ensure_geometry(w, h, b->nlevels)) != ORB_OK && (r = b->ensure_geometry(w, h, 1)) != ORB_OK) return r;
    hipError_t e;
    if ((size_t)n * 2 > b->pts_cap) {
        if (b->d_pts) (void)hipFree(b->d_pts);
        b->d_pts = nullptr;
        b->pts_cap = 0;
        if ((e = hipMalloc((void**)&b->d_pts, (size_t)n * 2 * sizeof(float))) != hipSuccess)
            return set_error("subpix points", e), ORB_ERR_NOMEM;
        b->pts_cap = (size_t)n * 2;
    }
    if ((r = b->upload(img, stride, nullptr, 0, false, false)) != ORB_OK) return r;
    const int iters = std::min(std::max(max_iter, 1), 100);
    const double ep = std::max(eps, 0.);
    SubpixSrc s{b->d_pyr + b->g.L[0].off, b->g.L[0].pitch, w, h};
    if ((e = hipMemcpyAsync(b->d_pts, pts, (size_t)n * 8, hipMemcpyHostToDevice, b->stream)) != hipSuccess)
        return set_error("subpix upload", e), ORB_ERR_HIP;
    hipLaunchKernelGGL(k_bird_subpix, dim3((n + 3) / 4), dim3(256), 0, b->stream, s, b->d_wmask, b->d_pts, 2, n, iters,
                       ep * ep, b->edge, (int*)nullptr);
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpyAsync(pts, b->d_pts, (size_t)n * 8, hipMemcpyDeviceToHost, b->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(b->stream)) != hipSuccess)
        return set_error("k_bird_subpix", e), ORB_ERR_HIP;
    return ORB_OK;
}

extern "C" int orb_bird_debug_candidates(orb_bird* b, int level, orb_keypoint* out, int cap) {
    if (!b || level < 0 || level >= (int)b->last_lvlcnt.size()) return ORB_ERR_ARG;
    size_t off = 0;
    for (int l = 0; l < level; l++) off += b->last_lvlcnt[l];
    const int n = b->last_lvlcnt[level];
    if (n > cap) return -n - 1;
    for (int i = 0; i < n; i++) {
        const BirdCand& c = b->last_cands[off + i];
        out[i] = {(float)(c.xy & 0xFFFF), (float)(c.xy >> 16), 7.f, -1.f, c.harris, level, c.score};
    }
    return n;
}

extern "C" int orb_bird_debug_level(orb_bird* b, int level, uint8_t* out, int* w, int* h) {
    if (!b || level < 0 || !b->have_geom || level >= b->g.nlevels || !w || !h) return ORB_ERR_ARG;
    const BirdLevel& L = b->g.L[level];
    *w = L.w;
    *h = L.h;
    if (!out) return ORB_OK;
    (void)hipSetDevice(b->device);
    hipError_t e = hipMemcpy2DAsync(out, L.w, b->d_pyr + L.off, L.pitch, L.w, L.h, hipMemcpyDeviceToHost, b->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
    return e == hipSuccess ? ORB_OK : (set_error("orb_bird_debug_level", e), ORB_ERR_HIP);
}
