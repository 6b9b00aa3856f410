// gfx950 kernels of the ORB extractor: pyramid, per-cell FAST+NMS, DistributeOctTree, and the fused
// IC-angle + 7x7 Gaussian + rBRIEF descriptor.  Integer/byte work, bound by HBM bytes and VALU issue
// (DESIGN.md §4); the one matrix-core use here is k_describe's blur row pass, an exact int8 product of the
// keypoint window and the banded 7-tap matrix (v_mfma_i32_16x16x64_i8).  The all-pairs
// Hamming top-2 (hamming_kernels.hip) is the other MFMA user.
//
// Compiled with -ffp-contract=off and correctly-rounded fp32 divide, so every float expression on the
// path (root split hX, fastAtan2, BRIEF rotation, keypoint scaling) is evaluated exactly as written; the
// two the reference's -O3 -march=native build contracts into FMAs (the BRIEF sample offsets) are
// written as explicit fmaf, and cos/sin follow glibc.
#include "glibc_trig.h"
#include "orbgpu_internal.h"
#include "pattern31_data.inc"

#include <algorithm>
#include <cstring>

namespace orbgpu {

__constant__ __attribute__((aligned(16))) int8_t c_pattern[1024] = {ORBGPU_PATTERN31_VALUES};
// the same pattern as floats (k_describe's BRIEF offsets are float products): one 16-byte load per test
// pair and lane, no conversions
__constant__ __attribute__((aligned(16))) float c_pattern_f[1024] = {ORBGPU_PATTERN31_VALUES};

// IC_Angle byte masks per lane (see ic_masks): lane l sums dwords 4h .. 4h+3 (h = l & 1) of patch row
// v = min(l >> 1, 30) - 15, bytes with |u| <= umax[|v|] (ORBextractor.cc:454-469)
struct IcMaskTable {
    uint32_t m[64][4];
};
constexpr IcMaskTable make_ic_masks() {
    IcMaskTable t{};
    constexpr int umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
    for (int l = 0; l < 64; l++) {
        const int r = (l >> 1) < 30 ? (l >> 1) : 30, v = r - 15, h = l & 1;
        const int d = umax[v < 0 ? -v : v];
        for (int i = 0; i < 4; i++) {
            uint32_t m = 0;
            for (int j = 0; j < 4; j++) {
                const int u = 4 * (4 * h + i) + j;   // byte of the row slice; u = -15 is byte 0
                if (u >= 15 - d && u <= 15 + d) m |= 0xFFu << (8 * j);
            }
            t.m[l][i] = m;
        }
    }
    return t;
}
__constant__ __attribute__((aligned(16))) IcMaskTable c_ic_masks = make_ic_masks();

namespace {

struct LevelPtr {
    const uint8_t* p;
    int stride;
};

__device__ __forceinline__ LevelPtr level_ptr(const Geom* __restrict__ g, int l, const uint8_t* frames,
                                              long long framePitch, int rowStride, const uint8_t* pyr, int f) {
    if (l == 0) return {frames + (long long)f * framePitch, rowStride};
    return {pyr + (long long)f * g->pyr_bytes + g->L[l].pyr_off, g->L[l].pitch};
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lanes_below(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0));
}

}  // namespace

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

// (a * b) >> 32 for a, b < 2^24: v_mul_hi_u32_u24 (the compiler does not form it from 64-bit products)
__device__ __forceinline__ unsigned mul_hi_u24(unsigned a, unsigned b) {
    unsigned r;
    asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
typedef unsigned int uint32x4_t __attribute__((ext_vector_type(4)));

/* ------------------------------------------------------------------------------------------------
 * Pyramid: cv::resize(level l-1 -> level l, INTER_LINEAR) for every frame of the batch
 * (ComputePyramid, ORBextractor.cc:1118-1120).  OpenCV-3.x 8U fixed point: 11-bit horizontal
 * weights, vertical pass ((b0*(H0>>4))>>16 + (b1*(H1>>4))>>16 + 2)>>2.
 * Only the ROI values matter: the reference's REFLECT_101 padding is never read on the path.
 * --------------------------------------------------------------------------------------------- */
// GENERIC (ORB_VARIANT_RESIZE_GENERIC): the vertical pass as the generic FixedPtCast,
// sat_u8((b0*H0 + b1*H1 + 2^21) >> 22), instead of the 3.x `>>4` form
template <bool GENERIC>
__global__ __launch_bounds__(256) void k_resize(const Geom* __restrict__ g, const ResizeCoef* __restrict__ coef,
                                                int level, const uint8_t* __restrict__ frames, long long framePitch,
                                                int rowStride, uint8_t* __restrict__ pyr) {
    const int f = blockIdx.z;
    const int dw = g->L[level].w, dh = g->L[level].h;
    const int x0 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;   // 4 output pixels -> one dword store
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x0 >= dw || y >= dh) return;
    const LevelPtr src = level_ptr(g, level - 1, frames, framePitch, rowStride, pyr, f);
    const ResizeCoef cy = coef[dw + y];
    const uint8_t* r0 = src.p + (long long)cy.s0 * src.stride;
    const uint8_t* r1 = src.p + (long long)cy.s1 * src.stride;
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int x = min(x0 + i, dw - 1);
        const ResizeCoef cx = coef[x];
        const unsigned h0 = __umul24(r0[cx.s0], (unsigned)cx.c0) + __umul24(r0[cx.s1], (unsigned)cx.c1);
        const unsigned h1 = __umul24(r1[cx.s0], (unsigned)cx.c0) + __umul24(r1[cx.s1], (unsigned)cx.c1);
        const unsigned v =
            GENERIC ? min((__umul24((unsigned)cy.c0, h0) + __umul24((unsigned)cy.c1, h1) + (1u << 21)) >> 22, 255u)
                    : ((__umul24((unsigned)cy.c0, h0 >> 4) >> 16) + (__umul24((unsigned)cy.c1, h1 >> 4) >> 16) + 2) >> 2;
        packed |= (uint32_t)v << (8 * i);
    }
    // the pitch is a multiple of 64, so the dword never leaves the row (pad bytes are never read)
    uint8_t* dst = pyr + (long long)f * g->pyr_bytes + g->L[level].pyr_off;
    *reinterpret_cast<uint32_t*>(dst + (long long)y * g->L[level].pitch + x0) = packed;
}

/* Same arithmetic, LDS-tiled: a block produces a 128 x TH output tile.  The tile's source span
 * (<= 272 x (2*TH+8) bytes from a 16-byte aligned column, checked on the host: LevelGeom::rs_tiled)
 * is staged with 16-byte loads, all issued before the first wait (dword / byte loads if the level
 * base or stride is not 16-byte aligned), the coefficients of the tile's columns/rows are staged
 * once, and each thread then produces 4 output pixels per row pass (one dword store) from LDS byte
 * reads. */
// s_cy entry of one output row: the LDS byte offsets of its two source rows and the vertical weights
// pre-shifted for the vertical pass, (c * (h >> 4)) >> 16 == mul_hi_u24(c << 12, h & ~15) (c <= 2048 and
// h < 2^19 keep both operands within 24 bits); unshifted for the generic form
template <bool GENERIC>
__device__ __forceinline__ int4 rs_row_entry(const ResizeCoef& c, int sy0) {
    return make_int4(__mul24(c.s0 - sy0, kRsPitch), __mul24(c.s1 - sy0, kRsPitch), GENERIC ? c.c0 : c.c0 << 12,
                     GENERIC ? c.c1 : c.c1 << 12);
}
// one output pixel's vertical pass from the two rows' horizontal sums (weights from rs_row_entry)
template <bool GENERIC>
__device__ __forceinline__ unsigned rs_vpass(unsigned c0, unsigned c1, unsigned h0, unsigned h1) {
    if (GENERIC) return min((__umul24(c0, h0) + __umul24(c1, h1) + (1u << 21)) >> 22, 255u);
    return (mul_hi_u24(c0, h0 & ~15u) + mul_hi_u24(c1, h1 & ~15u) + 2) >> 2;
}

// Cache policy of the loads and stores that hand data between workgroups inside one launch (the small-batch
// dataflow launch k_extract_flow, below): 0 everywhere else; kCpSc1 = sc1, the write-through stores and
// L1-bypassing loads of MI355X_MICROARCH.md's inter-workgroup hand-off (every producer store and every consumer
// load of the handed-off bytes carries it, so no release or acquire fence is needed)
constexpr int kCpSc1 = 16;

// One 128 x TH output tile (bx, by) of level `level` for frame f, by the 256 threads tid = 0..255 of a block (or
// of a quarter of k_extract_flow's 1024-thread block: every thread of the block reaches its one barrier; an
// inactive quarter stages nothing and stores nothing).
// (65536 + n - 1) / n for n = 0..17 (n = 0 unused): the staging loop's i / nq as a multiply; a table lookup with a
// block-uniform index is one scalar load, where the division is a VALU sequence with two quarter-rate multiplies
__constant__ unsigned kRsMagic[18] = {0,    65536, 32768, 21846, 16384, 13108, 10923, 9363, 8192,
                                      7282, 6554,  5958,  5462,  5042,  4682,  4370,  4096, 3856};
// KP: 16-byte source chunks each thread stages (0: the tile height's worst case; the batch launch picks the
// level's own bound, LevelGeom::rs_chunks, so a 1.2-scale level issues two loads per thread instead of five
// clamped duplicates).
template <int kRsTileH, bool GENERIC, int CP, int KP = 0>
__device__ __forceinline__ void resize_tile(const Geom* __restrict__ g, const ResizeCoef* __restrict__ coef, int level,
                                            const uint8_t* __restrict__ frames, long long framePitch, int rowStride,
                                            uint8_t* __restrict__ pyr, int f, int bx, int by, int tid, uint8_t* s_src,
                                            int4* s_cx, int4* s_cy, bool active) {
    constexpr int kRows = rs_rows(kRsTileH);
    constexpr int kQ = kRsPitch / 16;                                  // 16-byte chunks per LDS row
    constexpr int kPer = KP > 0 ? KP : (kRows * kQ + 255) / 256;       // chunks per thread (upper bound)
    const int dw = g->L[level].w, dh = g->L[level].h;
    const int x0 = bx * kRsTileW, y0 = by * kRsTileH;
    const LevelPtr src = level_ptr(g, level - 1, frames, framePitch, rowStride, pyr, f);
    const int nx = min(kRsTileW, dw - x0), ny = min(kRsTileH, dh - y0);
    if (!active) {
        __syncthreads();
        return;
    }
    // source span (the coefficient tables are monotone); wave-uniform, so these are scalar loads
    const bool vec16 = ((reinterpret_cast<uintptr_t>(src.p) | (uintptr_t)src.stride) & 15) == 0;
    const int sx0 = coef[x0].s0 & (vec16 ? ~15 : ~3), sx1 = coef[x0 + nx - 1].s1;
    const int sy0 = coef[dw + y0].s0, sy1 = coef[dw + y0 + ny - 1].s1;
    const int nr = sy1 - sy0 + 1;
    const uint8_t* base = src.p + (long long)sy0 * src.stride + sx0;
    int4 cxv = make_int4(0, 0, 0, 0), cyv = make_int4(0, 0, 0, 0);
    if (vec16) {
        const int nq = ((sx1 - sx0) >> 4) + 1;
        const unsigned magic = kRsMagic[nq];                            // i / nq for i < 4096, nq <= 17
        const int total = nr * nq;
        // a buffer descriptor over the span (SGPRs): 32-bit row offsets (r * stride < 2^24 * 100 fits), no
        // 64-bit address arithmetic per chunk
        const uint64_t pb = reinterpret_cast<uint64_t>(base);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(pb), 0, 0x7FFFFFFF, 0x00020000);
        uint4 v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {   // unconditional (clamped) loads: all in flight before the first wait
            const int i = min(tid + 256 * k, total - 1);
            const int r = (int)(__umul24((unsigned)i, magic) >> 16), q = i - (int)__umul24((unsigned)r, (unsigned)nq);
            const uint32x4_t w = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)__umul24((unsigned)r, (unsigned)src.stride) + 16 * q, 0, CP);
            v[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        if (tid < kRsTileW) {
            const ResizeCoef c = coef[x0 + min(tid, nx - 1)];
            cxv = make_int4(c.s0, c.s1, c.c0, c.c1);
        }
        if (tid < kRsTileH) {
            const ResizeCoef c = coef[dw + y0 + min(tid, ny - 1)];
            cyv = rs_row_entry<GENERIC>(c, sy0);
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {   // clamped duplicates store the same bytes to the same place
            const int i = min(tid + 256 * k, total - 1);
            const int r = (int)(__umul24((unsigned)i, magic) >> 16), q = i - (int)__umul24((unsigned)r, (unsigned)nq);
            *reinterpret_cast<uint4*>(&s_src[r * kRsPitch + 16 * q]) = v[k];
        }
    } else {
        if (tid < kRsTileW) {
            const ResizeCoef c = coef[x0 + min(tid, nx - 1)];
            cxv = make_int4(c.s0, c.s1, c.c0, c.c1);
        }
        if (tid < kRsTileH) {
            const ResizeCoef c = coef[dw + y0 + min(tid, ny - 1)];
            cyv = rs_row_entry<GENERIC>(c, sy0);
        }
        if (((reinterpret_cast<uintptr_t>(src.p) | (uintptr_t)src.stride) & 3) == 0) {
            const int nw = (sx1 - sx0 + 4) >> 2;
            for (int i = tid; i < nr * 68; i += 256) {   // 68 dwords per LDS row
                const int r = i / 68, wd = i - r * 68;
                if (wd < nw)
                    *reinterpret_cast<uint32_t*>(&s_src[r * kRsPitch + 4 * wd]) =
                        *reinterpret_cast<const uint32_t*>(base + (long long)r * src.stride + 4 * wd);
            }
        } else {
            const int nb = sx1 - sx0 + 1;
            for (int i = tid; i < nr * kRsPitch; i += 256) {
                const int r = i / kRsPitch, b = i - r * kRsPitch;
                if (b < nb) s_src[r * kRsPitch + b] = base[(long long)r * src.stride + b];
            }
        }
    }
    if (tid < kRsTileW) s_cx[tid] = cxv;
    if (tid < kRsTileH) s_cy[tid] = cyv;
    __syncthreads();
    // Weights are <= 2048 and pixels <= 255, so every product fits 24-bit multiplies (full rate;
    // a 32-bit v_mul_lo is quarter rate).  s_cx / s_cy hold clamped entries for the whole tile.
    const int tx = (tid & 31) * 4;
    int o0[4], o1[4];
    unsigned c0[4], c1[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int4 cx = s_cx[tx + i];
        o0[i] = cx.x - sx0;
        o1[i] = cx.y - sx0;
        c0[i] = cx.z;
        c1[i] = cx.w;
    }
    // the level's rows through a buffer descriptor (block-uniform base in SGPRs): 32-bit store offsets
    const uint64_t lb = reinterpret_cast<uint64_t>(pyr + (long long)f * g->pyr_bytes + g->L[level].pyr_off);
    const auto dsr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(lb >> 32)) << 32) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)lb)),
        0, 0x7FFFFFFF, 0x00020000);
    const int pitch = g->L[level].pitch;
    const unsigned dcol = (unsigned)(x0 + tx);
    if (tx >= nx) return;
    // The 4 pixels' source bytes lie within 8 bytes from o0[0] (scale factor <= ~1.6; otherwise the
    // byte path below): a row's 3 dwords from LDS, realigned to o0[0], give each pixel's byte pair as
    // 16-bit lanes through one v_perm, and the horizontal sum is one v_dot2 with (c0, c1).
    const int bo = o0[0];
    const bool packed_ok = o1[3] - bo <= 7;
    if (__builtin_amdgcn_ballot_w64(!packed_ok) == 0) {
        unsigned sel[4];
        uint32_t cc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            sel[i] = (unsigned)(o0[i] - bo) | 0x0C00u | ((unsigned)(o1[i] - bo) << 16) | 0x0C000000u;
            cc[i] = c0[i] | (c1[i] << 16);
        }
        const int bw = bo >> 2, bsh = bo & 3;
#pragma unroll
        for (int pass = 0; pass < kRsTileH / 8; pass++) {
            const int ty = pass * 8 + (tid >> 5);
            if (ty >= ny) break;
            const int4 cy = s_cy[ty];   // (LDS offsets of the two source rows, c0 << 12, c1 << 12)
            const unsigned cy0 = (unsigned)cy.z, cy1 = (unsigned)cy.w;
            const uint32_t* q0 = reinterpret_cast<const uint32_t*>(&s_src[cy.x]) + bw;
            const uint32_t* q1 = reinterpret_cast<const uint32_t*>(&s_src[cy.y]) + bw;
            const uint32_t u0 = q0[0], u1 = q0[1], u2 = q0[2], w0 = q1[0], w1 = q1[1], w2 = q1[2];
            const uint32_t a0 = __builtin_amdgcn_alignbyte(u1, u0, bsh), a1 = __builtin_amdgcn_alignbyte(u2, u1, bsh);
            const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, bsh), b1 = __builtin_amdgcn_alignbyte(w2, w1, bsh);
            uint32_t packed = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const unsigned h0 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cc[i]),
                                                           __builtin_bit_cast(ushort2_t, __builtin_amdgcn_perm(a1, a0, sel[i])), 0u, false);
                const unsigned h1 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cc[i]),
                                                           __builtin_bit_cast(ushort2_t, __builtin_amdgcn_perm(b1, b0, sel[i])), 0u, false);
                const unsigned v = rs_vpass<GENERIC>(cy0, cy1, h0, h1);
                packed |= v << (8 * i);
            }
            __builtin_amdgcn_raw_buffer_store_b32(packed, dsr, (int)(__umul24((unsigned)(y0 + ty), (unsigned)pitch) + dcol), 0, CP);
        }
        return;
    }
#pragma unroll
    for (int pass = 0; pass < kRsTileH / 8; pass++) {
        const int ty = pass * 8 + (tid >> 5);
        if (ty >= ny) break;
        const int4 cy = s_cy[ty];
        const uint8_t* r0 = &s_src[cy.x];
        const uint8_t* r1 = &s_src[cy.y];
        uint32_t packed = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const unsigned h0 = __umul24(r0[o0[i]], c0[i]) + __umul24(r0[o1[i]], c1[i]);
            const unsigned h1 = __umul24(r1[o0[i]], c0[i]) + __umul24(r1[o1[i]], c1[i]);
            const unsigned v = rs_vpass<GENERIC>((unsigned)cy.z, (unsigned)cy.w, h0, h1);
            packed |= v << (8 * i);
        }
        __builtin_amdgcn_raw_buffer_store_b32(packed, dsr, (int)(__umul24((unsigned)(y0 + ty), (unsigned)pitch) + dcol), 0, CP);
    }
}

template <int kRsTileH, bool GENERIC, int KP>
__global__ __launch_bounds__(256) void k_resize_tiled(const Geom* __restrict__ g,
                                                      const ResizeCoef* __restrict__ coef, int level,
                                                      const uint8_t* __restrict__ frames, long long framePitch,
                                                      int rowStride, uint8_t* __restrict__ pyr) {
    // the source tile, sized on the host to the level's largest span (LevelGeom::rs_span_rows <= kRows)
    // rather than kRows: a smaller block footprint, more resident blocks
    extern __shared__ __attribute__((aligned(16))) uint8_t s_src[];
    __shared__ int4 s_cx[kRsTileW];
    __shared__ int4 s_cy[kRsTileH];
    resize_tile<kRsTileH, GENERIC, 0, KP>(g, coef, level, frames, framePitch, rowStride, pyr, blockIdx.z, blockIdx.x,
                                          blockIdx.y, threadIdx.x, s_src, s_cx, s_cy, true);
}

/* Few-launch pyramid for small batches (the host path's single frame, C5's per-GPU frame): the levels
 * in segments of up to kChainSeg, ONE launch per segment instead of one per level.  A workgroup owns
 * an output tile of one level and recomputes, in LDS, the chain of regions it depends on from the
 * segment's base level up (ChainJob; the same fixed-point arithmetic as k_resize_tiled, so every value
 * is the per-level launch's), writing only its own tile.  The recomputation is redundant work, but a
 * single frame leaves most of the chip idle, and each dependent launch costs ~5 us of latency. */
// a dword / byte of a level the chain reads as its base: plain, or (CP) an sc1 load of a level handed off
// inside the dataflow launch
template <int CP>
__device__ __forceinline__ uint32_t chain_ld32(const uint8_t* p) {
    if constexpr (CP != 0)
        return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *reinterpret_cast<const uint32_t*>(p);
}
template <int CP>
__device__ __forceinline__ uint32_t chain_ld8(const uint8_t* p) {
    if constexpr (CP != 0) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        return (w >> (8 * (a & 3))) & 0xFFu;
    } else {
        return *p;
    }
}

// One ChainJob (an output tile of J->level from level J->base) by the 256 threads tid = 0..255 of a block or of a
// quarter of k_extract_flow's block (every thread of the block reaches the job's barriers, 2 + level - base of them:
// jobs run together share level and base).  sm: the segment's carve (sg.lds_bytes), sreg: ORBGPU_MAX_LEVELS int4.
template <bool GENERIC, int CP>
__device__ __forceinline__ void chain_job(const Geom* __restrict__ g, const ResizeCoef* __restrict__ coef,
                                          const ChainJob* __restrict__ J, const ChainSegment& sg, const RcoefOff& roff,
                                          const uint8_t* __restrict__ frames, long long framePitch, int rowStride,
                                          uint8_t* __restrict__ pyr, int f, int tid, uint8_t* sm, int4* sreg) {
    const int l = J->level, b = J->base;
    if (tid <= l) sreg[tid] = J->reg[tid];
    uint8_t* buf0 = sm;
    uint8_t* buf1 = sm + sg.buf_bytes;
    int4* sc = reinterpret_cast<int4*>(sm + 2 * sg.buf_bytes);
    uint8_t* fp = pyr + (long long)f * g->pyr_bytes;
    __syncthreads();
    // coefficients of every stage, relative to its source region in LDS: columns (o0, o1, c0, c1), rows
    // (byte offsets of the two source rows, vertical weights as rs_row_entry) -- all loads in flight at once
    {
        int e0 = 0;
        for (int k = b + 1; k <= l; k++) {
            const int4 R = sreg[k], S = sreg[k - 1];
            const int nx = R.y - R.x, ny = R.w - R.z;
            const int sp = (S.y - S.x + 3) & ~3;   // source region pitch
            const ResizeCoef* cx = coef + roff.o[k];
            const int wk = g->L[k].w;
            for (int e = tid; e < nx + ny; e += 256) {
                int4 v;
                if (e < nx) {
                    const ResizeCoef c = cx[min(R.x + e, wk - 1)];
                    v = make_int4(c.s0 - S.x, c.s1 - S.x, c.c0, c.c1);
                } else {
                    const ResizeCoef c = cx[wk + R.z + (e - nx)];
                    v = rs_row_entry<GENERIC>(c, S.z);
                    v.x = (c.s0 - S.z) * sp;
                    v.y = (c.s1 - S.z) * sp;
                }
                sc[e0 + e] = v;
            }
            e0 += nx + ny;
        }
    }
    // the base level's region: dwords where the rows allow, bytes at the right edge
    {
        const int4 R = sreg[b];
        const int p0 = (R.y - R.x + 3) & ~3, nq = p0 >> 2, ny = R.w - R.z, wb = g->L[b].w;
        const uint8_t* src = b == 0 ? frames + (long long)f * framePitch : fp + g->L[b].pyr_off;
        const int stride = b == 0 ? rowStride : g->L[b].pitch;
        const bool al = ((reinterpret_cast<uintptr_t>(src) | (uintptr_t)stride) & 3) == 0;
        const int QW = nq <= 16 ? 16 : nq <= 32 ? 32 : 64, RP = 256 / QW;
        for (int qb = 0; qb < nq; qb += QW)
            for (int r = tid / QW; r < ny; r += RP) {
                const int q = qb + (tid & (QW - 1));
                if (q >= nq) continue;
                const int col = R.x + 4 * q;
                const uint8_t* rp = src + (long long)(R.z + r) * stride;
                uint32_t v;
                if (al && col + 3 < wb) {
                    v = chain_ld32<CP>(rp + col);
                } else {
                    v = 0;
                    for (int t = 0; t < 4; t++)
                        if (col + t < wb) v |= chain_ld8<CP>(rp + col + t) << (8 * t);
                }
                *reinterpret_cast<uint32_t*>(buf0 + r * p0 + 4 * q) = v;
            }
    }
    __syncthreads();
    int e0 = 0;
    for (int k = b + 1; k <= l; k++) {
        const int4 R = sreg[k];
        const int nx = R.y - R.x, ny = R.w - R.z, nq = nx >> 2;
        const uint8_t* src = ((k - b) & 1) ? buf0 : buf1;
        uint8_t* dst = ((k - b) & 1) ? buf1 : buf0;
        const int4* cxs = sc + e0;
        const int4* cys = sc + e0 + nx;
        const bool last = k == l;
        uint8_t* gl = fp + g->L[k].pyr_off;
        const int gpitch = g->L[k].pitch, wk = g->L[k].w;
        const int QW = nq <= 16 ? 16 : nq <= 32 ? 32 : 64, RP = 256 / QW;
        for (int qb = 0; qb < nq; qb += QW) {
            const int q = qb + (tid & (QW - 1));
            const bool qon = q < nq;
            // the dword group's 4 pixels: source byte offsets, weights; their bytes lie within 8 from bo
            // when the scale factor is <= ~1.6 (then 3 dwords + v_perm + v_dot2 per row, else bytes)
            int o0[4], o1[4];
            unsigned c0[4], c1[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int4 cx = cxs[qon ? 4 * q + t : 0];
                o0[t] = cx.x;
                o1[t] = cx.y;
                c0[t] = cx.z;
                c1[t] = cx.w;
            }
            const int bo = o0[0], bw = bo >> 2, bsh = bo & 3;
            const bool packed_ok = o1[3] - bo <= 7;
            unsigned sel[4];
            uint32_t cc[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                sel[t] = (unsigned)(o0[t] - bo) | 0x0C00u | ((unsigned)(o1[t] - bo) << 16) | 0x0C000000u;
                cc[t] = c0[t] | (c1[t] << 16);
            }
            for (int r = tid / QW; r < ny; r += RP) {
                if (!qon) continue;
                const int4 cy = cys[r];
                uint32_t packed = 0;
                if (packed_ok) {
                    // a row's 3 dwords from the aligned one, realigned to bo (as k_resize_tiled)
                    const uint32_t* q0 = reinterpret_cast<const uint32_t*>(src + cy.x) + bw;
                    const uint32_t* q1 = reinterpret_cast<const uint32_t*>(src + cy.y) + bw;
                    const uint32_t u0 = q0[0], u1 = q0[1], u2 = q0[2], w0 = q1[0], w1 = q1[1], w2 = q1[2];
                    const uint32_t a0 = __builtin_amdgcn_alignbyte(u1, u0, bsh), a1 = __builtin_amdgcn_alignbyte(u2, u1, bsh);
                    const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, bsh), d1 = __builtin_amdgcn_alignbyte(w2, w1, bsh);
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        const unsigned h0 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cc[t]),
                                                                   __builtin_bit_cast(ushort2_t, __builtin_amdgcn_perm(a1, a0, sel[t])), 0u, false);
                        const unsigned h1 = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, cc[t]),
                                                                   __builtin_bit_cast(ushort2_t, __builtin_amdgcn_perm(d1, d0, sel[t])), 0u, false);
                        packed |= rs_vpass<GENERIC>((unsigned)cy.z, (unsigned)cy.w, h0, h1) << (8 * t);
                    }
                } else {
                    const uint8_t* r0 = src + cy.x;
                    const uint8_t* r1 = src + cy.y;
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        const unsigned h0 = __umul24(r0[o0[t]], c0[t]) + __umul24(r0[o1[t]], c1[t]);
                        const unsigned h1 = __umul24(r1[o0[t]], c0[t]) + __umul24(r1[o1[t]], c1[t]);
                        packed |= rs_vpass<GENERIC>((unsigned)cy.z, (unsigned)cy.w, h0, h1) << (8 * t);
                    }
                }
                if (!last) {
                    *reinterpret_cast<uint32_t*>(dst + r * nx + 4 * q) = packed;
                } else if (R.x + 4 * q < wk) {   // the pitch is a multiple of 64: the dword never leaves the row
                    uint32_t* dp = reinterpret_cast<uint32_t*>(gl + (long long)(R.z + r) * gpitch + R.x + 4 * q);
                    if constexpr (CP != 0) __hip_atomic_store(dp, packed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else *dp = packed;
                }
            }
        }
        e0 += nx + ny;
        if (!last) __syncthreads();
    }
}

template <bool GENERIC>
__global__ __launch_bounds__(256) void k_pyramid_chain(const Geom* __restrict__ g, const ResizeCoef* __restrict__ coef,
                                                       const ChainJob* __restrict__ jobs, ChainSegment sg,
                                                       RcoefOff roff, const uint8_t* __restrict__ frames,
                                                       long long framePitch, int rowStride, uint8_t* __restrict__ pyr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    __shared__ int4 sreg[ORBGPU_MAX_LEVELS];
    chain_job<GENERIC, 0>(g, coef, jobs + sg.job0 + blockIdx.x, sg, roff, frames, framePitch, rowStride, pyr,
                          blockIdx.y, threadIdx.x, sm, sreg);
}

/* ------------------------------------------------------------------------------------------------
 * FAST-9/16 + NMS per cell, with the iniThFAST -> minThFAST fallback
 * (ComputeKeyPointsOctTree, ORBextractor.cc:789-828; cv::FAST semantics SURVEY Appendix A.3).
 * One workgroup per (cell, frame).  The cell ROI is staged in LDS; M = max over the 16 9-arcs of
 * the min |difference| (bright or dark) is threshold-independent, so:
 *   corner(th)  <=>  M > th,     score = M - 1,
 * and NMS compares against neighbours inside the cell's detection domain only (cells' domains
 * tile the level without overlap; outside / non-corner neighbours count 0, as OpenCV's row
 * buffers do for a ROI).  Survivors are emitted in raster order (FAST emission order), packed
 * x_rel | y_rel<<12 | score<<24 with coordinates relative to minBorder (:822-823).
 * --------------------------------------------------------------------------------------------- */
// c = the centre pixel's byte; pixels CS bytes apart in a row, rows P bytes apart (the 16-bit tile's
// low bytes: CS = 2).  On the raw circle values p: the dark strength max over arcs of min (v - p) is
// v - X with X = min over arcs of max p, the bright one Y - v with Y = max over arcs of min p, so
// M = max(v - X, Y - v, 0) needs no per-pixel differences.
// Both sides run in one packed chain: each circle value is held as the f16 pair (p, -p) (bit patterns;
// p < 256 is a positive f16 denormal, -p its negation, and f16 order on them is integer order, denormals
// preserved: float_denorm_mode_16_64 = 3), so one v_pk_maximum3_f16 takes the max of p over a 3-run in
// the low half and the max of -p = -(min p) in the high half: the 9-arc extrema of both sides are 16 + 16
// pk_maximum3, their min over the 16 arcs 8 pk_minimum3 (the -p negation folds into neg_hi modifiers).
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2_t circle_pair(int p) {   // (p, -p)
    half2_t q = __builtin_bit_cast(half2_t, (uint32_t)p * 0x10001u);
    q.y = -q.y;
    return q;
}
__device__ __forceinline__ half2_t pk_max3h(half2_t a, half2_t b, half2_t c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ half2_t pk_min3h(half2_t a, half2_t b, half2_t c) {
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}

template <int P, int CS>
__device__ __forceinline__ int fast_arc_strength(const uint8_t* c) {
    const int v = c[0];
    half2_t q[16];
    q[0] = circle_pair(c[0 * CS + 3 * P]);
    q[1] = circle_pair(c[1 * CS + 3 * P]);
    q[2] = circle_pair(c[2 * CS + 2 * P]);
    q[3] = circle_pair(c[3 * CS + 1 * P]);
    q[4] = circle_pair(c[3 * CS + 0 * P]);
    q[5] = circle_pair(c[3 * CS + -1 * P]);
    q[6] = circle_pair(c[2 * CS + -2 * P]);
    q[7] = circle_pair(c[1 * CS + -3 * P]);
    q[8] = circle_pair(c[0 * CS + -3 * P]);
    q[9] = circle_pair(c[-1 * CS + -3 * P]);
    q[10] = circle_pair(c[-2 * CS + -2 * P]);
    q[11] = circle_pair(c[-3 * CS + -1 * P]);
    q[12] = circle_pair(c[-3 * CS + 0 * P]);
    q[13] = circle_pair(c[-3 * CS + 1 * P]);
    q[14] = circle_pair(c[-2 * CS + 2 * P]);
    q[15] = circle_pair(c[-1 * CS + 3 * P]);
    // 9-arc [k, k+8] = three 3-runs
    half2_t x3[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x3[k] = pk_max3h(q[k], q[(k + 1) & 15], q[(k + 2) & 15]);
    half2_t a = pk_max3h(x3[0], x3[3], x3[6]);
#pragma unroll
    for (int k = 1; k < 16; k += 2)   // two arcs per v_pk_minimum3
        a = pk_min3h(a, pk_max3h(x3[k], x3[(k + 3) & 15], x3[(k + 6) & 15]),
                     k + 1 < 16 ? pk_max3h(x3[k + 1], x3[(k + 4) & 15], x3[(k + 7) & 15]) : a);
    const uint32_t u = __builtin_bit_cast(uint32_t, a);   // low: X = min over arcs of max p; high: -Y
    const int X = (int)(u & 0xFFu), Y = (int)((u >> 16) & 0xFFu);
    return max(max(v - X, Y - v), 0);
}

// Host table of the cells (ComputeKeyPointsOctTree's grid, ORBextractor.cc:781-806), frame independent.
void build_cells(const Geom& g, std::vector<CellDesc>& cells) {
    cells.assign(g.ncells, CellDesc{});
    for (int l = 0; l < g.nlevels; l++) {
        const LevelGeom& L = g.L[l];
        for (int ci = 0; ci < L.nRows; ci++)
            for (int cj = 0; cj < L.nCols; cj++) {
                const int cc = ci * L.nCols + cj;
                CellDesc& d = cells[L.cell_base + cc];
                const int iniY = kMinBorder + ci * L.hCell, iniX = kMinBorder + cj * L.wCell;
                bool valid = !(iniY >= L.maxBY - 3 || iniX >= L.maxBX - 6);   // :794-806
                const int maxY = std::min(iniY + L.hCell + 6, L.maxBY), maxX = std::min(iniX + L.wCell + 6, L.maxBX);
                const int rw = maxX - iniX, rh = maxY - iniY;
                valid = valid && rw - 6 > 0 && rh - 6 > 0;
                d.lv = l | (valid ? 1 << 8 : 0);
                d.iniX = iniX;
                d.iniY = iniY;
                d.rwrh = (rw & 0xFFFF) | (rh << 16);
                d.out_off = L.cand_base + cc * L.cell_cap;
                d.xoyo = (3 + cj * L.wCell) | ((3 + ci * L.hCell) << 16);
                d.pitch = L.pitch;
                d.pyr_off = (int)L.pyr_off;
                const int x0w = iniX >> 2, nw = std::max(1, ((iniX + rw + 3) >> 2) - x0w);
                const int nruns = std::max(1, (rw - 6 + 15) / 16);   // 16-pixel prefilter runs
                d.roi = nw | ((64 / nw) << 8) | (x0w << 16);
                d.m_nw = (int)recip20((uint32_t)nw);
                d.runs = nruns | ((64 / nruns) << 8);
                d.m_runs = (int)recip20((uint32_t)nruns);
            }
    }
}

// Byte offset of row yy at column byte cb (yy, stride < 2^24, yy * stride < 2^32): one 24-bit multiply
// (full rate) instead of 64-bit address arithmetic (quarter-rate v_mul_lo_u32 / v_mad_u64_u32).
__device__ __forceinline__ unsigned roi_off(int yy, int stride, int cb) {
    return __umul24((unsigned)yy, (unsigned)stride) + (unsigned)cb;
}

struct FastCellT {
    int f, cell, iniX, rw, rh, dw, dh, x0w, nw, rpr, m_nw, nruns, rpi, m_runs, out_off, xo, yo;
    bool valid, aligned;
    const uint8_t* base;   // ROI row 0, column 0
    int stride;
};

__device__ __forceinline__ FastCellT fast_cell_t(const Geom* __restrict__ g, const CellDesc* __restrict__ cells,
                                                 int item, const uint8_t* frames, long long framePitch, int rowStride,
                                                 const uint8_t* pyr, int cbeg, int cnum) {
    FastCellT c;   // items cover cells [cbeg, cbeg + cnum) of every frame
    c.f = item / cnum;
    c.cell = cbeg + item - c.f * cnum;
    const CellDesc d = cells[c.cell];   // one scalar load
    const int l = d.lv & 0xFF;
    c.valid = (d.lv >> 8) & 1;
    c.iniX = d.iniX;
    c.rw = d.rwrh & 0xFFFF;
    c.rh = d.rwrh >> 16;
    c.dw = c.rw - 6;
    c.dh = c.rh - 6;
    c.out_off = d.out_off;
    c.xo = d.xoyo & 0xFFFF;
    c.yo = d.xoyo >> 16;
    const uint8_t* lp = l == 0 ? frames + (long long)c.f * framePitch : pyr + (long long)c.f * g->pyr_bytes + d.pyr_off;
    c.stride = l == 0 ? rowStride : d.pitch;
    c.base = lp + (long long)d.iniY * c.stride;
    c.aligned = ((reinterpret_cast<uintptr_t>(lp) | (uintptr_t)c.stride) & 3) == 0;
    c.nw = d.roi & 0xFF;
    c.rpr = (d.roi >> 8) & 0xFF;
    c.x0w = d.roi >> 16;
    c.m_nw = d.m_nw;
    c.nruns = d.runs & 0xFF;
    c.rpi = (d.runs >> 8) & 0xFF;
    c.m_runs = d.m_runs;
    return c;
}

// wave-level scans (DPP) for the wave-per-cell FAST kernel below
__device__ __forceinline__ int wave_excl_scan(int v) {
    const int lane = threadIdx.x & 63;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x - v;
}

// Wavefront inclusive scan with DPP: row_shr 1/2/4/8 inside each 16-lane row (zero fill at the row
// start), then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the row totals.
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    return x;
}

__device__ __forceinline__ int wave_sum(int v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }

// q = x / n for x < 2^20 / n via the 20-bit reciprocal m = recip20(n) (n <= 64): two VALU ops, exact.
__device__ __forceinline__ uint32_t div20(uint32_t x, uint32_t m) { return __umul24(x, m) >> 20; }

typedef short short2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {   // per 16-bit lane a - b (v_pk_sub_i16)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, a) - __builtin_bit_cast(short2_t, b));
}
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {   // per 16-bit lane a + b (v_pk_add_i16)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, a) + __builtin_bit_cast(short2_t, b));
}

// Compass prefilter (see fast_maybe) for two pixels held as 16-bit lanes: returns sign bits 15/31
// set where the pixel may be a corner at threshold t.  Bright: (v+t) - p < 0, dark: p - (v-t) < 0;
// the four cyclically adjacent compass pairs reduce to (b0|b8) & (b4|b12).
// As min/max: bright needs min(max(p0, p8), max(p4, p12)) > v + t, dark max(min(p0, p8), min(p4, p12))
// < v - t, i.e. max(hi - v, v - lo) > t (10 packed ops for the two pixels instead of 16).
typedef unsigned short ushort2_pk __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t compass2(uint32_t v, uint32_t p0, uint32_t p4, uint32_t p8, uint32_t p12,
                                             uint32_t tt) {
    const ushort2_pk a0 = __builtin_bit_cast(ushort2_pk, p0), a4 = __builtin_bit_cast(ushort2_pk, p4),
                     a8 = __builtin_bit_cast(ushort2_pk, p8), a12 = __builtin_bit_cast(ushort2_pk, p12);
    const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_max(a0, a8),
                                                                               __builtin_elementwise_max(a4, a12)));
    const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_elementwise_min(a0, a8),
                                                                               __builtin_elementwise_min(a4, a12)));
    // bright (hi > v + t) or dark (lo < v - t)  <=>  max(hi - v, v - lo) > t: the sign of t - max
    const short2_t d = __builtin_elementwise_max(__builtin_bit_cast(short2_t, pk_sub16(hi, v)),
                                                 __builtin_bit_cast(short2_t, pk_sub16(v, lo)));
    return pk_sub16(tt, __builtin_bit_cast(uint32_t, d));
}

// optional phase timestamps (a build with -DORBGPU_KERNEL_STAMPS=1, run with ORBGPU_FAST_STAMPS=1):
// s_memtime at the phase boundaries, lane 0.  Off by default: each stamp is a branch that splits the
// kernel's scheduling regions (describe 0.533 -> 0.528, octree 0.102 -> 0.100 ms per 256 C3 frames)
#ifndef ORBGPU_KERNEL_STAMPS
#define ORBGPU_KERNEL_STAMPS 0
#endif
#if ORBGPU_KERNEL_STAMPS
#define ORBGPU_STAMP(k) \
    if (stamps && lane == 0) stamps[(long long)item * 8 + (k)] = __builtin_amdgcn_s_memtime();
#elif defined(ORBGPU_ISA_MARKS)   // tools/fast_isa_phases.py: phase boundaries as assembly comments (no instruction)
#define ORBGPU_STAMP(k) asm volatile(";ORBGPU_MARK " #k);
#else
#define ORBGPU_STAMP(k)
#endif

// ROI dwords of a cell (aligned levels) issued into registers, so that the next cell's loads are in
// flight while the current one is processed.  lane = (row yy0 = lane / nw, dword ww = lane % nw);
// round k takes row yy0 + k * rpr (rpr = 64 / nw rows per round): the lane's offset is computed once
// and each round adds a wave-uniform row step to the voffset of a buffer load whose descriptor (SGPRs)
// starts at the ROI's first dword.  Rows past the ROI and lanes past rpr rows are out of the
// descriptor's range (read 0).  Rows from 8 * rpr on (tall cells) are loaded by fast_roi_store.
struct RoiLanes {
    int yy0, ww, rpr, off;
    __amdgpu_buffer_rsrc_t rsrc;
};

__device__ __forceinline__ RoiLanes roi_lanes(const FastCellT& c, int lane) {
    RoiLanes r;
    const int nw = __builtin_amdgcn_readfirstlane(c.nw), stride = __builtin_amdgcn_readfirstlane(c.stride);
    r.rpr = c.rpr;
    r.yy0 = (int)div20(lane, c.m_nw);
    r.ww = lane - (int)__umul24((unsigned)r.yy0, (unsigned)nw);
    r.off = (int)roi_off(r.yy0, stride, 4 * r.ww);
    // the cell is wave-uniform (readfirstlane returns int: zero-extend both halves)
    const uint64_t pb = reinterpret_cast<uint64_t>(c.base + 4 * c.x0w);
    const uint64_t pu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(pb >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)pb);
    r.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(pu), 0, (c.rh - 1) * stride + 4 * nw, 0x00020000);
    return r;
}

__device__ __forceinline__ bool roi_row_ok(const FastCellT& c, const RoiLanes& r, int k) {
    return r.yy0 < r.rpr && r.yy0 + k * r.rpr < c.rh;
}

template <int CP = 0>
__device__ __forceinline__ void fast_roi_issue(const FastCellT& c, int lane, uint32_t (&v)[8]) {
    const RoiLanes r = roi_lanes(c, lane);
    // rows past the ROI lie past the descriptor's num_records ((rh - 1) * stride + 4 nw <= rh * stride
    // + 4 ww) and read 0 without a per-row test: the row step goes into voffset, which the range check
    // covers (soffset would not be checked); lanes past rpr rows start out of range
    const int off = r.yy0 < r.rpr ? r.off : 0x40000000;
#pragma unroll
    for (int k = 0; k < 8; k++)
        v[k] = __builtin_amdgcn_raw_buffer_load_b32(r.rsrc, off + k * r.rpr * c.stride, 0, CP);
}

// ROI -> 16-bit LDS tile (rows TQ elements apart): ROI column c at element c + 1, so that every
// prefilter window starts on a 16-byte boundary (see prefilter16).  The bytes are widened as they are
// stored.  ROI column c is byte c + B of the loaded row (B = the ROI's byte offset in its first dword),
// so a lane's dword (bytes 4 ww .. 4 ww + 3) goes to elements 4 ww - B + 1 .. 4 ww - B + 4, i.e. the
// pixel pairs at dwords 2 ww - (B >> 1) and + 1 are (b0, b1), (b2, b3) for B odd and (prev b3, b0),
// (b1, b2) for B even — prev = the row's previous dword, lane - 1's (DPP wave_shr), and the row's last
// dword also stores (b3, 0).  Dword -1 of row 0 lies in the carve's 16-byte lead pad, that of a later row
// in the previous row's unused tail (TQ >= rw + 6).  Rows of a tall ROI past the prefetched ones are
// loaded here; a level whose base / stride is not dword aligned is stored per byte.
__device__ __forceinline__ uint32_t dpp_prev_lane(uint32_t v) {   // lane - 1's value (lane 0: 0)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}

// v_perm selectors as SGPRs (a VOP3 takes no literal on gfx9: left to itself the compiler re-materialises
// one per store with a v_mov)
struct WidenSel {
    uint32_t lo, hi;
};
__device__ __forceinline__ uint32_t sgpr_const(uint32_t x) {
    uint32_t r;
    asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(x));
    return r;
}

template <bool ODD>
__device__ __forceinline__ void widen_store(uint32_t* q, uint32_t v, uint32_t pv, bool last, const WidenSel& S) {
    if (ODD) {   // (b0, b1), (b2, b3)
        q[0] = __builtin_amdgcn_perm(0u, v, S.lo);
        q[1] = __builtin_amdgcn_perm(0u, v, S.hi);
    } else {     // (prev b3, b0), (b1, b2) [, (b3, 0)]
        q[0] = __builtin_amdgcn_perm(v, pv, S.lo);
        q[1] = __builtin_amdgcn_perm(0u, v, S.hi);
        if (last) q[2] = v >> 24;
    }
}

// the prefetched rows (round k: ROI row yy0 + k * rpr) and, for a tall ROI, the rows past them
template <int TQ, bool ODD, int CP>
__device__ __forceinline__ void widen_rows(const FastCellT& c, const RoiLanes& r, const uint32_t (&v)[8], uint32_t* t32,
                                           int B, bool last) {
    const WidenSel S = ODD ? WidenSel{sgpr_const(0x0c010c00u), sgpr_const(0x0c030c02u)}
                           : WidenSel{sgpr_const(0x0c040c03u), sgpr_const(0x0c020c01u)};
    uint32_t* t = t32 + (r.yy0 * (TQ / 2) + 2 * r.ww - (B >> 1));
    const bool on = r.yy0 < r.rpr;
    const int rpr = __builtin_amdgcn_readfirstlane(r.rpr), rh = __builtin_amdgcn_readfirstlane(c.rh);
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int k0 = k * rpr;
        if (k0 >= rh) break;   // wave-uniform
        const uint32_t pv = ODD ? 0u : dpp_prev_lane(v[k]);
        if (on && r.yy0 + k0 < rh) widen_store<ODD>(t + k0 * (TQ / 2), v[k], pv, last, S);
    }
    if (on)
        for (int yy = r.yy0 + 8 * rpr; yy < rh; yy += rpr) {   // lanes of one row iterate together
            uint32_t w;
            if constexpr (CP != 0) w = __builtin_amdgcn_raw_buffer_load_b32(r.rsrc, (int)roi_off(yy, c.stride, 4 * r.ww), 0, CP);
            else w = *reinterpret_cast<const uint32_t*>(c.base + roi_off(yy, c.stride, (c.x0w + r.ww) * 4));
            const uint32_t pw = ODD ? 0u : dpp_prev_lane(w);
            widen_store<ODD>(t32 + (yy * (TQ / 2) + 2 * r.ww - (B >> 1)), w, pw, last, S);
        }
}

// (CP: the unaligned byte path below reads only the caller's frame, level 0, never handed-off pyramid bytes: the
// pyramid levels are 64-byte aligned rows in a 256-byte aligned slot)
template <int TQ, int CP = 0>
__device__ __forceinline__ void fast_roi_store(const FastCellT& c, int lane, const uint32_t (&v)[8], uint16_t* tile) {
    uint32_t* t32 = reinterpret_cast<uint32_t*>(tile);
    if (c.aligned) {
        const RoiLanes r = roi_lanes(c, lane);
        const int B = c.iniX & 3;
        const bool last = r.ww == __builtin_amdgcn_readfirstlane(c.nw) - 1;
        if (B & 1) widen_rows<TQ, true, CP>(c, r, v, t32, B, last);
        else widen_rows<TQ, false, CP>(c, r, v, t32, B, last);
        return;
    }
    const uint32_t mrw = recip20(c.rw);
    for (int idx = lane; idx < c.rh * c.rw; idx += 64) {
        const int yy = (int)div20(idx, mrw), xx = idx - (int)__umul24((unsigned)yy, (unsigned)c.rw);
        tile[yy * TQ + xx + 1] = c.base[roi_off(yy, c.stride, c.iniX + xx)];
    }
}

// Survivor bits (bit k = pixel x0 + k) of the compass prefilter at threshold t (tt = t | t << 16) for 8
// pixels of domain row dy, in the 16-bit tile where domain pixel (x, y) is element (y + 3) * TQ + x + 4.
// Each tile dword is a pixel pair, so the centre row's 8 dwords from element x0 (two 16-byte reads) hold
// the centre pairs (x0 + 2j, x0 + 2j + 1) at dwords j + 2 and the pairs at columns -3 / +3 (odd
// elements) as one v_alignbyte each; rows -3 / +3 are two 8-byte reads each.  No byte unpacking.
typedef const uint32_t __attribute__((address_space(3))) lds_cu32;
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef const u32x2_t __attribute__((address_space(3))) lds_cu32x2;
typedef const uint32x4_t __attribute__((address_space(3))) lds_cu32x4;

template <int TQ>   // the tile's high bytes are 0 here (pass 1 clears pass 0's arc strengths first)
__device__ __forceinline__ uint32_t prefilter16(lds_cu32* w, uint32_t tt) {   // w: element dy * TQ + x0
    static_assert(TQ % 8 == 0, "tile rows must keep 16-byte alignment");
    const uint32x4_t c0 = *(lds_cu32x4*)(w + 3 * TQ / 2), c1 = *(lds_cu32x4*)(w + 3 * TQ / 2 + 4);
    // rows +3 / -3: four 8-byte reads (volatile: merged into ds_read2_b64 they would take 8 LDS cycles
    // instead of 2 x 2)
    const u32x2_t p0 = *(volatile lds_cu32x2*)(w + 6 * TQ / 2 + 2), p1 = *(volatile lds_cu32x2*)(w + 6 * TQ / 2 + 4);
    const u32x2_t m0 = *(volatile lds_cu32x2*)(w + 2), m1 = *(volatile lds_cu32x2*)(w + 4);
    uint32_t D[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    uint32_t P[4] = {p0[0], p0[1], p1[0], p1[1]}, M[4] = {m0[0], m0[1], m1[0], m1[1]};
    uint32_t r[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t P12 = __builtin_amdgcn_alignbyte(D[j + 1], D[j], 2);   // column -3
        const uint32_t P4 = __builtin_amdgcn_alignbyte(D[j + 4], D[j + 3], 2);  // column +3
        r[j] = compass2(D[j + 2], P[j], P4, M[j], P12, tt);
    }
    // sign bits 15 / 31 of r[j] are pixels 2j / 2j + 1: gather the high bytes (one v_perm per two
    // results), put pixel i and i+4 in byte i's bits 0 and 4, and weight the four bytes by 1, 2, 4, 8
    // with one v_dot4 (a 32-bit multiply is quarter rate)
    const uint32_t X = __builtin_amdgcn_perm(r[1], r[0], 0x07050301u);
    const uint32_t Y = __builtin_amdgcn_perm(r[3], r[2], 0x07050301u);
    const uint32_t Z = ((X >> 7) & 0x01010101u) | ((Y >> 3) & 0x10101010u);
    return __builtin_amdgcn_udot4(Z, 0x08040201u, 0u, false);
}

// Stage 1 of a cell at threshold tt: the prefilter over every domain row, survivors compacted into
// sList in raster order (one wave prefix sum of the per-lane counts per row round, then each lane
// writes its entries at its offset).  Returns the list length.
template <int TQ>
__device__ __forceinline__ int prefilter_cell(const uint32_t* t32, int dh, int rpi, int lrow, bool lane_on, int x0,
                                              uint32_t xvalid, uint32_t tt, uint16_t* sList) {
    int nlist = 0;
    for (int r0 = 0; r0 < dh; r0 += rpi) {
        const int dy = r0 + lrow;
        int pm = 0;
        if (lane_on && dy < dh) {
            // one VGPR address per row round (the asm keeps the compiler from re-deriving it per load)
            lds_cu32* w = (lds_cu32*)(t32 + r0 * (TQ / 2));
            asm volatile("" : "+v"(w));
            pm = (int)((prefilter16<TQ>(w, tt) | (prefilter16<TQ>(w + 4, tt) << 8)) & xvalid);
        }
        const int cnt = __popc(pm);
        const int incl = wave_incl_scan(cnt);
        int pos = nlist + incl - cnt;
        // entries are the pixels' byte offsets in the tile from domain pixel (0, 0): dy * 2TQ + 2x
        const int base = dy * (2 * TQ) + 2 * x0;
        // one iteration per set bit (survivors are sparse: the wave runs max-popcount iterations)
        for (uint32_t b = (uint32_t)pm; b; b &= b - 1) sList[pos++] = (uint16_t)(base + 2 * __builtin_ctz(b));
        nlist += __builtin_amdgcn_readlane(incl, 63);
    }
    return nlist;
}

// One cell after its ROI is in the tile: prefilter, exact arc strength, cell-local NMS with the
// minThFAST fallback, raster-order emission (see k_fast above for the semantics).  The arc strength M
// of a scored pixel is kept in the high byte of its tile element (pixels are < 256, and the widening
// store leaves every high byte 0), so the NMS reads neighbours' M from the tile: no separate map to
// clear, and unscored pixels read 0.
template <int TQ, int CP = 0>
__device__ __forceinline__ void fast_cell_body(const Geom* __restrict__ g, const FastCellT& c, int lane,
                                               uint16_t* tile, uint16_t* sList,
                                               uint32_t* __restrict__ cands, uint32_t* __restrict__ candFirst,
                                               int* cntOut, unsigned long long* __restrict__ stamps, int item) {
    constexpr int PX = 16, TB = 2 * TQ;   // PX: pixels per lane and row round; TB: tile row pitch in bytes
    constexpr unsigned kRecipTB = (1u << 20) / TB + 1;
    const int dw = c.dw, dh = c.dh;
    ORBGPU_STAMP(1);
    // lane -> (run of PX = 16 pixels, row) of the prefilter, fixed for the cell (rows advance by 64 / nruns)
    const int nruns = c.nruns;                           // (dw + PX - 1) / PX
    const int rpi = c.rpi;                               // rows per iteration, 64 / nruns
    const int lrow = (int)div20(lane, c.m_runs);
    const int x0 = PX * (lane - lrow * nruns);
    const bool lane_on = lrow < rpi;
    const uint32_t xvalid = x0 + PX <= dw ? (1u << PX) - 1u : (1u << max(dw - x0, 0)) - 1u;
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tile) + ((lrow * TQ + x0) >> 1);   // row step TQ / 2
    uint8_t* t0 = reinterpret_cast<uint8_t*>(&tile[3 * TQ + 4]);   // domain pixel (0, 0), low byte
    // Pass 0 runs the whole cell at iniThFAST; only a cell left with no keypoint (:812-816) runs pass 1
    // at minThFAST.  The prefilter is a necessary condition for M > th at the pass threshold, so a
    // pass only scores the pixels that can matter at its threshold, and only its corners (M > th) are
    // written to the map: everything else reads 0 (M <= th counts 0 in the NMS).  Before pass 1 the
    // pass-0 corners (the list NMS ran over) are cleared, so its prefilter reads clean pixel pairs.
    int th = g->iniTh;
    int kept = 0;
    for (int pass = 0; pass < 2; pass++) {
        // ---- stage 1: compass prefilter at th, 8 pixels per lane as 16-bit pixel pairs, survivors
        // compacted into sList by one wave scan
        const uint32_t tt = (uint32_t)th | ((uint32_t)th << 16);
        const int nlist = prefilter_cell<TQ>(t32, dh, rpi, lrow, lane_on, x0, xvalid, tt, sList);
        wave_lds_sync();
        ORBGPU_STAMP(2);
#if defined(ORBGPU_FAST_CUT) && ORBGPU_FAST_CUT == 2
        if (lane == 0) *cntOut = nlist & 0;
        return;
#endif
        // ---- stage 2: exact arc strength for the survivors; corners at th are compacted in place
        // (each chunk is read into registers before any lane writes, and writes land at or before it)
        int ncorner = 0;
        for (int b0 = 0; b0 < nlist; b0 += 64) {
            const int i = b0 + lane;
            int p = 0, m = 0;
            if (i < nlist) {
                p = sList[i];
                m = fast_arc_strength<TB, 2>(t0 + p);
            }
            const bool corner = m > th;
            const unsigned long long cm = __ballot(corner);
            if (corner) {
                t0[p + 1] = (uint8_t)m;
                sList[ncorner + lanes_below(cm)] = (uint16_t)p;
            }
            ncorner += __popcll(cm);
        }
        wave_lds_sync();
        ORBGPU_STAMP(3);
#if defined(ORBGPU_FAST_CUT) && ORBGPU_FAST_CUT == 3
        if (lane == 0) *cntOut = ncorner & 0;
        return;
#endif
        // ---- cell-local NMS at th.  Neighbours outside the domain are ROI border pixels (M = 0);
        // M <= th counts 0.  The corner list is in raster order (the prefilter compacts rows in order, pixels
        // ascending within a lane's run, runs in lane order), so the kept corners are emitted as they
        // are found: one ballot compaction per chunk of 64, FAST emission order.
        kept = 0;
        for (int b0 = 0; b0 < ncorner; b0 += 64) {
            const int i = b0 + lane;
            bool k = false;
            uint32_t packed = 0;
            if (i < ncorner) {
                const int p = sList[i];
                const uint8_t* q = t0 + p + 1;
                const int m = q[0];
                const int s = m - 1;
                // the reference keeps score s = M - 1 iff s > sn for every neighbour, sn = Mn - 1 for a
                // corner neighbour (Mn > th) and 0 otherwise.  A neighbour with Mn <= th < M is below M
                // anyway, so this is M > max(every Mn, 1)
                const int n0 = max(max((int)q[-TB - 2], (int)q[-TB]), (int)q[-TB + 2]);
                const int n1 = max(max((int)q[-2], (int)q[2]), 1);
                const int n2 = max(max((int)q[TB - 2], (int)q[TB]), (int)q[TB + 2]);
                k = m > max(max(n0, n1), n2);
                // (x, y) from the byte offset: y = p / TB by a 20-bit reciprocal (exact for even p < 2^15 at
                // TB = 96 or 160; a tile holds hCell + 6 rows, about 40), x = (p - y TB) / 2
                const int py = (int)(__umul24((unsigned)p, kRecipTB) >> 20), px = (p - py * TB) >> 1;
                packed = (uint32_t)(px + c.xo) | ((uint32_t)(py + c.yo) << 12) | ((uint32_t)s << 24);
            }
            // a cell's first kCandFirst corners go to its dense record after the count (the octree reads most
            // cells' count and corners with two coalesced 16-byte loads), the rest to its slots
            const unsigned long long km = __ballot(k);
            const int slot = kept + lanes_below(km);
            if (k) {
                if constexpr (CP != 0) {
                    uint32_t* dst = slot < kCandFirst ? &candFirst[((long long)c.f * g->ncells + c.cell) * kCandRec + 1 + slot]
                                                      : &cands[(long long)c.f * g->ncand + c.out_off + slot];
                    __hip_atomic_store(dst, packed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    if (slot < kCandFirst) candFirst[((long long)c.f * g->ncells + c.cell) * kCandRec + 1 + slot] = packed;
                    else cands[(long long)c.f * g->ncand + c.out_off + slot] = packed;
                }
            }
            kept += __popcll(km);
        }
        if (kept > 0 || th == g->minTh) break;
        th = g->minTh;   // nothing kept: nothing was emitted
        for (int i = lane; i < ncorner; i += 64) t0[sList[i] + 1] = 0;   // pass 0's map entries
        wave_lds_sync();
    }
    ORBGPU_STAMP(4);
    if (lane == 0) {
        if constexpr (CP != 0) __hip_atomic_store(cntOut, kept, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *cntOut = kept;
    }
    ORBGPU_STAMP(5);
}

/* Wave-per-cell form of the same algorithm: a wavefront owns two consecutive (frame, cell) items
 * (four waves, eight cells per block), so every synchronisation is a wave barrier; the second
 * cell's ROI loads are issued before the first cell is processed, hiding their latency.  The
 * per-wave LDS carve is sized on the host from the level grids (Geom::fast_*).  Prefilter survivors
 * are compacted by one wave scan into a raster-ordered list, so corners keep that order and the NMS
 * pass emits the kept ones directly (FAST emission order) by ballot compaction. */
template <int TQ>
__global__ __launch_bounds__(256) void k_fast_wave(const Geom* __restrict__ g, const CellDesc* __restrict__ cells,
                                                   const uint8_t* __restrict__ frames,
                                                   long long framePitch, int rowStride, const uint8_t* __restrict__ pyr,
                                                   uint32_t* __restrict__ cands, uint32_t* __restrict__ candFirst,
                                                   int total,
                                                   int cbeg, int cnum, unsigned long long* __restrict__ stamps,
                                                   int* __restrict__ err, int ipw) {
    extern __shared__ __attribute__((aligned(16))) int smem_fast[];
    uint8_t* smem = reinterpret_cast<uint8_t*>(smem_fast);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave-uniform: SALU
    // blocks dealt round-robin over the 8 XCDs: give each XCD a contiguous range of blocks (8 cells each)
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int blk = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    const int item0 = (blk * (int)(blockDim.x >> 6) + wv) * ipw;   // ipw = items per wave, 2 (1 for latency)
    if (item0 >= total) return;   // whole wave; nothing below uses a block barrier
    const int wb = g->fast_wave_bytes;
    // 16-bit pixel tile, TQ per row, after a 16-byte lead pad (fast_roi_store's dword -1 of row 0)
    uint16_t* tile = reinterpret_cast<uint16_t*>(smem + (size_t)wv * wb + 16);
    uint16_t* sList = reinterpret_cast<uint16_t*>(smem + (size_t)wv * wb + ((g->fast_rows * TQ * 2 + 32 + 15) & ~15));
    const bool has1 = ipw == 2 && item0 + 1 < total;
    const FastCellT c0 = fast_cell_t(g, cells, item0, frames, framePitch, rowStride, pyr, cbeg, cnum);
    const FastCellT c1 = fast_cell_t(g, cells, has1 ? item0 + 1 : item0, frames, framePitch, rowStride, pyr, cbeg, cnum);
    uint32_t v0[8], v1[8];
    if (c0.valid && c0.aligned) fast_roi_issue(c0, lane, v0);
    if (has1 && c1.valid && c1.aligned) fast_roi_issue(c1, lane, v1);
    if (err && blockIdx.x == 0 && threadIdx.x == 0) {   // k_octree's overflow flag (set after this kernel)
        err[0] = 0;
        if (cnum == g->ncells) err[1] = 0;   // a launch over every level also clears the forked branch's flag
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (k == 1 && !has1) break;
        const FastCellT& c = k == 0 ? c0 : c1;
        const int item = item0 + k;
        int* cntOut = reinterpret_cast<int*>(candFirst + ((long long)c.f * g->ncells + c.cell) * kCandRec);   // record[0]
        if (!c.valid) {
            if (lane == 0) *cntOut = 0;
            continue;
        }
        ORBGPU_STAMP(0);
        wave_lds_sync();   // the previous cell's last LDS reads happen before this one's writes
        fast_roi_store<TQ>(c, lane, k == 0 ? v0 : v1, tile);
        ORBGPU_STAMP(6);
#if defined(ORBGPU_FAST_CUT) && ORBGPU_FAST_CUT == 1   // instruction-count diagnostics only (tools/diag_cut.sh)
        wave_lds_sync();
        if (lane == 0) *cntOut = (int)tile[lane] & 0;
        continue;
#endif
        fast_cell_body<TQ>(g, c, lane, tile, sList, cands, candFirst, cntOut, stamps, item);
    }
}

// Per-wave LDS carve of k_fast_wave.  Cells at most 36 px wide (every BASELINE config) use the
// compact tile pitch of 48 elements, wider ones 80: a tile row holds the
// widened ROI (rw + 2 elements) and an unused tail for the next row's dword -1, a multiple of 8 elements
// (16-byte reads), with row strides of 24 / 40 dwords (2-way LDS bank conflicts at most for the
// prefilter's 16- and 8-byte reads).
// Prefilter windows of pixels past the domain may read into the next row: those bits are masked.
void fast_wave_layout(Geom& g) {
    int rows = 1, drows = 1, list = 1, maxw = 1;
    for (int l = 0; l < g.nlevels; l++) {
        const LevelGeom& L = g.L[l];
        rows = std::max(rows, L.hCell + 6);
        drows = std::max(drows, L.hCell);
        list = std::max(list, L.hCell * L.wCell);
        maxw = std::max(maxw, L.wCell);
    }
    g.fast_rows = rows;
    g.fast_drows = drows;
    g.fast_list = list;
    g.fast_compact = maxw <= 36 ? 1 : 0;
    const int tq = g.fast_compact ? 48 : kFastTilePitch;
    g.fast_wave_bytes = ((rows * tq * 2 + 32 + 15) & ~15) + ((list * 2 + 15) & ~15);
    g.fast_wave_bytes = (g.fast_wave_bytes + 15) & ~15;
}

/* ------------------------------------------------------------------------------------------------
 * DistributeOctTree (ORBextractor.cc:539-763) — one workgroup per (level, frame).
 *
 * The reference's std::list of ExtractorNodes is kept as a node TABLE IN LIST ORDER in LDS; keys
 * (the FAST candidates, in vToDistributeKeys order) stay in a per-level global scratch with a node
 * index each.  A round divides a set of nodes; children are pushed to the list front in
 * processing order (n1..n4), so the new table is
 *     [children of the last-processed node (n4..n1)] ... [children of the first] [unprocessed nodes].
 * Phase 1 (:594-665) processes every node with > 1 key in list order; phase 2 (:676-737) sorts the
 * > 1-key nodes by (size, creation sequence) — the pinned stand-in for the pair's heap pointer
 * (:684) — and divides from the largest down, stopping as soon as the list reaches N nodes (:730).
 * Finally each node keeps its max-response key, first in key order on ties (:741-762).
 * --------------------------------------------------------------------------------------------- */
__device__ __forceinline__ int quadrant_of(uint32_t key, uint32_t rx, uint32_t ry) {
    const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
    const int x0 = rx & 0xFFFF, x1 = rx >> 16, y0 = ry & 0xFFFF, y1 = ry >> 16;
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;   // ceil((float)w/2) (:483-484)
    return (x >= x0 + hx ? 1 : 0) | (y >= y0 + hy ? 2 : 0);     // n1 TL, n2 TR, n3 BL, n4 BR (:512-526)
}

__device__ __forceinline__ void child_rect(uint32_t rx, uint32_t ry, int q, uint32_t& crx, uint32_t& cry) {
    const int x0 = rx & 0xFFFF, x1 = rx >> 16, y0 = ry & 0xFFFF, y1 = ry >> 16;
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
    const int xm = x0 + hx, ym = y0 + hy;
    const int cx0 = (q & 1) ? xm : x0, cx1 = (q & 1) ? x1 : xm;
    const int cy0 = (q & 2) ? ym : y0, cy1 = (q & 2) ? y1 : ym;
    crx = (uint32_t)cx0 | ((uint32_t)cx1 << 16);
    cry = (uint32_t)cy0 | ((uint32_t)cy1 << 16);
}

// The thread index as the octree code reads it: threadIdx.x, or (CP != 0: inside k_extract_flow's task loop) the
// same value through an opaque move, so that nothing derived from it is hoisted out of the loop and held live
// across every task (which pushed the octree from 101 to 128 VGPRs with spills)
template <int CP>
__device__ __forceinline__ int tidx() {
    if constexpr (CP == 0) return threadIdx.x;
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
    return t;
}

// Exclusive scan over the k_octree block with one barrier: wave totals go to one of two 16-int
// buffers (`par` flips on every call, which every thread makes in the same order), and every thread
// adds the totals of the waves before its own.  The buffer written by call k+2 was last read in
// call k, before every thread reached call k+1's barrier, so no trailing barrier is needed.
template <int NT, int CP = 0>   // NT: the k_octree block size
__device__ __forceinline__ int oct_scan(int v, int* sc, int& par, int& total) {
    constexpr int NW = NT / 64;
    const int lane = tidx<CP>() & 63, wave = tidx<CP>() >> 6;
    const int x = wave_incl_scan(v);
    int* buf = sc + 16 * par;
    par ^= 1;
    if (lane == 63) buf[wave] = x;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const int t = buf[i];
        pre += i < wave ? t : 0;
        tot += t;
    }
    total = tot;
    return pre + x - v;
}

// Wave-aggregated LDS counter add: one atomic per distinct target in the wave (LDS atomics from many
// lanes to one address serialise at ~2 cycles per lane).  Uniform control flow required.
template <int CP = 0>
__device__ __forceinline__ void wave_agg_add(int* ctr, bool ok, int tgt) {
    unsigned long long pending = __ballot(ok);
    while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const int tl = __builtin_amdgcn_readlane(tgt, leader);
        const unsigned long long m = __ballot(ok && tgt == tl);
        if ((int)(tidx<CP>() & 63) == leader) atomicAdd(&ctr[tl], __popcll(m));
        pending &= ~m;
    }
}

__device__ __forceinline__ int quad_mask(const int* qd) {
    return (qd[0] > 0) | ((qd[1] > 0) << 1) | ((qd[2] > 0) << 2) | ((qd[3] > 0) << 3);
}

/* Phase-1 fast-forward.  Phase 1 (:594-672) divides every node with > 1 key in every round, so the
 * node set after round r is a function of the quadtree alone: the non-empty depth-r cells whose parent
 * holds >= 2 keys, plus the one-key cells of every shallower depth (bNoMore).  Its list order follows
 * from push_front (:617-652) and the in-order sweep: round r puts the children of the last-divided node
 * first, n4..n1 each, ahead of the undivided nodes in their old order, so
 *     L_r = [depth-r nodes in order_r] [one-key depth-(r-1) nodes in order_(r-1)] ... [one-key roots],
 * where order_0 sorts roots ascending and order_r = (parent's order_(r-1) reversed, quadrant descending):
 * a node's rank is its path code with the root reversed when r is odd and quadrant k reversed when
 * r - k is even (XOR 3), i.e. code ^ 0x3333... on the quadrant bits.  Creation order within round r is
 * the reverse of order_r (the next round's phase-2 tie key, :684).  So the list after R rounds is built
 * in one pass: per-key path codes to depth F, cell counts in dense per-depth tables (LDS), per-depth
 * node counts, the stop / phase-2 tests of :669-673 evaluated on those counts, and one scan over the
 * tables of depths R..0 in rank order.  The round loop then continues from round R (phase 2, or phase
 * 1 past depth F) exactly as before. */
constexpr int kFfMaxDepth = 6;

// depth F of the tables: the first depth whose cells can hold N nodes (phase 1 usually switches to phase 2
// the round before, so phase 2's first round still finds its quadrant counts in the table), at most what
// fits in `room` ints with codes in 16 bits; 0 = no fast-forward
__device__ __forceinline__ int ff_depth(int nIni, int N, int room) {
    int F = 0, tot = 0, want = kFfMaxDepth;
    for (int d = 1; d <= kFfMaxDepth; d++)
        if ((nIni << (2 * d)) >= N) {
            want = d;
            break;
        }
    for (int d = 1; d <= want && d <= kFfMaxDepth; d++) {
        const int sz = nIni << (2 * d);
        if (sz > 65536 || tot + sz > room) break;
        tot += sz;
        F = d;
    }
    return F;
}

// table offset of depth d (1..F) inside the tables area
__device__ __forceinline__ int ff_base(int nIni, int d) { return nIni * (((1 << (2 * d)) - 4) / 3); }

// One (frame, level) of DistributeOctTree once the candidate count C is known.  KeysInLds selects
// whether keys / knode live in LDS (after the node tables) or in the per-level global scratch; the
// two instantiations let the compiler use ds_* or global_* accesses instead of flat ones.
// a store of the octree's outputs (lvlKps, lvlCount): write-through sc1 in the dataflow launch (CP != 0)
template <int CP, class T>
__device__ __forceinline__ void oct_out(T* p, T v) {
    if constexpr (CP != 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

template <bool KeysInLds, int NT, int CP = 0>
__device__ __forceinline__ void octree_level(const Geom* __restrict__ g, const LevelGeom& L, int f, int l, int* smem,
                                             int C, uint32_t* keys, uint16_t* knode, uint32_t* __restrict__ lvlKps,
                                             int* __restrict__ lvlCount, int* __restrict__ err, int par,
                                             unsigned long long* __restrict__ ost) {
    const int NC = g->node_cap;
    const int tid = tidx<CP>();
    const int tieMask = (g->variant & ORB_VARIANT_TIE_REVERSE) ? 0xFFFFFF : 0;   // :684 tie policy
    // LDS carve: tables P and Q (ping-pong: A = current list, B = next), quad, rank, info, ord, nchr,
    // scan buffers, scalars.  Phase 2's dense sort keys alias B's rx/ry, its per-rank d / prefix
    // alias B's cnt/seq (all consumed before B is written).
    uint32_t* rxA = (uint32_t*)smem;
    uint32_t* ryA = rxA + NC;
    int* cntA = (int*)(ryA + NC);
    int* seqA = cntA + NC;
    uint32_t* rxB = (uint32_t*)(seqA + NC);
    uint32_t* ryB = rxB + NC;
    int* cntB = (int*)(ryB + NC);
    int* seqB = cntB + NC;
    int* quad = seqB + NC;        // 4*NC (the candidate gather's cell offsets before round 1)
    int* rank = quad + 4 * NC;    // node -> processing rank, -1 = not divided this round
    int* info = rank + NC;        // node -> new position (| child mask << 16 for divided nodes)
    int* ord = info + NC;         // rank -> node
    int* nchr = ord + NC;         // node -> children of the nodes divided before it
    int* sc = nchr + NC;          // 2 x 16 ints of scan buffers
    int* sv = sc + 32;            // scalars
#if ORBGPU_KERNEL_STAMPS
#define OCT_STAMP(k) \
    if (ost && tid == 0) ost[(k)] = __builtin_amdgcn_s_memtime();
#else
#define OCT_STAMP(k)
#endif

    // 1. the keys (vToDistributeKeys order) are in place: k_octree gathered them
    __syncthreads();
    OCT_STAMP(1);
    if (ost && tid == 0) ost[29] = (unsigned long long)C;

    // 2. root nodes (:543-585): nIni columns of the level's border-trimmed area; empty ones erased
    const int N = L.nfeat;
    const int nIni = L.nIni;
    const float hX = L.hX;
    const int Hn = L.maxBY - kMinBorder;
    if (nIni > NC) {
        if (tid == 0) { atomicOr(err, 1); oct_out<CP>(&lvlCount[f * g->nlevels + l], 0); }
        return;
    }
    int S = 0, nextSeq = 0, phase = 1, round0 = 0;
    bool ffDone = false, quadReady = false;
    const int F = C < (1 << 20) ? ff_depth(nIni, N, 8 * NC) : 0;
    if (F > 0) {
        // ---- phase-1 fast-forward (see above).  Tables: depth 0 = root counts in cntB, depths 1..F in
        // the quad..nchr area (8 NC ints); entries cnt | pos << 20 once the node is placed.
        int* T = quad;
        int* ffc = reinterpret_cast<int*>(rxB);   // per depth d: [2d] nodes, [2d + 1] nodes with > 1 key
        const int bF = ff_base(nIni, F);
        const int szF = nIni << (2 * F);
        for (int t = tid; t < szF; t += NT) T[bF + t] = 0;
        for (int t = tid; t < 2 * (kFfMaxDepth + 1); t += NT) ffc[t] = 0;
        __syncthreads();
        OCT_STAMP(12);
        // A. every key's path code down to depth F (the quadrants the rounds would send it to,
        // DivideNode :477-535: children split at ceil(w / 2), x and y independently), counted at F
        for (int i = tid; i < C; i += NT) {
            const uint32_t k = keys[i];
            const int x = k & 0xFFF, y = (k >> 12) & 0xFFF;
            const int t = min((int)((float)x / hX), nIni - 1);
            int x0 = (int)(hX * (float)t), x1 = (int)(hX * (float)(t + 1)), y0 = 0, y1 = Hn;
            int code = t;
            for (int d = 1; d <= F; d++) {
                const int xm = x0 + ((x1 - x0 + 1) >> 1), ym = y0 + ((y1 - y0 + 1) >> 1);
                const bool bx = x >= xm, by = y >= ym;
                x0 = bx ? xm : x0;
                x1 = bx ? x1 : xm;
                y0 = by ? ym : y0;
                y1 = by ? y1 : ym;
                code = code * 4 + ((int)bx | ((int)by << 1));
            }
            knode[i] = (uint16_t)code;
            atomicAdd(&T[bF + code], 1);
        }
        __syncthreads();
        OCT_STAMP(13);
        // B. the shallower depths' counts (sums of four children), and per depth the node counts: a
        // non-empty cell whose parent holds >= 2 keys is a node (and divisible if it holds >= 2)
        for (int d = F - 1; d >= 0; d--) {
            const int sz = d == 0 ? nIni : nIni << (2 * d);
            int* td = d == 0 ? cntB : T + ff_base(nIni, d);
            const int* tc = T + ff_base(nIni, d + 1);
            int dn = 0, en = 0, d0 = 0, e0 = 0;
            for (int c = tid; c < sz; c += NT) {
                const int4 ch = *reinterpret_cast<const int4*>(&tc[4 * c]);
                const int pc = ch.x + ch.y + ch.z + ch.w;
                td[c] = pc;
                if (pc >= 2) {
                    dn += (ch.x > 0) + (ch.y > 0) + (ch.z > 0) + (ch.w > 0);
                    en += (ch.x > 1) + (ch.y > 1) + (ch.z > 1) + (ch.w > 1);
                }
                d0 += pc > 0;
                e0 += pc > 1;
            }
            dn = wave_sum(dn);
            en = wave_sum(en);
            if ((tidx<CP>() & 63) == 0 && (dn | en)) {
                atomicAdd(&ffc[2 * (d + 1)], dn);
                atomicAdd(&ffc[2 * (d + 1) + 1], en);
            }
            if (d == 0) {   // the roots themselves (erased when empty, :577-588)
                d0 = wave_sum(d0);
                e0 = wave_sum(e0);
                if ((tidx<CP>() & 63) == 0 && (d0 | e0)) {
                    atomicAdd(&ffc[0], d0);
                    atomicAdd(&ffc[1], e0);
                }
            }
            __syncthreads();
        }
        OCT_STAMP(14);
        // C. the rounds' size bookkeeping on the counts (:600, :669-673), identical in every thread
        int Sr = ffc[0], Eprev = ffc[1], R = 0, base = 0, nseq = 0;
        bool fin = false, ph2 = false, over = false;
        for (int r = 1; r <= F; r++) {
            const int Dr = ffc[2 * r], Er = ffc[2 * r + 1];
            const int prev = Sr;
            Sr = Sr - Eprev + Dr;
            base = nseq;
            nseq += Dr;
            R = r;
            if (Sr > NC) { over = true; break; }
            if (Sr >= N || Sr == prev) { fin = true; break; }
            if (Sr + Er * 3 > N) { ph2 = true; break; }
            Eprev = Er;
        }
        if (over) {
            if (tid == 0) { atomicOr(err, 2); oct_out<CP>(&lvlCount[f * g->nlevels + l], 0); }
            return;
        }
        const int DR = ffc[2 * R];
        // D. the list after round R: one scan over the tables [depth R] [depth R-1] ... [roots], each
        // in rank order, flagging depth R's nodes and the shallower one-key nodes
        int V = 0;
        for (int d = R; d >= 0; d--) V += d == 0 ? nIni : nIni << (2 * d);
        OCT_STAMP(15);
        int run = 0;
        for (int v0 = 0; v0 < V; v0 += NT) {   // uniform trip count (the scan)
            const int v = v0 + tid;
            int c = 0, n = 0, d = 0;
            bool on = false;
            int* td = cntB;
            if (v < V) {
                int off = 0;
                d = R;
                for (;;) {
                    const int sz = d == 0 ? nIni : nIni << (2 * d);
                    if (v < off + sz) break;
                    off += sz;
                    d--;
                }
                const int p = v - off;
                const int lowMask = (1 << (2 * d)) - 1;
                const int rt = p >> (2 * d);
                // rank -> cell: root reversed for odd d, quadrant k reversed where d - k is even
                c = (((d & 1) ? nIni - 1 - rt : rt) << (2 * d)) | ((p & lowMask) ^ (0x33333333 & lowMask));
                td = d == 0 ? cntB : T + ff_base(nIni, d);
                n = td[c] & 0xFFFFF;
                const int* ptab = d == 1 ? cntB : T + ff_base(nIni, d > 1 ? d - 1 : 1);
                const bool node = n > 0 && (d == 0 || (ptab[c >> 2] & 0xFFFFF) >= 2);
                on = node && (d == R || n == 1);
            }
            int tot;
            const int pos = run + oct_scan<NT, CP>(on ? 1 : 0, sc, par, tot);
            if (on) {
                const int t = c >> (2 * d);
                int x0 = (int)(hX * (float)t), x1 = (int)(hX * (float)(t + 1)), y0 = 0, y1 = Hn;
                for (int k2 = d - 1; k2 >= 0; k2--) {
                    const int q = (c >> (2 * k2)) & 3;
                    const int xm = x0 + ((x1 - x0 + 1) >> 1), ym = y0 + ((y1 - y0 + 1) >> 1);
                    x0 = (q & 1) ? xm : x0;
                    x1 = (q & 1) ? x1 : xm;
                    y0 = (q & 2) ? ym : y0;
                    y1 = (q & 2) ? y1 : ym;
                }
                rxA[pos] = (uint32_t)x0 | ((uint32_t)x1 << 16);
                ryA[pos] = (uint32_t)y0 | ((uint32_t)y1 << 16);
                cntA[pos] = n;
                // creation order in round R is the reverse of the rank (phase 2's tie key, :684); the
                // one-key nodes are never divided and their seq is never read
                seqA[pos] = d == 0 ? -1 - t : d == R ? base + DR - 1 - pos : base;
                td[c] = n | (pos << 20);
                if (d == R) ryB[pos] = (uint32_t)c;   // the node's depth-R cell (phase 2's quadrant counts)
            }
            run += tot;
        }
        __syncthreads();
        OCT_STAMP(16);
        // E. each key's node: its first one-key ancestor, else its depth-R cell
        for (int i = tid; i < C; i += NT) {
            const int code = knode[i];
            int node = 0;
            for (int d = 0; d <= R; d++) {
                const int c = code >> (2 * (F - d));
                const int e = d == 0 ? cntB[c] : T[ff_base(nIni, d) + c];
                if (d == R || (e & 0xFFFFF) == 1) {
                    node = e >> 20;
                    break;
                }
            }
            knode[i] = (uint16_t)node;
        }
        // phase 2 starts at round R + 1 and divides depth-R nodes: their quadrant counts are the depth-(R+1)
        // table's, so its first round needs no pass over the keys (read here, written once every read of
        // the tables is done: quad aliases them)
        if (ph2 && R + 1 <= F) {
            constexpr int kMaxPer = 8;   // node_cap <= 8 * NT (host: octree_lds_bytes <= 160 KiB)
            int4 qv[kMaxPer];
            const int* tq = T + ff_base(nIni, R + 1);
#pragma unroll
            for (int j = 0; j < kMaxPer; j++) {
                const int pos = tid + j * NT;
                qv[j] = make_int4(0, 0, 0, 0);
                if (pos < run && pos < DR && cntA[pos] >= 2) qv[j] = *reinterpret_cast<const int4*>(&tq[4 * (int)ryB[pos]]);
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kMaxPer; j++) {
                const int pos = tid + j * NT;
                if (pos < run) *reinterpret_cast<int4*>(&quad[4 * pos]) = qv[j];
            }
            quadReady = true;
        }
        S = run;
        nextSeq = nseq;
        round0 = R;
        ffDone = fin;
        if (ph2) phase = 2;
    } else {
        for (int t = tid; t < nIni; t += NT) cntB[t] = 0;
        __syncthreads();
        for (int i0 = 0; i0 < C; i0 += NT) {   // uniform trip count: the ballots need the whole wave
            const int i = i0 + tid;
            const bool ok = i < C;
            int r = 0;
            if (ok) {
                const int x = keys[i] & 0xFFF;
                r = min((int)((float)x / hX), nIni - 1);
                knode[i] = (uint16_t)r;
            }
            wave_agg_add<CP>(cntB, ok, r);   // the roots are few: a wave's keys usually share one or two
        }
        __syncthreads();
        for (int t0 = 0; t0 < nIni; t0 += NT) {   // keep the non-empty roots in order
            const int t = t0 + tid;
            const int n = t < nIni ? cntB[t] : 0;
            int tot;
            const int pos = S + oct_scan<NT, CP>(n > 0 ? 1 : 0, sc, par, tot);
            if (n > 0) {
                const int x0 = (int)(hX * (float)t), x1 = (int)(hX * (float)(t + 1));
                rxA[pos] = (uint32_t)x0 | ((uint32_t)x1 << 16);
                ryA[pos] = (uint32_t)Hn << 16;
                cntA[pos] = n;
                seqA[pos] = -1 - t;
            }
            if (t < nIni) info[t] = pos;
            S += tot;
        }
        __syncthreads();
        for (int i = tid; i < C; i += NT) knode[i] = (uint16_t)info[knode[i]];
    }
    if (tid == 0) sv[3] = 0;
    __syncthreads();
    OCT_STAMP(2);

    for (int round = round0; round < 4 * NC + 64 && !ffDone; round++) {
        const int prevSize = S;
        // sub-step stamps of round 0 (slots 12..16) and of the last phase-2 round (20..28)
        [[maybe_unused]] const int subBase = round == 0 ? 12 : phase == 2 ? 20 : -1;   // (the last phase-2 round's)
#if ORBGPU_KERNEL_STAMPS
#define OCT_SUB(k) \
    if (ost && tid == 0 && subBase >= 0 && subBase + (k) < 29) ost[subBase + (k)] = __builtin_amdgcn_s_memtime();
#else
#define OCT_SUB(k)
#endif
        if (!quadReady) for (int t = tid; t < 4 * S; t += NT) quad[t] = 0;
        for (int t = tid; t < S; t += NT) rank[t] = -1;
        __syncthreads();
        OCT_SUB(0);
        for (int i0 = 0; i0 < (quadReady ? 0 : C); i0 += 4 * NT) {   // 4 keys per thread, branch-free reads (clamped)
            int tt[4], tg[4];
            uint32_t kk[4];
            bool inc[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int ic = min(i0 + u * NT + tid, C - 1);
                tt[u] = knode[ic];
                kk[u] = keys[ic];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = tt[u];
                inc[u] = i0 + u * NT + tid < C && cntA[t] > 1;
                tg[u] = 4 * t + quadrant_of(kk[u], rxA[t], ryA[t]);
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (inc[u]) atomicAdd(&quad[tg[u]], 1);
        }
        if (tid == 0) sv[4] = 0;   // (phase 2's oversize-bin count)
        __syncthreads();
        OCT_SUB(1);
        quadReady = false;
        int CH = 0, ndiv = 0;   // children created / nodes divided this round
        if (phase == 1) {
            // every node with > 1 key, in list order: one scan of (divided, #children) packed 16:16;
            // rank / children-before are written for the node's own thread (same mapping below)
            int nproc = 0;
            for (int t0 = 0; t0 < S; t0 += NT) {
                const int t = t0 + tid;
                int val = 0, mask = 0;
                if (t < S && cntA[t] > 1) {
                    mask = quad_mask(&quad[4 * t]);
                    val = 1 | (__popc(mask) << 16);
                }
                int tot;
                const int pre = oct_scan<NT, CP>(val, sc, par, tot);
                if (t < S) {
                    if (val) {
                        rank[t] = nproc + (pre & 0xFFFF);
                        nchr[t] = CH + (pre >> 16);
                        info[t] = mask << 16;
                    } else {
                        info[t] = t - nproc - (pre & 0xFFFF);   // index among the undivided nodes
                    }
                }
                nproc += tot & 0xFFFF;
                CH += tot >> 16;
            }
            ndiv = nproc;
            OCT_SUB(2);
        } else {
            // sort the > 1-key nodes by (size, seq) descending (:684-685).  The list holds the > 1-key nodes in
            // descending creation order (the roots ascending, then every round puts the last-created children first,
            // n4..n1, ahead of the older nodes: phase-1 fast-forward and rounds alike), so seq order is list order,
            // reversed under ORB_VARIANT_TIE_REVERSE, and the sort is a stable counting sort by size over the list:
            // rank = (nodes with a larger size) + (nodes of the same size earlier in that order).  Sizes below
            // kRkV - 1 have exact bins; the few larger nodes share the last bin and are ranked pairwise by (size,
            // order).  (node tables too small for the bin table: the pairwise rank of all keys, below)
            int* dd = cntB;     // rank -> #children - 1
            int* dpre = seqB;   // rank -> exclusive prefix of dd
            int nsort = 0;
            constexpr int kRkV = 32, NWv = NT / 64;   // size bins; waves
            const bool binned = 2 * NC >= kRkV * 16 && NC >= kRkV;
            if (binned) {
                int* T2 = reinterpret_cast<int*>(rxB);   // [bin][wave] counts, then their per-bin exclusive wave prefixes
                int* HV = seqB;                          // [bin] totals
                int* ovl = nchr;                         // the oversize bin's nodes (nchr is rewritten before it is read)
                const int lane = tid & 63, wave = tid >> 6;
                const bool rev = tieMask != 0;
                // 1. per wave, over its own contiguous run of the (tie-)ordered list: each node's position among the
                // earlier nodes of its bin in that run, and the run's bin counts (no barrier inside a wave)
                if (lane < kRkV) T2[lane * 16 + wave] = 0;   // (sv[4], the oversize count, was zeroed before the last barrier)
                const int PW = (S + NWv - 1) / NWv;
                const unsigned long long below = (1ull << lane) - 1ull;
                for (int c0 = wave * PW; c0 < min(S, (wave + 1) * PW); c0 += 64) {   // wave-uniform
                    const int pidx = c0 + lane;
                    const bool in = pidx < min(S, (wave + 1) * PW);
                    const int t = rev ? S - 1 - pidx : pidx;
                    const int cnt = in ? cntA[t] : 0;
                    const bool bg = cnt > 1;
                    const int v = min(cnt, kRkV - 1);
                    // the lanes holding this lane's bin: five bit-plane ballots, no loop
                    unsigned long long m = __ballot(bg);
#pragma unroll
                    for (int b = 0; b < 5; b++) {
                        const unsigned long long bal = __ballot((v >> b) & 1);
                        m &= ((v >> b) & 1) ? bal : ~bal;
                    }
                    // the run's earlier chunks of this bin, then this chunk's count added by the bin's lowest lane
                    const int prev = bg ? T2[v * 16 + wave] : 0;
                    __builtin_amdgcn_wave_barrier();
                    if (bg && (m & below) == 0) T2[v * 16 + wave] = prev + __popcll(m);
                    wave_lds_sync();
                    if (bg) {
                        info[t] = prev + __popcll(m & below);   // (info is rewritten for every node below)
                        if (v == kRkV - 1) ovl[atomicAdd(&sv[4], 1)] = t;
                    }
                }
                __syncthreads();
                // 2. per bin, the exclusive prefix of its wave counts (a 16-lane DPP row per bin) and its total
                for (int i = tid; i < kRkV * 16; i += NT) {   // (whole waves: NT is a multiple of 64)
                    const int x = (i & 15) < NWv ? T2[i] : 0;
                    int y = x;
                    y += __builtin_amdgcn_update_dpp(0, y, 0x111, 0xf, 0xf, true);
                    y += __builtin_amdgcn_update_dpp(0, y, 0x112, 0xf, 0xf, true);
                    y += __builtin_amdgcn_update_dpp(0, y, 0x114, 0xf, 0xf, true);
                    y += __builtin_amdgcn_update_dpp(0, y, 0x118, 0xf, 0xf, true);
                    T2[i] = y - x;
                    if ((i & 15) == 15) HV[i >> 4] = y;
                }
                __syncthreads();
                // 3. ranks: larger bins' totals + the wave prefix of the node's bin + its position in its wave's run
#pragma unroll 1
                for (int i = 0; i < kRkV; i += 4) {
                    const int4 h = *reinterpret_cast<const int4*>(&HV[i]);
                    nsort += h.x + h.y + h.z + h.w;
                }
                const int nov = sv[4];
                for (int t = tid; t < S; t += NT) {
                    const int cnt = cntA[t];
                    if (cnt <= 1) continue;
                    const int v = min(cnt, kRkV - 1);
                    const int pidx = rev ? S - 1 - t : t;
                    int r = 0;
                    if (v < kRkV - 1) {
                        r = info[t] + T2[v * 16 + pidx / PW];
#pragma unroll 1
                        for (int i = (v + 1) & ~3; i < kRkV; i += 4) {
                            const int4 h = *reinterpret_cast<const int4*>(&HV[i]);
                            r += (i > v ? h.x : 0) + (i + 1 > v ? h.y : 0) + (i + 2 > v ? h.z : 0) + (i + 3 > v ? h.w : 0);
                        }
                    } else {   // the oversize bin: pairwise by (size desc, then order)
                        for (int i = 0; i < nov; i++) {
                            const int u = ovl[i];
                            const int cu = cntA[u], pu = rev ? S - 1 - u : u;
                            r += cu > cnt || (cu == cnt && pu < pidx);
                        }
                    }
                    ord[r] = t;
                    dd[r] = __popc(quad_mask(&quad[4 * t])) - 1;
                }
                if (tid == 0) sv[2] = nsort;
                OCT_SUB(2);
            } else {
                unsigned long long* skey = reinterpret_cast<unsigned long long*>(rxB);
                for (int t0 = 0; t0 < S; t0 += NT) {
                    const int t = t0 + tid;
                    const bool big = t < S && cntA[t] > 1;
                    int tot;
                    const int pos = nsort + oct_scan<NT, CP>(big ? 1 : 0, sc, par, tot);
                    // seq in 24 bits: creation order, or its complement for ORB_VARIANT_TIE_REVERSE (a later-
                    // created node counts as the smaller pointer); roots (seq < 0) never reach this sort
                    if (big)
                        skey[pos] = ((unsigned long long)cntA[t] << 40) |
                                    ((unsigned long long)((unsigned)(seqA[t] ^ tieMask) & 0xFFFFFFu) << 16) |
                                    (unsigned long long)t;
                    nsort += tot;
                }
                if (tid == 0) sv[2] = nsort;
                __syncthreads();
                OCT_SUB(2);
                // G lanes per key (G = 8, 4, 2 or 1 so that the keys fill the block), each comparing a
                // strided 8-key slice, summed with xor shuffles inside the lane group
                const int G = nsort <= NT / 8 ? 8 : nsort <= NT / 4 ? 4 : nsort <= NT / 2 ? 2 : 1;
                const int lg = tid & (G - 1);
                for (int j0 = 0; j0 < nsort * G; j0 += NT) {   // uniform trip count (shuffles below)
                    const int j = (j0 + tid) / G;
                    const bool ok = j < nsort;
                    const unsigned long long key = ok ? skey[j] : ~0ull;
                    int r = 0;
                    for (int i = 8 * lg; i + 8 <= nsort; i += 8 * G) {
                        const ulonglong2* p = reinterpret_cast<const ulonglong2*>(skey + i);
                        const ulonglong2 a = p[0], b = p[1], c = p[2], d = p[3];
                        r += (a.x > key) + (a.y > key) + (b.x > key) + (b.y > key) + (c.x > key) + (c.y > key) +
                             (d.x > key) + (d.y > key);
                    }
                    if (lg == 0)
                        for (int i = nsort & ~7; i < nsort; i++) r += skey[i] > key;
                    for (int o = 1; o < G; o <<= 1) r += __shfl_xor(r, o);
                    if (ok && lg == 0) {
                        const int t = (int)(key & 0xFFFF);
                        ord[r] = t;
                        dd[r] = __popc(quad_mask(&quad[4 * t])) - 1;
                    }
                }
            }
            __syncthreads();
            OCT_SUB(3);
            // cut at N (:730): divide ranks 0..j while the list stays below N, plus the one reaching it
            int run = 0;
            for (int r0 = 0; r0 < nsort; r0 += NT) {
                const int r = r0 + tid;
                const int d = r < nsort ? dd[r] : 0;
                int tot;
                const int pre = run + oct_scan<NT, CP>(d, sc, par, tot);
                if (r < nsort) dpre[r] = pre;
                const unsigned long long fail = __ballot(r < nsort && S + pre + d >= N);
                if (fail && (tidx<CP>() & 63) == 0) atomicMin(&sv[2], r0 + (tid & ~63) + __ffsll((long long)fail) - 1);
                run += tot;
            }
            __syncthreads();
            OCT_SUB(4);
            const int first_stop = sv[2];
            const int nproc = first_stop < nsort ? first_stop + 1 : nsort;
            ndiv = nproc;
            CH = nproc > 0 ? dpre[nproc - 1] + dd[nproc - 1] + nproc : 0;
            for (int r = tid; r < nproc; r += NT) {
                const int t = ord[r];
                rank[t] = r;
                nchr[t] = dpre[r] + r;
                info[t] = quad_mask(&quad[4 * t]) << 16;
            }
            __syncthreads();
            OCT_SUB(5);
            int und = 0;
            for (int t0 = 0; t0 < S; t0 += NT) {   // index among the undivided nodes, list order
                const int t = t0 + tid;
                const bool keep = t < S && rank[t] < 0;
                int tot;
                const int pre = und + oct_scan<NT, CP>(keep ? 1 : 0, sc, par, tot);
                if (keep) info[t] = pre;
                und += tot;
            }
            OCT_SUB(6);
        }
        // new list: [children of the last-divided node (n4..n1)] ... [of the first] [undivided nodes]
        const int Snew = CH + S - ndiv;
        if (Snew > NC) {
            if (tid == 0) { atomicOr(err, 2); oct_out<CP>(&lvlCount[f * g->nlevels + l], 0); }
            return;
        }
        int big = 0;
        for (int t0 = 0; t0 < S; t0 += NT) {   // same node -> thread mapping as the scans above
            const int t = t0 + tid;
            if (t >= S) break;
            // every read first (one LDS wait), then the writes of whichever case applies
            const int rk = rank[t], inf = info[t], P = nchr[t], cnt = cntA[t], sq = seqA[t];
            const uint32_t rx = rxA[t], ry = ryA[t];
            const int4 qd = *reinterpret_cast<const int4*>(&quad[4 * t]);
            if (rk >= 0) {
                const int qc[4] = {qd.x, qd.y, qd.z, qd.w};
                const int mask = inf >> 16;
                const int start = CH - P - __popc(mask);   // later-divided nodes end up nearer the front
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (!(mask & (1 << q))) continue;
                    const int pos = start + __popc(mask >> (q + 1));          // n4 first .. n1 last
                    uint32_t crx, cry;
                    child_rect(rx, ry, q, crx, cry);
                    rxB[pos] = crx;
                    ryB[pos] = cry;
                    cntB[pos] = qc[q];
                    seqB[pos] = nextSeq + P + __popc(mask & ((1 << q) - 1));  // creation order n1..n4
                    big += qc[q] > 1;
                }
                info[t] = start | (mask << 16);
            } else {
                const int pos = CH + inf;
                rxB[pos] = rx;
                ryB[pos] = ry;
                cntB[pos] = cnt;
                seqB[pos] = sq;
                info[t] = pos;
            }
        }
        big = wave_sum(big);
        if ((tidx<CP>() & 63) == 0 && big) atomicAdd(&sv[3], big);
        __syncthreads();
        OCT_SUB(phase == 1 ? 3 : 7);
        for (int i0 = 0; i0 < C; i0 += 4 * NT) {   // 4 keys per thread, branch-free reads (clamped)
            int tt[4], nt[4];
            uint32_t kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int ic = min(i0 + u * NT + tid, C - 1);
                tt[u] = knode[ic];
                kk[u] = keys[ic];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = tt[u];
                const int inf = info[t], rk = rank[t];
                const int q = quadrant_of(kk[u], rxA[t], ryA[t]);
                nt[u] = rk >= 0 ? (inf & 0xFFFF) + __popc((inf >> 16) >> (q + 1)) : inf;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (i0 + u * NT + tid < C) knode[i0 + u * NT + tid] = (uint16_t)nt[u];
        }
        const int nToExpand = sv[3];
        __syncthreads();
        OCT_SUB(phase == 1 ? 4 : 8);
        if (tid == 0) sv[3] = 0;
        {   // B becomes the current list
            uint32_t* p = rxA; rxA = rxB; rxB = p;
            p = ryA; ryA = ryB; ryB = p;
            int* q = cntA; cntA = cntB; cntB = q;
            q = seqA; seqA = seqB; seqB = q;
        }
        nextSeq += CH;
        S = Snew;
        if (round < 9) OCT_STAMP(3 + round);
        if (S >= N || S == prevSize) break;                       // :669-672 / :734-735
        if (phase == 1 && S + nToExpand * 3 > N) {                // :673
            phase = 2;
            if (ost && tid == 0) ost[30] = (unsigned long long)(round + 1);
        }
    }

#undef OCT_SUB
    // 3. retain the best key per node (:741-762): max response, first in key order on ties
    uint32_t* best = (uint32_t*)quad;
    for (int t = tid; t < S; t += NT) best[t] = 0;
    __syncthreads();
    OCT_STAMP(17);
    for (int i = tid; i < C; i += NT) {
        const uint32_t v = ((keys[i] >> 24) << 24) | (uint32_t)(0xFFFFFF - i);
        atomicMax(&best[knode[i]], v);
    }
    __syncthreads();
    OCT_STAMP(18);
    uint32_t* outK = lvlKps + (long long)f * g->nkpcap + L.kp_base;
    for (int t = tid; t < S; t += NT) {
        const int i = 0xFFFFFF - (int)(best[t] & 0xFFFFFF);
        const uint32_t k = keys[i];
        const uint32_t x = (k & 0xFFF) + kMinBorder, y = ((k >> 12) & 0xFFF) + kMinBorder;   // :841-847
        oct_out<CP>(&outK[t], x | (y << 12) | (k & 0xFF000000u));
    }
    if (tid == 0) oct_out<CP>(&lvlCount[f * g->nlevels + l], S);
    OCT_STAMP(31);
#undef OCT_STAMP
}

// a candidate word (record or slot) at element i of the dataflow launch: an sc1 buffer load
template <int CP>
__device__ __forceinline__ uint32_t cand_slot(__amdgpu_buffer_rsrc_t rs, unsigned i) {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * i), 0, CP);
}

// One (frame f, level l) of the octree by the whole block of NT threads: the candidate gather, then
// octree_level.  smem: octree_lds_bytes(node_cap) + lds_keys * 6 bytes.
template <int NT, int CP>
__device__ __forceinline__ void octree_task(const Geom* __restrict__ g, int f, int l, int* smem,
                                            const uint32_t* __restrict__ cands, const uint32_t* __restrict__ candFirst,
                                            uint32_t* __restrict__ keysAll, uint16_t* __restrict__ knodeAll,
                                            uint32_t* __restrict__ lvlKps, int* __restrict__ lvlCount,
                                            int* __restrict__ err, int lds_keys, unsigned long long* __restrict__ ostamps) {
    const int NC = g->node_cap;
    const int tid = tidx<CP>();
    const LevelGeom& L = g->L[l];
    // optional timestamps (ORBGPU_FAST_STAMPS=1): 32 per (frame, level): 0 start, 1 gathered, 2 roots,
    // 3.. end of round r (up to 9), 12.. / 20.. sub-steps of round 0 / the first phase-2 round,
    // 29 = C, 30 = phase-2 start round, 31 done
    unsigned long long* ost = ostamps ? ostamps + ((long long)f * g->nlevels + l) * 32 : nullptr;
#if ORBGPU_KERNEL_STAMPS
    if (ost && tid == 0) ost[0] = __builtin_amdgcn_s_memtime();
#endif
    // 1. gather the candidates in cell order (vToDistributeKeys, :818-825) in one global round trip: a
    // thread per cell loads its record, the corner count and the first kFirst corners (two 16-byte loads:
    // 32 B per cell instead of a line per cell); block scans give the cells' offsets; a cell
    // with more corners loads the rest from its slots after them.  Keys go to LDS after the node tables
    // when they fit (every pass re-reads them), else to the per-level global scratch.
    constexpr int kFirst = kCandFirst;
    const int ncl = L.nCols * L.nRows;
    const uint32_t* cs = cands + (long long)f * g->ncand + L.cand_base;
    const uint4* cf = reinterpret_cast<const uint4*>(candFirst) + ((long long)f * g->ncells + L.cell_base) * 2;
    const uint32_t* cr = candFirst + ((long long)f * g->ncells + L.cell_base) * kCandRec;
    static_assert(kCandRec == 8, "two uint4 per cell record");
    // (CP: the records and slots are read through buffer descriptors with sc1 loads; unused otherwise)
    // (made where used, so that the plain instantiation carries no descriptor registers)
    auto crsf = [&]() { return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(cr), 0, ncl * kCandRec * 4, 0x00020000); };
    auto csrf = [&]() { return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(cs), 0, L.cand_cap * 4, 0x00020000); };
    int* sc = smem + 16 * NC;   // after the node tables (octree_lds_bytes)
    int* sv = sc + 32;
    uint32_t* keysL = reinterpret_cast<uint32_t*>(sv + 8);
    const long long o = ((long long)f * g->nlevels + l) * g->max_level_cand;
    int par = 0;
    // the common case: at most kMaxChunks chunks of NT cells, every load issued before the first scan and
    // the values held in registers until the keys' home (LDS or scratch, known once C is) is decided
    constexpr int kMaxChunks = 4;
    const int nch = (ncl + NT - 1) / NT;
    int C = 0;
    bool inLds;
    uint32_t* keys;
    if (nch <= kMaxChunks) {
        int n[kMaxChunks], off[kMaxChunks];
        uint32_t v[kMaxChunks][kFirst];
#pragma unroll
        for (int j = 0; j < kMaxChunks; j++) {
            n[j] = 0;
#pragma unroll
            for (int k = 0; k < kFirst; k++) v[j][k] = 0;
            const int c = j * NT + tid;
            if (j < nch && c < ncl) {
                uint4 r0, r1;
                if constexpr (CP != 0) {
                    const uint32x4_t a = __builtin_amdgcn_raw_buffer_load_b128(crsf(), 32 * c, 0, CP);
                    const uint32x4_t b = __builtin_amdgcn_raw_buffer_load_b128(crsf(), 32 * c + 16, 0, CP);
                    r0 = make_uint4(a[0], a[1], a[2], a[3]);
                    r1 = make_uint4(b[0], b[1], b[2], b[3]);
                } else {
                    r0 = cf[2 * c];
                    r1 = cf[2 * c + 1];
                }
                n[j] = (int)r0.x;
                v[j][0] = r0.y;
                v[j][1] = r0.z;
                v[j][2] = r0.w;
                v[j][3] = r1.x;
                v[j][4] = r1.y;
                v[j][5] = r1.z;
                v[j][6] = r1.w;
            }
        }
#pragma unroll
        for (int j = 0; j < kMaxChunks; j++) {
            if (j < nch) {   // uniform
                int tot;
                off[j] = C + oct_scan<NT, CP>(n[j], sc, par, tot);
                C += tot;
            }
        }
        inLds = C <= lds_keys;
        keys = inLds ? keysL : keysAll + o;
#pragma unroll
        for (int j = 0; j < kMaxChunks; j++) {
            const int c = j * NT + tid;
            if (j < nch && c < ncl) {
#pragma unroll
                for (int k = 0; k < kFirst; k++)
                    if (k < n[j]) keys[off[j] + k] = v[j][k];
                if constexpr (CP != 0) {
                    for (int k = kFirst; k < n[j]; k++) keys[off[j] + k] = cand_slot<CP>(csrf(), __umul24((unsigned)c, (unsigned)L.cell_cap) + k);
                } else {
                    for (int k = kFirst; k < n[j]; k++) keys[off[j] + k] = cs[__umul24((unsigned)c, (unsigned)L.cell_cap) + k];
                }
            }
        }
    } else {   // many cells (large images / fine grids): two passes, a chunk of NT cells at a time
        int base = 0;
        for (int c0 = 0; c0 < ncl; c0 += NT) {
            const int c = c0 + tid;
            int n = 0;
            if constexpr (CP != 0) n = c < ncl ? (int)cand_slot<CP>(crsf(), (unsigned)c * kCandRec) : 0;
            else n = c < ncl ? (int)cr[(long long)c * kCandRec] : 0;
            int tot;
            (void)oct_scan<NT, CP>(n, sc, par, tot);
            base += tot;
        }
        C = base;
        inLds = C <= lds_keys;
        keys = inLds ? keysL : keysAll + o;
        base = 0;
        for (int c0 = 0; c0 < ncl; c0 += NT) {
            const int c = c0 + tid;
            int n = 0;
            if constexpr (CP != 0) n = c < ncl ? (int)cand_slot<CP>(crsf(), (unsigned)c * kCandRec) : 0;
            else n = c < ncl ? (int)cr[(long long)c * kCandRec] : 0;
            int tot;
            const int off = base + oct_scan<NT, CP>(n, sc, par, tot);
            if constexpr (CP != 0) {
                for (int k = 0; k < n; k++)
                    keys[off + k] = k < kFirst ? cand_slot<CP>(crsf(), (unsigned)c * kCandRec + 1 + k)
                                               : cand_slot<CP>(csrf(), __umul24((unsigned)c, (unsigned)L.cell_cap) + k);
            } else {
                for (int k = 0; k < n; k++)
                    keys[off + k] = k < kFirst ? cr[(long long)c * kCandRec + 1 + k]
                                               : cs[__umul24((unsigned)c, (unsigned)L.cell_cap) + k];
            }
            base += tot;
        }
    }
    if (inLds)
        octree_level<true, NT, CP>(g, L, f, l, smem, C, keys, reinterpret_cast<uint16_t*>(keysL + lds_keys), lvlKps, lvlCount,
                               err, par, ost);
    else
        octree_level<false, NT, CP>(g, L, f, l, smem, C, keys, knodeAll + o, lvlKps, lvlCount, err, par, ost);
}


template <int NT>   // block size: kOctreeThreads (512); the dataflow launch runs the same body at 1024
__global__ __launch_bounds__(NT) void k_octree(const Geom* __restrict__ g,
                                                           const uint32_t* __restrict__ cands,
                                                           const uint32_t* __restrict__ candFirst,
                                                           uint32_t* __restrict__ keysAll,
                                                           uint16_t* __restrict__ knodeAll,
                                                           uint32_t* __restrict__ lvlKps, int* __restrict__ lvlCount,
                                                           int* __restrict__ err, int lds_keys,
                                                           unsigned long long* __restrict__ ostamps, int lbase) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    // frames along x so that every frame's level-0 block (the longest) is dispatched first
    octree_task<NT, 0>(g, blockIdx.x, lbase + (int)blockIdx.y, smem, cands, candFirst, keysAll, knodeAll, lvlKps,
                       lvlCount, err, lds_keys, ostamps);
}

/* ------------------------------------------------------------------------------------------------
 * Fused IC_Angle (ORBextractor.cc:77-104) + GaussianBlur 7x7 sigma 2 (:1085-1086) +
 * computeOrbDescriptor (:108-147) + output assembly (:1093-1103).  One wavefront per keypoint:
 * a 43x43 window of the unblurred level (REFLECT_101 at the level border) is staged in LDS, the
 * 37x37 blurred patch is computed from it (exact integer row pass, column pass rounded as the
 * pinned OpenCV 3.2 8U path does), and the 256 tests are four 64-lane ballots.
 * --------------------------------------------------------------------------------------------- */
constexpr float kAtanScale = (float)(180 / 3.14159265358979323846);
constexpr float kP1 = 0.9997878412794807f * kAtanScale;
constexpr float kP3 = -0.3258083974640975f * kAtanScale;
constexpr float kP5 = 0.1555786518463281f * kAtanScale;
constexpr float kP7 = -0.04432655554792128f * kAtanScale;
constexpr float kFactorPI = (float)(3.14159265358979323846 / 180.f);

__device__ __forceinline__ float fast_atan2(float y, float x) {   // cv::fastAtan2 (Appendix A.4)
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



// Per-wave LDS: RT (kDescRtCols columns of kRtPitch u16) from offset 0, the 43 x 48 window from kDescWinOff,
// overlapping RT's tail by less than six window rows: every RT store lands in window rows 0..5, which only
// the row pass's first row tile reads (before any store; IC_Angle reads rows 6..36), checked below.  5,040 B
// per wave instead of 5,520: 8 workgroups (32 waves) per CU instead of 7.
constexpr int kDescRtCols = 37, kDescWinOff = 2976, kDescWaveBytes = kDescWinOff + kDescWin * kDescWinPitch;
constexpr bool desc_overlap_ok() {
    return 2 * kRtPitch * kDescRtCols <= kDescWinOff + 6 * kDescWinPitch && kDescWinOff % 16 == 0 &&
           kDescWaveBytes % 16 == 0 && 4 * kDescWaveBytes + 256 <= 160 * 1024 / 8;
}
static_assert(desc_overlap_ok(), "k_describe LDS overlap");

// One keypoint slot of k_describe: decoded from the octree output (level, coordinates, output index).
struct DescSlot {
    bool ok, interior;   // a keypoint; its 48-byte aligned window rows stay inside the level (dword loads)
    int s, l, x, y, score, outIdx;
    LevelPtr src;
};

// (CP: the octree's counts and keypoints were written by other workgroups of the same launch: sc1 vector loads,
// never the scalar cache)
template <int CP = 0>
__device__ __forceinline__ DescSlot desc_slot(const Geom* __restrict__ g, int f, int s, const int* cnts,
                                              const uint32_t* __restrict__ lvlKps, const uint8_t* frames,
                                              long long framePitch, int rowStride, const uint8_t* pyr) {
    DescSlot d;
    d.s = s;
    d.ok = false;
    d.interior = false;
    if (s >= g->nkpcap) return d;
    const int nl = g->nlevels;
    int l = 0;
    while (l + 1 < nl && s >= g->L[l + 1].kp_base) ++l;
    const LevelGeom& L = g->L[l];
    const int k = s - L.kp_base;
    auto cnt = [&](int i) -> int {
        if constexpr (CP != 0) return __hip_atomic_load(&cnts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else return cnts[i];
    };
    if (k >= cnt(l)) return d;
    int outIdx = k;
    for (int i = 0; i < l; i++) outIdx += cnt(i);
    uint32_t kp;
    if constexpr (CP != 0) kp = __hip_atomic_load(&lvlKps[(long long)f * g->nkpcap + s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else kp = lvlKps[(long long)f * g->nkpcap + s];
    d.ok = true;
    d.l = l;
    d.x = kp & 0xFFF;
    d.y = (kp >> 12) & 0xFFF;
    d.score = kp >> 24;
    d.outIdx = outIdx;
    d.src = level_ptr(g, l, frames, framePitch, rowStride, pyr, f);
    const bool aligned = ((reinterpret_cast<uintptr_t>(d.src.p) | (uintptr_t)d.src.stride) & 3) == 0;
    d.interior = aligned && d.x >= 21 && d.x + 27 <= L.w && d.y >= 21 && d.y + 21 < L.h;
    return d;
}

// 43 rows x 12 dwords of an interior window, issued into registers: lane = (row wy0 = lane / 12,
// dword ww = lane % 12), round r loads row wy0 + 5r (9 rounds).  Lanes 60..63 duplicate lanes 0..3 of
// the next round (same dword, same value); rows 43..47 of the last round are not read.  The per-lane
// offset is computed once; each round adds a wave-uniform soffset.
template <int CP = 0>
__device__ __forceinline__ void desc_issue(const DescSlot& d, int lane, uint32_t (&v)[9]) {
    const int a0 = (d.x - 21) & ~3;
    // the slot is wave-uniform: a buffer descriptor over the window rows (SGPRs), the lane's dword as
    // voffset and the round's row step as soffset, so no per-round address arithmetic
    const int stride = __builtin_amdgcn_readfirstlane(d.src.stride);
    const uint64_t rb = reinterpret_cast<uint64_t>(d.src.p + (long long)(d.y - 21) * stride + a0);
    // (readfirstlane returns int: zero-extend both halves)
    const uint64_t rbu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(rb >> 32)) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)rb);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(rbu), 0, (kDescWin - 1) * stride + 48,
                                                          0x00020000);
    const int wy0 = (int)(__umul24((unsigned)lane, 2731u) >> 15), ww = lane - wy0 * 12;   // lane / 12
    const int off = (int)roi_off(wy0, stride, 4 * ww);
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 5 * r * stride, CP);
    // last round: rows 40..42 only (lane < 36); the others take a voffset past the range (reads 0 whether
    // or not the range check counts soffset)
    v[8] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, lane < 36 ? off : 0x40000000, 40 * stride, CP);
}

// 256 rBRIEF tests of one keypoint, the blurred samples computed at the sample pixels only (the column
// pass of the 7x7 blur over RT[bx][by .. by+6], rounded as the pinned OpenCV 3.2 8U path: half-to-even
// where the SSE2 body runs (x < W & ~3), half-up in the scalar tail).  ALLEVEN: every sampled column
// lies in the SSE2 body (x + 18 < W & ~3), so the per-sample column test drops out.  FMA: the sample
// offsets contracted as the reference's -march=native build does (else ORB_VARIANT_NO_FMA: uncontracted).
template <bool ALLEVEN, bool FMA>
__device__ __forceinline__ void brief_sampled(const uint16_t* rt, float a, float b, const float (&pf)[4][4], int colBase,
                                              int xsimd, ushort2_t K01, ushort2_t K23, ushort2_t K45, ushort2_t K60,
                                              int lane, unsigned long long* __restrict__ dst) {
    // RT's LDS byte address, biased by -2kC (see below): sample addresses are 32-bit LDS offsets
    typedef const uint32_t __attribute__((address_space(3))) lds_u32;
    constexpr uint32_t kC = (uint32_t)kRtPitch * 0x400000u + 0x4B400000u;   // even (see below)
    static_assert((kC & 1u) == 0, "the element bias must keep the parity");
    const uint32_t lbase = (uint32_t)(uintptr_t)(lds_u32*)reinterpret_cast<const uint32_t*>(rt) - 2u * kC;
    // the scalar-tail test colBase + xb < xsimd on the raw x bits (xbits = 0x4B400000 + xb)
    const uint32_t xlim = (uint32_t)(xsimd - colBase) + 0x4B400000u;
    const uint32_t bias = sgpr_const(32767u);
    // S + rounding bias of the blurred pixel at offset (cvRound(fx), cvRound(fy)) from the centre;
    // the blurred value is the high half
    typedef float f32x2_t __attribute__((ext_vector_type(2)));
    const f32x2_t ab = {a, b}, nba = {-b, a}, cr = {12582930.0f, 12582930.0f};
    // the sample offsets as the reference's -O3 -march=native build contracts them (:119-120;
    // tools/ref_flags_probe.cpp): x = fma(px, a, -(py*b)), y = fma(px, b, py*a), both coordinates in
    // packed f32 ops (ORB_VARIANT_NO_FMA: px * a - py * b and px * b + py * a, each product rounded; the
    // kernels build with -ffp-contract=off)
    auto sample = [&](f32x2_t pp) -> uint32_t {   // pp = (px, py)
        const f32x2_t pyv = __builtin_shufflevector(pp, pp, 1, 1), pxv = __builtin_shufflevector(pp, pp, 0, 0);
        const f32x2_t t = pyv * nba;
        const f32x2_t r = (FMA ? __builtin_elementwise_fma(pxv, ab, t) : pxv * ab + t) + cr;
        const float fx = r.x, fy = r.y;
        // cvRound (half-to-even) as one add: v + 1.5*2^23 rounds to an integer for |v| < 2^22, and the
        // +18 centre offset is folded into the constant (it is even, so ties still go to even).  The sum's
        // bits are 0x4B400000 + xb: v_mad_u32_u24 on the raw bits (its 24-bit operand keeps 0x400000 + xb)
        // gives RT element xb * kRtPitch + yb plus kC = kRtPitch * 0x400000 + 0x4B400000, even, so it
        // keeps the element's parity and cancels against lbase's -2C in the 32-bit LDS address
        const uint32_t xbits = __builtin_bit_cast(uint32_t, fx);
        const uint32_t ybits = __builtin_bit_cast(uint32_t, fy);
        const uint32_t idx = __umul24(xbits, (unsigned)kRtPitch) + ybits;
        uint32_t ie = idx & ~1u;
        asm("" : "+v"(ie));   // keeps and + v_lshl_add (the compiler would re-form shl, and, add)
        lds_u32* rp = (lds_u32*)(uintptr_t)(lbase + (ie << 1));
        const uint32_t sh = idx << 4;   // v_alignbit reads bits 4:0: 16 for an odd element, realigning the u16 pairs
        // 7 taps from 4 dwords: the last pair's high element has weight 0 (K60), so whatever alignbit
        // shifts into it (d3 again for an odd element) drops out -- no fifth dword
        const uint32_t d0 = rp[0], d1 = rp[1], d2 = rp[2], d3 = rp[3];
        uint32_t S = __builtin_amdgcn_udot2(K01, __builtin_bit_cast(ushort2_t, __builtin_amdgcn_alignbit(d1, d0, sh)), 0u, false);
        S = __builtin_amdgcn_udot2(K23, __builtin_bit_cast(ushort2_t, __builtin_amdgcn_alignbit(d2, d1, sh)), S, false);
        S = __builtin_amdgcn_udot2(K45, __builtin_bit_cast(ushort2_t, __builtin_amdgcn_alignbit(d3, d2, sh)), S, false);
        S = __builtin_amdgcn_udot2(K60, __builtin_bit_cast(ushort2_t, __builtin_amdgcn_alignbit(d3, d3, sh)), S, false);
        // round(S / 65536): half-to-even = (S + 32767 + q&1) >> 16, half-up = (S + 32768) >> 16
        if (ALLEVEN) return S + bias + ((S >> 16) & 1u);
        return S + (xbits < xlim ? bias + ((S >> 16) & 1u) : 32768u);
    };
    unsigned long long mq[4];
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {   // test pair lane + 64 gq: (x0, y0, x1, y1) = pf[gq]
        const uint32_t r0 = sample(f32x2_t{pf[gq][0], pf[gq][1]});
        const uint32_t r1 = sample(f32x2_t{pf[gq][2], pf[gq][3]});
        // saturate_cast<uchar>: only the right-hand side needs the clamp (t0 = 256 compares as 255 would)
        mq[gq] = __ballot((r0 >> 16) < min(r1 >> 16, 255u));
    }
    // the four 64-test words in one store (lanes 0..3)
    if (lane < 4) dst[lane] = lane == 0 ? mq[0] : lane == 1 ? mq[1] : lane == 2 ? mq[2] : mq[3];
}

template <bool FMA, int CP = 0>
__device__ __forceinline__ void desc_body(const Geom* __restrict__ g, const DescSlot& d, int f, int lane,
                                          const uint32_t (&v)[9], uint8_t* wbase, uint16_t* rt,
                                          orb_keypoint* __restrict__ outK, uint8_t* __restrict__ outD, int kpCap,
                                          unsigned long long* __restrict__ dstamps) {
    const int l = d.l, x = d.x, y = d.y, score = d.score, outIdx = d.outIdx;
    const LevelGeom& L = g->L[l];
    const LevelPtr src = d.src;
    [[maybe_unused]] unsigned long long* dst_st = dstamps ? dstamps + ((long long)f * g->nkpcap + d.s) * 8 : nullptr;
#if ORBGPU_KERNEL_STAMPS
#define DESC_STAMP(k) \
    if (dst_st && lane == 0) dst_st[(k)] = __builtin_amdgcn_s_memtime();
#else
#define DESC_STAMP(k)
#endif
    DESC_STAMP(0);
    // the lane's IC_Angle byte masks (constant table), issued before the window is stored
    const uint4 mm = reinterpret_cast<const uint4*>(&c_ic_masks.m[0][0])[lane];
    const uint32_t icm[4] = {mm.x, mm.y, mm.z, mm.w};
    uint32_t* w32 = reinterpret_cast<uint32_t*>(wbase);
    int sh;
    if (d.interior) {
#pragma unroll
        for (int r = 0; r < 9; r++)   // window dword (wy0 + 5r) * 12 + ww = lane + 60 r; rows < 43 only
            if (r < 8 || lane < 36) w32[lane + 60 * r] = v[r];
        sh = (x - 21) & 3;
    } else {
               // flight in two batches of 15 (fewer live registers than one batch of 29)
#pragma unroll
        for (int hb = 0; hb < 2; hb++) {
            uint8_t v[15];
#pragma unroll
            for (int r = 0; r < 15; r++) {   // 43*43 = 1849 <= 30 x 64
                const int idx = lane + 64 * (15 * hb + r);
                const int wy = (int)(__umul24((unsigned)idx, 24386u) >> 20), wx = idx - wy * kDescWin;   // idx / 43
                int sy = y - 21 + wy, sx = x - 21 + wx;
                sy = sy < 0 ? -sy : (sy >= L.h ? 2 * L.h - 2 - sy : sy);
                sx = sx < 0 ? -sx : (sx >= L.w ? 2 * L.w - 2 - sx : sx);
                if constexpr (CP != 0) {   // a border window of a pyramid level: sc1 byte loads
                    const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src.p), 0, 0x7FFFFFFF, 0x00020000);
                    v[r] = idx < kDescWin * kDescWin ? __builtin_amdgcn_raw_buffer_load_b8(brs, (int)roi_off(sy, src.stride, sx), 0, CP)
                                                     : (uint8_t)0;
                } else {
                    v[r] = idx < kDescWin * kDescWin ? src.p[roi_off(sy, src.stride, sx)] : (uint8_t)0;
                }
            }
#pragma unroll
            for (int r = 0; r < 15; r++) {
                const int idx = lane + 64 * (15 * hb + r);
                const int wy = (int)(__umul24((unsigned)idx, 24386u) >> 20), wx = idx - wy * kDescWin;
                if (idx < kDescWin * kDescWin) wbase[wy * kDescWinPitch + wx] = v[r];
            }
        }
        sh = 0;
    }
    wave_lds_sync();
    DESC_STAMP(1);
#if defined(ORBGPU_DESC_CUT) && ORBGPU_DESC_CUT == 1   // instruction-count diagnostics only (tools/diag_cut.sh)
    if (lane == 0) outD[((long long)f * kpCap + outIdx) * 32] = wbase[lane];
    return;
#endif

    // ---- IC_Angle (:77-104) on the unblurred window: lanes 2r, 2r+1 (r < 31) sum halves of row v = r - 15
    // over the circular patch |u| <= umax[|v|] with v_dot4_u32_u8 (u*I = (u+16)*I - 16*I); two lanes per
    // row halve the wave's instructions
    int m10 = 0, m01 = 0;
    if (lane < 62) {
        const int v = (lane >> 1) - 15, h = lane & 1;
        const int base = (21 + v) * kDescWinPitch + sh + 6;   // byte of u = -15
        const int d0 = (base >> 2) + 4 * h, bs = base & 3;
        uint32_t w[5];
#pragma unroll
        for (int i = 0; i < 5; i++) w[i] = w32[d0 + i];
        // weights (u + 16) for u = 4c-15 .. 4c-12, c = 4h + i  ->  4c+1 .. 4c+4
        const uint32_t wt0 = 0x04030201u + (uint32_t)h * 0x10101010u;
        uint32_t sI = 0, sW = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t bytes = __builtin_amdgcn_alignbyte(w[i + 1], w[i], bs) & icm[i];
            sI = __builtin_amdgcn_udot4(bytes, 0x01010101u, sI, false);
            sW = __builtin_amdgcn_udot4(bytes, wt0 + (uint32_t)i * 0x04040404u, sW, false);
        }
        m10 = (int)sW - 16 * (int)sI;
        m01 = v * (int)sI;
    }
    m10 = wave_sum(m10);   // DPP reductions: no LDS round trips
    m01 = wave_sum(m01);
    const float angle = fast_atan2((float)m01, (float)m10);
    DESC_STAMP(2);
#if defined(ORBGPU_DESC_CUT) && ORBGPU_DESC_CUT == 2
    if (lane == 0) outD[((long long)f * kpCap + outIdx) * 32] = (uint8_t)angle;
    return;
#endif

    // ---- GaussianBlur 7x7 sigma 2 (:1085-1086), exact integer row pass on the matrix cores: RT[c][y] =
    // sum_t k_t * window[y][sh + c + t] is D = W T with W the window (43 x 64 bytes: row y's 48 loaded bytes,
    // the rest of the K range meets zero taps) and T the banded tap matrix (Geom::desc_taps, per sh).  Nine
    // v_mfma_i32_16x16x64_i8 (y and c in tiles of 16); the window bytes are signed by ^ 0x80 (i8 operands)
    // and the accumulator starts at 128 * sum(k) = 128 * 257, which restores the unsigned sums exactly
    // (every sum < 2^16).  Lane l holds W[y = 16 ty + (l & 15)][16 (l >> 4) .. + 15] (one 16-byte LDS read)
    // and, of D, column c = 16 tc + (l & 15) at rows 4 (l >> 4) .. + 3: four u16 of RT's column c, one
    // 8-byte store (kRtPitch even).
    {
        typedef int v4i_t __attribute__((ext_vector_type(4)));
        const int4* tp = g->desc_taps + sh * kDescTapTiles * 64 + lane;
        v4i_t bt[kDescTapTiles];
#pragma unroll
        for (int tc = 0; tc < kDescTapTiles; tc++) {
            const int4 q = tp[tc * 64];
            bt[tc] = v4i_t{q.x, q.y, q.z, q.w};
        }
        const int yl = lane & 15, kq = lane >> 4;
        const int bias = 128 * (g->gk[0] + g->gk[1] + g->gk[2] + g->gk[3] + g->gk[4] + g->gk[5] + g->gk[6]);
#pragma unroll
        for (int ty = 0; ty < 3; ty++) {
            const int y = min(16 * ty + yl, kDescWin - 1);   // rows 43..47 repeat row 42 (not stored)
            const uint4 w = *reinterpret_cast<const uint4*>(wbase + y * kDescWinPitch + 16 * kq);
            const v4i_t a = v4i_t{(int)(w.x ^ 0x80808080u), (int)(w.y ^ 0x80808080u), (int)(w.z ^ 0x80808080u),
                                  (int)(w.w ^ 0x80808080u)};
            const int y0 = 16 * ty + 4 * kq;   // this lane's first D row
#pragma unroll
            for (int tc = 0; tc < kDescTapTiles; tc++) {
                v4i_t d = v4i_t{bias, bias, bias, bias};
                d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bt[tc], d, 0, 0, 0);
                const int c = 16 * tc + yl;
                if (y0 < kDescWin && c < kDescRtCols) {   // (row 43 of the last group lands in the column's pad)
                    uint2 pk;   // the low halves of two results per dword: one v_perm each
                    pk.x = __builtin_amdgcn_perm((uint32_t)d[1], (uint32_t)d[0], 0x05040100u);
                    pk.y = __builtin_amdgcn_perm((uint32_t)d[3], (uint32_t)d[2], 0x05040100u);
                    *reinterpret_cast<uint2*>(rt + c * kRtPitch + y0) = pk;
                }
            }
        }
    }
    wave_lds_sync();
    DESC_STAMP(3);
#if defined(ORBGPU_DESC_CUT) && ORBGPU_DESC_CUT == 3
    if (lane == 0) outD[((long long)f * kpCap + outIdx) * 32] = (uint8_t)(angle + rt[lane]);
    return;
#endif

    // ---- column pass: evaluated only at the 512 BRIEF sample pixels (brief_sampled), v_dot2_u32_u16 on
    // row pairs of RT; rounding as the pinned OpenCV 3.2 8U path: half-to-even where the SSE2 body runs
    // (x < W & ~3), half-up in the scalar tail; ORB_VARIANT_BLUR_HALFUP: half-up everywhere (no SSE2 body).
    const int xsimd = (g->variant & ORB_VARIANT_BLUR_HALFUP) ? 0 : (L.w & ~3);
    const int k0 = g->gk[0], k1 = g->gk[1], k2 = g->gk[2], k3 = g->gk[3], k4 = g->gk[4], k5 = g->gk[5],
              k6 = g->gk[6];
    const ushort2_t K01 = {(unsigned short)k0, (unsigned short)k1}, K23 = {(unsigned short)k2, (unsigned short)k3},
                    K45 = {(unsigned short)k4, (unsigned short)k5}, K60 = {(unsigned short)k6, 0};
    DESC_STAMP(4);

    // BRIEF test pairs of this lane (lane + 64 gq) from the constant table, issued before the trig so their
    // latency hides under it; loaded here rather than once per wave to keep them out of the row pass's
    // live registers
    float pf[4][4];
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {
        const float4 pp = reinterpret_cast<const float4*>(c_pattern_f)[lane + 64 * gq];
        pf[gq][0] = pp.x;
        pf[gq][1] = pp.y;
        pf[gq][2] = pp.z;
        pf[gq][3] = pp.w;
    }
    // ---- rBRIEF (:108-147): cos/sin as glibc's cosf/sinf compute them (:113, glibc_trig.h); 256 tests
    // as four 64-lane ballots; sample (ix, iy) of the blurred patch at blurT[(18+ix)*40 + 18+iy]
    const float ang = angle * kFactorPI;
    float a, b;
    glibc_sincosf(ang, &b, &a);
    DESC_STAMP(5);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(outD + ((long long)f * kpCap + outIdx) * 32);
    if (x + 18 < xsimd) brief_sampled<true, FMA>(rt, a, b, pf, x - 18, xsimd, K01, K23, K45, K60, lane, dst);
    else brief_sampled<false, FMA>(rt, a, b, pf, x - 18, xsimd, K01, K23, K45, K60, lane, dst);
    if (lane == 0) {
        orb_keypoint o;
        o.x = (float)x;
        o.y = (float)y;
        if (l != 0) {   // :1095-1101
            o.x *= L.scale;
            o.y *= L.scale;
        }
        o.size = L.patch_size;
        o.angle = angle;
        o.response = (float)score;
        o.octave = l;
        o.class_id = -1;
        outK[(long long)f * kpCap + outIdx] = o;
    }
    DESC_STAMP(6);
#undef DESC_STAMP
}

/* Fused IC angle + 7x7 blur + rBRIEF, one wavefront per keypoint slot; a wavefront owns two consecutive
 * slots and issues the second interior window's loads before processing the first. */
constexpr int kDescWaves = 4, kDescSlotsPerWave = 2;
template <bool FMA>   // false: ORB_VARIANT_NO_FMA
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_describe(const Geom* __restrict__ g, const uint8_t* __restrict__ frames,
                                                  long long framePitch, int rowStride, const uint8_t* __restrict__ pyr,
                                                  const uint32_t* __restrict__ lvlKps,
                                                  const int* __restrict__ lvlCount, orb_keypoint* __restrict__ outK,
                                                  uint8_t* __restrict__ outD, int* __restrict__ outN, int kpCap,
                                                  unsigned long long* __restrict__ dstamps, int spw,
                                                  const int* __restrict__ err, int* __restrict__ errHost) {
    // per wave: the transposed row-pass sums RT[rx][wy] (u16, 37 x kRtPitch; an odd pitch spreads the
    // transposed stores of the 10 column groups over distinct banks) and the 43x48 window overlapping RT's
    // tail (kDescWinOff); 256 B past the last wave for the row pass's reads of rows 43..47
    __shared__ __attribute__((aligned(16))) uint8_t s_desc[kDescWaves * kDescWaveBytes + 256];
    uint8_t* const s_wave = s_desc + (size_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kDescWaveBytes;
    // 1-D grid, blocks dealt round-robin over the 8 XCDs: XCD x takes a contiguous run of the (frame,
    // slot-block) sequence, so a frame's windows are fetched into one L2 (PMC: 0.71 GB per 256 C3
    // frames against 1.96 GB with the frames spread over every XCD)
    const int gx = (g->nkpcap + kDescWaves * spw - 1) / (kDescWaves * spw);   // spw: slots per wave, 2 (1 for latency)
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int lb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    const int f = lb / gx, bx = lb - f * gx;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave-uniform: SALU
    const int nl = g->nlevels;
    const int* cnts = lvlCount + f * nl;
    const int s0 = (bx * kDescWaves + wv) * spw;
    // the frame's keypoint count, by its first block's thread 0 (on every path out of the kernel)
    auto write_n = [&]() {
        if (bx == 0 && threadIdx.x == 0) {
            int tot = 0;
            for (int i = 0; i < nl; i++) tot += cnts[i];
            outN[f] = tot;
            if (errHost && f == 0) *errHost = err[0] | err[1];   // the octrees' overflow flags, for the host path
        }
    };
    if (s0 >= g->nkpcap) {
        write_n();
        return;
    }
    const DescSlot d0 = desc_slot(g, f, s0, cnts, lvlKps, frames, framePitch, rowStride, pyr);
    const DescSlot d1 = spw == 2 ? desc_slot(g, f, s0 + 1, cnts, lvlKps, frames, framePitch, rowStride, pyr)
                                 : DescSlot{};
    if (!d0.ok && !d1.ok) {   // (the two slots may straddle a level boundary)
        write_n();
        return;
    }
    uint32_t v0[9], v1[9];
    if (d0.ok && d0.interior) desc_issue(d0, lane, v0);
    if (d1.ok && d1.interior) desc_issue(d1, lane, v1);
    write_n();   // (after the window loads are issued)
    if (d0.ok) desc_body<FMA>(g, d0, f, lane, v0, s_wave + kDescWinOff, reinterpret_cast<uint16_t*>(s_wave), outK, outD, kpCap, dstamps);
    if (d1.ok) {
        __builtin_amdgcn_sched_barrier(0);
        wave_lds_sync();   // the first keypoint's LDS reads precede these window stores
        desc_body<FMA>(g, d1, f, lane, v1, s_wave + kDescWinOff, reinterpret_cast<uint16_t*>(s_wave), outK, outD, kpCap, dstamps);
    }
}

/* The host path's image upload, streamed: the host copies the caller's image band by band into pinned,
 * host-coherent memory and raises a per-band flag (the call's sequence number); this kernel is launched before
 * the host copy starts, each workgroup waits for its band's flag (one lane polls with a system-scope load and
 * s_sleep) and copies the band into HBM over PCIe.  So the PCIe transfer overlaps the host memcpy, and the
 * extraction kernels, launched right after the host copy, queue behind this one (a pageable hipMemcpy2DAsync
 * returns only after its DMA, and the first kernel then starts ~18 us later, profiles/r03/v11_host_path_timeline.txt).  The poll is bounded: a band that never arrives sets the host-side
 * failure flag *err and the workgroup exits (every wave reaches the end).  Band b = rows [b R, min(h, (b + 1) R)); blockIdx.y splits a band. */
__global__ __launch_bounds__(256) void k_upload_stream(const uint8_t* __restrict__ h_img, const uint32_t* h_flags,
                                                       uint32_t seq, uint8_t* __restrict__ d_img, int pitch, int h,
                                                       int band_rows, uint32_t* __restrict__ err) {
    __shared__ int s_ok;
    const int b = blockIdx.x;
    if (threadIdx.x == 0) {
        int ok = 0;
        for (int it = 0; it < (1 << 22); it++) {   // >= 0.5 s: a safety bound, never reached while the host runs
            if (__hip_atomic_load(h_flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == seq) {
                ok = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) *err = 1;   // (vector store to the host flag; the extraction reads a stale image, the host fails the call)
        s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);   // (the band's bytes are read after the flag)
    const int r0 = b * band_rows, r1 = min(h, r0 + band_rows);
    const size_t n16 = (size_t)(r1 - r0) * pitch / 16;   // pitch is a multiple of 64
    const uint4* src = reinterpret_cast<const uint4*>(h_img + (size_t)r0 * pitch);
    uint4* dst = reinterpret_cast<uint4*>(d_img + (size_t)r0 * pitch);
    // four loads in flight per thread before the stores (PCIe latency ~2 us per round trip)
    const size_t st = (size_t)gridDim.y * 256;
    for (size_t i = blockIdx.y * 256 + threadIdx.x; i < n16; i += 4 * st) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * st < n16) v[u] = src[i + u * st];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * st < n16) dst[i + u * st] = v[u];
    }
}

hipError_t launch_upload_stream(const uint8_t* h_img, const uint32_t* h_flags, uint32_t seq, uint8_t* d_img, int pitch,
                                int h, int nbands, int band_rows, uint32_t* h_fail, hipStream_t stream) {
    hipLaunchKernelGGL(k_upload_stream, dim3(nbands, 4), dim3(256), 0, stream, h_img, h_flags, seq, d_img, pitch, h,
                       band_rows, h_fail);
    return hipGetLastError();
}

/* glibc_sincosf over an array of angles (the C-ABI's orb_debug_sincosf: the GPU test pins the device
 * restatement against the oracle's and libm on the host) */
__global__ __launch_bounds__(256) void k_debug_sincosf(const float* __restrict__ x, int n, float* __restrict__ s,
                                                       float* __restrict__ c) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float sv, cv;
    glibc_sincosf(x[i], &sv, &cv);
    s[i] = sv;
    c[i] = cv;
}

hipError_t launch_debug_sincosf(const float* d_x, int n, float* d_s, float* d_c, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_debug_sincosf, dim3((n + 255) / 256), dim3(256), 0, stream, d_x, n, d_s, d_c);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------------------------------
 * The small-batch dataflow launch (orbgpu_internal.h FlowTask).  One frame leaves most of the chip idle, and the
 * per-kernel launches serialise every level behind the slowest one at each stage (the chain of ten dependent
 * launches measured 74-79 us per C5 frame, profiles/r05/c5b1_trace.txt): here each level's FAST, octree and
 * describe start as soon as that level exists, so the small upper levels and level 0 run beside the pyramid and the
 * slow middle-level octrees.  Hand-offs between workgroups follow MI355X_MICROARCH.md's write-through form: every
 * store of handed-off bytes (pyramid levels, candidate records and slots, octree outputs) and every load of them
 * carries sc1 (kCpSc1: the bodies' CP parameter), each storing wave drains its stores (s_waitcnt vmcnt(0)) before the
 * workgroup barrier after which one lane raises the task's counter (an agent-scope atomic); a waiting workgroup's
 * lane 0 polls its counters with relaxed agent loads and s_sleep, then releases the workgroup through a barrier.
 * Tasks are taken from one ticket counter in the host's topological order, so a task only ever waits on tasks that
 * running workgroups hold (no residency assumption), and every wait is bounded (a timeout raises an error flag the
 * host reads).  The launch's last workgroup re-zeroes the counters for the next launch.
 * --------------------------------------------------------------------------------------------- */

__device__ __forceinline__ int flow_ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void flow_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int flow_add(int* p, int v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The stages of one task.  Each reads the launch's arguments itself from the argument block in device memory (Ap),
// inside its own branch: nothing but the ticket is carried around the task loop, so the loop adds no registers to the
// largest body's (kernel-argument fields held across the loop spilled the octree's SGPRs into VGPRs).
template <int TQ>
__device__ __forceinline__ void flow_fast(const FlowArgs* __restrict__ Ap, int l, int f, int a, int b, int wv, int lane,
                                          uint8_t* smem) {
    if (wv >= b) return;
    const Geom* __restrict__ g = Ap->g;
    const int wb = g->fast_wave_bytes;
    uint16_t* tile = reinterpret_cast<uint16_t*>(smem + (size_t)wv * wb + 16);
    uint16_t* sList = reinterpret_cast<uint16_t*>(smem + (size_t)wv * wb + ((g->fast_rows * TQ * 2 + 32 + 15) & ~15));
    const int cell = g->L[l].cell_base + a + wv;
    const FastCellT c = fast_cell_t(g, Ap->cells, f * g->ncells + cell, Ap->frames, Ap->framePitch, Ap->rowStride,
                                    Ap->pyr, 0, g->ncells);
    uint32_t* candFirst = Ap->candFirst;
    int* cntOut = reinterpret_cast<int*>(candFirst + ((long long)c.f * g->ncells + c.cell) * kCandRec);
    if (!c.valid) {
        if (lane == 0) flow_st(cntOut, 0);
        return;
    }
    uint32_t v[8];
    if (c.aligned) fast_roi_issue<kCpSc1>(c, lane, v);
    fast_roi_store<TQ, kCpSc1>(c, lane, v, tile);
    fast_cell_body<TQ, kCpSc1>(g, c, lane, tile, sList, Ap->cands, candFirst, cntOut, nullptr, 0);
}

__device__ __forceinline__ void flow_resize(const FlowArgs* __restrict__ Ap, int l, int f, int a, int b, int tid,
                                            uint8_t* smem) {
    const Geom* __restrict__ g = Ap->g;
    const int q = tid >> 8;   // 256-thread quarter: one output tile each
    const int th = (g->L[l].rs_tiled & 2) ? 32 : 16;
    const int gxl = (g->L[l].w + kRsTileW - 1) / kRsTileW;
    const int tile = a + q;
    const int by = tile / gxl, bx = tile - by * gxl;
    const int rq = Ap->rsQuarter;
    uint8_t* qb = smem + (size_t)q * rq;
    int4* scx = reinterpret_cast<int4*>(qb + rq - (kRsTileW + 32) * 16);
    int4* scy = scx + kRsTileW;
    const ResizeCoef* cf = Ap->rcoef + Ap->roff.o[l];
    const bool on = q < b;
    const bool gen = (g->variant & ORB_VARIANT_RESIZE_GENERIC) != 0;
    const uint8_t* frames = Ap->frames;
    const long long fp = Ap->framePitch;
    const int rs = Ap->rowStride;
    uint8_t* pyr = Ap->pyr;
    if (th == 32) {
        if (gen) resize_tile<32, true, kCpSc1>(g, cf, l, frames, fp, rs, pyr, f, bx, by, tid & 255, qb, scx, scy, on);
        else resize_tile<32, false, kCpSc1>(g, cf, l, frames, fp, rs, pyr, f, bx, by, tid & 255, qb, scx, scy, on);
    } else {
        if (gen) resize_tile<16, true, kCpSc1>(g, cf, l, frames, fp, rs, pyr, f, bx, by, tid & 255, qb, scx, scy, on);
        else resize_tile<16, false, kCpSc1>(g, cf, l, frames, fp, rs, pyr, f, bx, by, tid & 255, qb, scx, scy, on);
    }
}

// chain task: up to 4 ChainJobs of one level, one per 256-thread quarter (a quarter past the task's jobs repeats its
// first job: the same bytes to the same place)
__device__ __forceinline__ void flow_chain(const FlowArgs* __restrict__ Ap, int f, int a, int b, int seg, int tid,
                                           uint8_t* smem) {
    const Geom* __restrict__ g = Ap->g;
    const int q = tid >> 8;
    const int rq = Ap->rsQuarter;
    uint8_t* qb = smem + (size_t)q * rq;
    int4* sreg = reinterpret_cast<int4*>(qb + rq - ORBGPU_MAX_LEVELS * 16);
    const ChainJob* J = Ap->chainJobs + a + (q < b ? q : 0);
    const ChainSegment sg = Ap->chainSeg[seg];
    RcoefOff ro = Ap->roff;
    if (g->variant & ORB_VARIANT_RESIZE_GENERIC)
        chain_job<true, kCpSc1>(g, Ap->rcoef, J, sg, ro, Ap->frames, Ap->framePitch, Ap->rowStride, Ap->pyr, f, tid & 255, qb, sreg);
    else
        chain_job<false, kCpSc1>(g, Ap->rcoef, J, sg, ro, Ap->frames, Ap->framePitch, Ap->rowStride, Ap->pyr, f, tid & 255, qb, sreg);
}

template <bool FMA>
__device__ __forceinline__ void flow_describe(const FlowArgs* __restrict__ Ap, int f, int a, int b, int wv, int lane,
                                              uint8_t* smem) {
    if (wv >= b) return;
    const Geom* __restrict__ g = Ap->g;
    uint8_t* sw = smem + (size_t)wv * kDescWaveBytes;
    const DescSlot d = desc_slot<kCpSc1>(g, f, a + wv, Ap->lvlCount + f * g->nlevels, Ap->lvlKps, Ap->frames,
                                         Ap->framePitch, Ap->rowStride, Ap->pyr);
    if (!d.ok) return;
    uint32_t v[9];
    if (d.interior) desc_issue<kCpSc1>(d, lane, v);
    desc_body<FMA, kCpSc1>(g, d, f, lane, v, sw + kDescWinOff, reinterpret_cast<uint16_t*>(sw), Ap->outK, Ap->outD,
                           Ap->kpCap, nullptr);
}

template <int TQ, bool FMA>
__global__ __launch_bounds__(kFlowThreads) void k_extract_flow(const FlowArgs* __restrict__ Ap0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t fl_smem[];
    __shared__ int s_tk[2];
    if (threadIdx.x == 0) s_tk[0] = flow_add(&Ap0->ctr[0], 1);
    __syncthreads();
    int cur = __builtin_amdgcn_readfirstlane(s_tk[0]);   // (uniform: the task's fields become scalar loads)
    while (cur < Ap0->ntasks) {   // (cur is block-uniform: every thread read the same LDS word)
        // the thread index and the argument block through opaque moves each task: nothing derived from them is
        // hoisted out of the loop and held live across every task (the largest body keeps its own register count)
        int tid;
        asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
        const int lane = tid & 63;
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
        const FlowArgs* __restrict__ Ap = Ap0;
        asm volatile("" : "+s"(Ap));
        const FlowTask t = Ap->tasks[cur];
        const int kind = t.klf & 0xFF, l = (t.klf >> 8) & 0xFF, f = t.klf >> 16;
        unsigned long long* st = Ap->stamps ? Ap->stamps + 4 * (size_t)cur : nullptr;
        if (tid == 0) {
            if (st) st[0] = __builtin_amdgcn_s_memrealtime();
            int* ctr = Ap->ctr;
            s_tk[1] = flow_add(&ctr[0], 1);   // the next ticket, taken now so its round trip overlaps this task
            if (t.nd > 0 && !flow_ld(&ctr[48])) {   // (once any wait has given up, no task waits any more)
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
                bool late = false;
                for (int k = 0; k < t.nd && !late; k++)
                    while (flow_ld(&ctr[t.dep + k]) < t.tgt) {
                        __builtin_amdgcn_s_sleep(1);
                        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull || flow_ld(&ctr[48])) {
                            // 0.2 s: give up and flag it (the host sees ORB_ERR_INTERNAL from orb_sync)
                            __hip_atomic_fetch_or(&ctr[48], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            late = true;
                            break;
                        }
                    }
            }
        }
        __syncthreads();
        if (st && tid == 0) st[1] = __builtin_amdgcn_s_memrealtime();
        const int nxt = __builtin_amdgcn_readfirstlane(s_tk[1]);
        if (kind == kFlowChain) {
            flow_chain(Ap, f, t.a, t.b, t.seg, tid, fl_smem);
        } else if (kind == kFlowResize) {
            flow_resize(Ap, l, f, t.a, t.b, tid, fl_smem);
        } else if (kind == kFlowFast) {
            flow_fast<TQ>(Ap, l, f, t.a, t.b, wv, lane, fl_smem);
        } else if (kind == kFlowOctree) {
            const Geom* __restrict__ g = Ap->g;
            const int nl = g->nlevels;
            int* eword = &Ap->ctr[kFlowCtrBase + 4 * nl * f + 3 * nl + l];
            octree_task<kFlowThreads, kCpSc1>(g, f, l, reinterpret_cast<int*>(fl_smem), Ap->cands, Ap->candFirst,
                                              Ap->keys, Ap->knode, Ap->lvlKps, Ap->lvlCount, eword, Ap->ldsKeys, nullptr);
        } else {
            flow_describe<FMA>(Ap, f, t.a, t.b, wv, lane, fl_smem);
        }
        // publish: every wave's stores drained, then one lane raises the task's counter
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (st && tid == 0) {
            st[2] = __builtin_amdgcn_s_memrealtime();
            st[3] = (unsigned long long)(unsigned)t.klf | ((unsigned long long)blockIdx.x << 32);
        }
        if (tid == 0 && t.sig >= 0) {
            int* ctr = Ap->ctr;
            flow_add(&ctr[t.sig], 1);
            const int nl = Ap->g->nlevels, nfr = Ap->nframes;
            if (kind == kFlowOctree && flow_add(&ctr[32], 1) == nfr * nl - 1) {
                // the last octree of the launch: every frame's keypoint count and the overflow flags (the other
                // octrees' outputs were drained before their counter adds, which this add follows)
                int e = 0;
                const int* lc = Ap->lvlCount;
                for (int fr = 0; fr < nfr; fr++) {
                    int tot = 0;
                    for (int i = 0; i < nl; i++) {
                        tot += flow_ld(&lc[fr * nl + i]);
                        e |= flow_ld(&ctr[kFlowCtrBase + 4 * nl * fr + 3 * nl + i]);
                    }
                    Ap->outN[fr] = tot;
                }
                Ap->err[0] = e;
                Ap->err[1] = 0;
                if (Ap->errHost) *Ap->errHost = e;
            }
        }
        cur = nxt;
    }
    // the launch's last workgroup re-zeroes every counter (the others have taken their last ticket and touch none)
    if (threadIdx.x == 0) {
        const FlowArgs* __restrict__ Ap = Ap0;
        int* ctr = Ap->ctr;
        if (flow_add(&ctr[16], 1) == (int)gridDim.x - 1) {
            if (flow_ld(&ctr[48])) {   // a wait gave up: the outputs are not valid
                Ap->err[1] = 4;
                if (Ap->errHost) *Ap->errHost = 4;
            }
            const int n = kFlowCtrBase + 4 * Ap->g->nlevels * Ap->nframes;
            for (int i = 0; i < n; i++) flow_st(&ctr[i], 0);
        }
    }
}

/* ------------------------------------------------------------------------------------------------ */
static inline unsigned cdiv(unsigned a, unsigned b) { return (a + b - 1) / b; }

size_t octree_lds_bytes(int node_cap) { return (size_t)node_cap * (16 * 4) + (32 + 8) * 4; }

// Keys (u32 + u16 node index) that fit in LDS after the node tables with the block at <= 52 KiB, so
// that three octree workgroups share a CU (a level with more candidates keeps them in the global
// scratch: the KeysInLds = false instantiation).
static int octree_lds_keys(int node_cap) {
    const long long room = 52 * 1024 - (long long)octree_lds_bytes(node_cap);
    return room > 0 ? (int)((room / 6) & ~7LL) : 0;
}
// one block per CU (small batches): the keys of the largest level, within the CU's 160 KiB
static int octree_lds_keys_whole_cu(const Geom& g) {
    const long long room = 160 * 1024 - (long long)octree_lds_bytes(g.node_cap);
    const long long want = ((long long)g.max_level_cand + 7) & ~7LL;
    return room > 0 ? (int)std::min(want, (room / 6) & ~7LL) : 0;
}

// The dataflow launch's task list (see k_extract_flow): per frame, the stages in the order
//     R1 F0 O0 R2 F1 O1 ... R(n-1) F(n-2) O(n-2) F(n-1) O(n-1) D0 .. D(n-1)
// (Rl: level l's resize tiles, Fl: its FAST cells, Ol: its octree, Dl: its describe slots), the frames interleaved
// task-group by task-group, so the pyramid chain (the critical path to the slow middle-level octrees) is taken
// first and every octree is held by a workgroup as soon as its cells are.  A describe task of level l waits for the
// octrees of levels 0..l (its output index adds their counts, ORBextractor.cc:1103).
bool build_flow(const Geom& g, int nframes, int blocks, const ChainPlan* chain, const std::vector<ChainJob>* jobs,
                std::vector<FlowTask>& tasks, FlowPlan& plan) {
    tasks.clear();
    plan = FlowPlan{};
    const int nl = g.nlevels;
    if (nframes < 1 || nframes > 0xFFFF) return false;
    const bool chained = chain && jobs && chain->nseg > 0 && chain->first_base == 0;
    int rsq = 0;   // one pyramid quarter: the largest source tile + the column / row coefficient slots (or a chain job)
    for (int l = 1; l < nl && !chained; l++) {
        if (!(g.L[l].rs_tiled & 3)) return false;   // (large scale factors: the untiled k_resize)
        rsq = std::max(rsq, ((g.L[l].rs_span_rows * kRsPitch + 15) & ~15) + (kRsTileW + 32) * 16);
    }
    if (chained)
        for (int sgi = 0; sgi < chain->nseg; sgi++)
            rsq = std::max(rsq, ((chain->seg[sgi].lds_bytes + 15) & ~15) + ORBGPU_MAX_LEVELS * 16);
    int nres[ORBGPU_MAX_LEVELS] = {0}, nfast[ORBGPU_MAX_LEVELS] = {0};
    for (int l = 0; l < nl; l++) {
        if (l > 0) {
            const int th = (g.L[l].rs_tiled & 2) ? 32 : 16;
            const int tiles = (int)(cdiv(g.L[l].w, kRsTileW) * cdiv(g.L[l].h, th));
            nres[l] = (tiles + 3) / 4;
        }
        nfast[l] = (g.L[l].nCols * g.L[l].nRows + 15) / 16;
    }
    auto ctr = [&](int f, int part, int l) { return kFlowCtrBase + 4 * nl * f + part * nl + l; };
    auto push = [&](int kind, int l, int f, int sig, int a, int b, int dep, int nd, int tgt) {
        FlowTask t;
        t.klf = kind | (l << 8) | (f << 16);
        t.sig = sig;
        t.a = a;
        t.b = b;
        t.dep = dep;
        t.nd = nd;
        t.tgt = tgt;
        t.seg = 0;
        tasks.push_back(t);
    };
    // chain tasks: per level, its jobs in groups of 4 (jobs of a level are contiguous, one segment each)
    int nchain[ORBGPU_MAX_LEVELS] = {0}, cj0[ORBGPU_MAX_LEVELS] = {0}, cjn[ORBGPU_MAX_LEVELS] = {0},
        cseg[ORBGPU_MAX_LEVELS] = {0}, cbase[ORBGPU_MAX_LEVELS] = {0};
    if (chained) {
        for (int sgi = 0; sgi < chain->nseg; sgi++) {
            const ChainSegment& sg = chain->seg[sgi];
            for (int j = sg.job0; j < sg.job0 + sg.njobs; j++) {
                const int l = (*jobs)[j].level;
                if (cjn[l] == 0) cj0[l] = j;
                cjn[l]++;
                cseg[l] = sgi;
                cbase[l] = (*jobs)[j].base;
            }
        }
        for (int l = 1; l < nl; l++) {
            if (cjn[l] == 0) return false;
            nchain[l] = (cjn[l] + 3) / 4;
            nres[l] = nchain[l];   // (the FAST tasks of level l wait for this many pyramid tasks)
        }
    }
    auto chainl = [&](int l) {
        for (int i = 0; i < nchain[l]; i++)
            for (int f = 0; f < nframes; f++) {
                push(kFlowChain, l, f, ctr(f, 0, l), cj0[l] + 4 * i, std::min(4, cjn[l] - 4 * i),
                     cbase[l] > 0 ? ctr(f, 0, cbase[l]) : 0, cbase[l] > 0 ? 1 : 0, cbase[l] > 0 ? nres[cbase[l]] : 0);
                tasks.back().seg = cseg[l];
            }
    };
    auto resize = [&](int l) {
        const int th = (g.L[l].rs_tiled & 2) ? 32 : 16;
        const int tiles = (int)(cdiv(g.L[l].w, kRsTileW) * cdiv(g.L[l].h, th));
        for (int i = 0; i < nres[l]; i++)
            for (int f = 0; f < nframes; f++)
                push(kFlowResize, l, f, ctr(f, 0, l), 4 * i, std::min(4, tiles - 4 * i), l > 1 ? ctr(f, 0, l - 1) : 0,
                     l > 1 ? 1 : 0, l > 1 ? nres[l - 1] : 0);
    };
    auto fast = [&](int l) {
        const int n = g.L[l].nCols * g.L[l].nRows;
        for (int i = 0; i < nfast[l]; i++)
            for (int f = 0; f < nframes; f++)
                push(kFlowFast, l, f, ctr(f, 1, l), 16 * i, std::min(16, n - 16 * i), l > 0 ? ctr(f, 0, l) : 0,
                     l > 0 ? 1 : 0, l > 0 ? nres[l] : 0);
    };
    auto octree = [&](int l) {
        for (int f = 0; f < nframes; f++) push(kFlowOctree, l, f, ctr(f, 2, l), 0, 0, ctr(f, 1, l), 1, nfast[l]);
    };
    if (!chained) {
        for (int l = 0; l < nl; l++) {
            if (l + 1 < nl) resize(l + 1);
            fast(l);
            octree(l);
        }
    } else {
        // level 0's cells and octree first (they read only the frame), then the first segment's levels, deepest
        // first (the slow middle-level octrees are on the critical path), their cells and octrees, then the later
        // segments' levels (each waits for its base level) with theirs
        fast(0);
        octree(0);
        for (int sgi = 0; sgi < chain->nseg; sgi++) {
            int lo = nl, hi = 0;
            for (int l = 1; l < nl; l++)
                if (cseg[l] == sgi) lo = std::min(lo, l), hi = std::max(hi, l);
            for (int l = hi; l >= lo; l--) chainl(l);
            for (int l = hi; l >= lo; l--) {
                fast(l);
                octree(l);
            }
        }
    }
    for (int l = 0; l < nl; l++) {
        const int cap = g.L[l].kp_cap;
        for (int i = 0; i < cap; i += 16)
            for (int f = 0; f < nframes; f++)
                push(kFlowDescribe, l, f, -1, g.L[l].kp_base + i, std::min(16, cap - i), ctr(f, 2, 0), l + 1, 1);
    }
    // LDS: the largest of the stages' carves (one 1024-thread workgroup per CU either way: its waves' registers
    // fill the CU), the rest of the CU's 160 KiB holding the octree's keys
    constexpr int kLds = 160 * 1024 - 64;
    const int need = std::max({16 * g.fast_wave_bytes, 16 * kDescWaveBytes + 256, 4 * rsq, (int)octree_lds_bytes(g.node_cap)});
    if (need > kLds) return false;
    plan.ntasks = (int)tasks.size();
    plan.nframes = nframes;
    plan.nctr = kFlowCtrBase + 4 * nl * nframes;
    plan.lds_bytes = kLds;
    const long long room = kLds - (long long)octree_lds_bytes(g.node_cap);
    const long long want = ((long long)g.max_level_cand + 7) & ~7LL;
    plan.lds_keys = room > 0 ? (int)std::min(want, (room / 6) & ~7LL) : 0;
    plan.rs_quarter = rsq;
    plan.blocks = std::max(1, blocks);
    return true;
}

FlowArgs flow_args(const ExtractBuffers& b, const uint8_t* d_frames, long long frame_pitch, int row_stride, int nframes,
                   orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int kp_cap) {
    FlowArgs A;
    std::memset(&A, 0, sizeof A);   // (compared bytewise by the caller: no indeterminate padding)
    A.g = b.d_geom;
    A.rcoef = b.d_rcoef;
    std::memcpy(A.roff.o, b.rcoef_off, sizeof A.roff.o);
    A.cells = b.d_cells;
    A.frames = d_frames;
    A.framePitch = frame_pitch;
    A.rowStride = row_stride;
    A.pyr = b.d_pyr;
    A.cands = b.d_cands;
    A.candFirst = b.d_candFirst;
    A.keys = b.d_keys;
    A.knode = b.d_knode;
    A.lvlKps = b.d_lvlKps;
    A.lvlCount = b.d_lvlCount;
    A.err = b.d_err;
    A.errHost = b.err_host;
    A.outK = d_kps;
    A.outD = d_desc;
    A.outN = d_counts;
    A.kpCap = kp_cap;
    A.tasks = b.d_flow;
    A.ntasks = b.flow.ntasks;
    A.nframes = nframes;
    A.ctr = b.d_flow_ctr;
    A.ldsKeys = b.flow.lds_keys;
    A.rsQuarter = b.flow.rs_quarter;
    A.stamps = b.d_flow_stamps;
    A.chainJobs = b.d_chain;
    for (int i = 0; i < ORBGPU_MAX_LEVELS; i++) A.chainSeg[i] = b.flow_chain.seg[i];
    return A;
}

hipError_t launch_extract(const Geom& g, const ExtractBuffers& b, const uint8_t* d_frames, long long frame_pitch,
                          int row_stride, int nframes, orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                          int kp_cap, hipStream_t stream, KernelMarker marker, void* user) {
    if (nframes <= 0) return hipSuccess;
    if (b.d_flow && b.flow.nframes == nframes) {   // the small-batch dataflow launch (k_extract_flow)
        // (its arguments are in device memory, b.d_flow_args, written by the caller for this call: flow_args())
        const bool fma = !(g.variant & ORB_VARIANT_NO_FMA);
        auto kern = g.fast_compact ? (fma ? k_extract_flow<48, true> : k_extract_flow<48, false>)
                                   : (fma ? k_extract_flow<kFastTilePitch, true> : k_extract_flow<kFastTilePitch, false>);
        if (marker) marker(user, ORB_K_FLOW, 1, stream);
        hipLaunchKernelGGL(kern, dim3(b.flow.blocks), dim3(kFlowThreads), (size_t)b.flow.lds_bytes, stream, b.d_flow_args);
        if (marker) marker(user, ORB_K_FLOW, 0, stream);
        return hipGetLastError();
    }
    auto resize = [&](int l, hipStream_t s) {
        // 32-row tiles where the level's source spans fit the LDS tile, else 16-row tiles, else the
        // untiled kernel (large scale factors): chosen per level from the geometry (LevelGeom::rs_tiled)
        const int t = g.L[l].rs_tiled;
        const ResizeCoef* cf = b.d_rcoef + b.rcoef_off[l];
        const bool gen = (g.variant & ORB_VARIANT_RESIZE_GENERIC) != 0;
        if (t & 3) {
            const int th = (t & 2) ? 32 : 16;
            const dim3 grid(cdiv(g.L[l].w, kRsTileW), cdiv(g.L[l].h, th), nframes);
            const size_t lds = (size_t)g.L[l].rs_span_rows * kRsPitch;
            // staging loads per thread: the level's own bound where two or three cover it, else the worst case
            const int kp = g.L[l].rs_chunks <= 512 ? 2 : g.L[l].rs_chunks <= 768 ? 3 : 0;
            auto kern = th == 32 ? (gen ? (kp == 2 ? k_resize_tiled<32, true, 2> : kp == 3 ? k_resize_tiled<32, true, 3>
                                                                                          : k_resize_tiled<32, true, 0>)
                                        : (kp == 2 ? k_resize_tiled<32, false, 2> : kp == 3 ? k_resize_tiled<32, false, 3>
                                                                                           : k_resize_tiled<32, false, 0>))
                                 : (gen ? (kp == 2 ? k_resize_tiled<16, true, 2> : k_resize_tiled<16, true, 0>)
                                        : (kp == 2 ? k_resize_tiled<16, false, 2> : k_resize_tiled<16, false, 0>));
            hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, b.d_geom, cf, l, d_frames, frame_pitch, row_stride,
                               b.d_pyr);
        } else {
            hipLaunchKernelGGL(gen ? k_resize<true> : k_resize<false>, dim3(cdiv(g.L[l].w, 256), cdiv(g.L[l].h, 4), nframes),
                               dim3(256), 0, s, b.d_geom, cf, l, d_frames, frame_pitch, row_stride, b.d_pyr);
        }
    };
    // FAST over cells [cbeg, cbeg + cnum) of every frame: one-wave workgroups, two (frame, cell) items per
    // wave (a workgroup's LDS is held until its slowest wave ends, so single waves waste the least of a
    // CU on uneven cells)
    auto fast = [&](int cbeg, int cnum, hipStream_t s, int* zero) {
        const int items = cnum * nframes;
        auto kern = g.fast_compact ? k_fast_wave<48> : k_fast_wave<kFastTilePitch>;
        // a single frame (the host path's latency) takes one cell per wave: twice the waves, half each one's chain
        const int ipw = nframes == 1 ? 1 : 2;
        hipLaunchKernelGGL(kern, dim3(cdiv(items, ipw)), dim3(64), (size_t)g.fast_wave_bytes, s, b.d_geom, b.d_cells,
                           d_frames, frame_pitch, row_stride, b.d_pyr, b.d_cands, b.d_candFirst, items, cbeg, cnum,
                           b.d_stamps, zero, ipw);
    };
    auto octree = [&](int lbase, int nl, hipStream_t s, int* err) {
        // a small batch (the host path's single frame, C5's 8-frame step) has fewer blocks than CUs, so the
        // keys get all the LDS a CU has (no global key scratch: at 4,000 features the node tables alone pass
        // the 52 KiB of the batch layout); larger batches keep 52 KiB (three blocks per CU).  512 threads in
        // both: 1024-thread blocks for small batches read 25.8 against 25.0 us per C5 frame after the
        // counting-sort rank (profiles/r06/octree_block_ab.txt; 256 threads 33.3 us)
        const bool one = nframes * nl <= 256;
        const int lk = one ? octree_lds_keys_whole_cu(g) : octree_lds_keys(g.node_cap);
        hipLaunchKernelGGL(k_octree<kOctreeThreads>, dim3(nframes, nl), dim3(kOctreeThreads),
                           octree_lds_bytes(g.node_cap) + (size_t)lk * 6, s, b.d_geom, b.d_cands, b.d_candFirst,
                           b.d_keys, b.d_knode, b.d_lvlKps, b.d_lvlCount, err, lk,
                           b.d_stamps ? b.d_stamps + (size_t)nframes * g.ncells * 8 : nullptr, lbase);
    };
    auto describe = [&](hipStream_t s) {
        unsigned long long* dst = b.d_stamps ? b.d_stamps + (size_t)nframes * (g.ncells * 8 + g.nlevels * 32) : nullptr;
        const int spw = nframes == 1 ? 1 : kDescSlotsPerWave;   // a single frame: one keypoint per wave
        const unsigned gx = cdiv(g.nkpcap, kDescWaves * spw);
        hipLaunchKernelGGL((g.variant & ORB_VARIANT_NO_FMA) ? k_describe<false> : k_describe<true>, dim3(gx * nframes), dim3(64 * kDescWaves), 0, s, b.d_geom, d_frames, frame_pitch,
                           row_stride, b.d_pyr, b.d_lvlKps, b.d_lvlCount, d_kps, d_desc, d_counts, kp_cap, dst, spw,
                           b.d_err, b.err_host);
    };
    int* zero = b.zero_err ? b.d_err : nullptr;
    hipError_t fe = hipSuccess;
    const bool forked = b.fork_s2 != nullptr && g.nlevels > 1;
    const int c0 = g.L[1].cell_base;   // level 0's cells
    if (forked) {
        // level 0's FAST -> octree reads only the input frame (ORBextractor.cc:1115, 1127): its own stream and
        // overflow flag (d_err[1], zeroed by its FAST launch), joined before k_describe
        if ((fe = hipEventRecord(b.ev_fork, stream)) != hipSuccess || (fe = hipStreamWaitEvent(b.fork_s2, b.ev_fork, 0)) != hipSuccess)
            return fe;
        fast(0, c0, b.fork_s2, b.d_err + 1);
        octree(0, 1, b.fork_s2, b.d_err + 1);
        if ((fe = hipEventRecord(b.ev_join, b.fork_s2)) != hipSuccess) return fe;
    }
    if (marker) marker(user, ORB_K_RESIZE, 1, stream);
    if (b.chain.nseg && nframes <= kChainMaxFrames) {   // the few-launch pyramid (k_pyramid_chain)
        RcoefOff ro;
        std::memcpy(ro.o, b.rcoef_off, sizeof ro.o);
        const bool gen = (g.variant & ORB_VARIANT_RESIZE_GENERIC) != 0;
        for (int l = 1; l <= b.chain.first_base; l++) resize(l, stream);
        for (int sgi = 0; sgi < b.chain.nseg; sgi++) {
            const ChainSegment& sg = b.chain.seg[sgi];
            hipLaunchKernelGGL(gen ? k_pyramid_chain<true> : k_pyramid_chain<false>, dim3(sg.njobs, nframes), dim3(256),
                               (size_t)sg.lds_bytes, stream, b.d_geom, b.d_rcoef, b.d_chain, sg, ro, d_frames, frame_pitch,
                               row_stride, b.d_pyr);
        }
    } else {
        for (int l = 1; l < g.nlevels; l++) resize(l, stream);
    }
    if (marker) marker(user, ORB_K_RESIZE, 0, stream);
    if (marker) marker(user, ORB_K_FAST, 1, stream);
    if (forked) fast(c0, g.ncells - c0, stream, zero);
    else fast(0, g.ncells, stream, zero);
    if (marker) marker(user, ORB_K_FAST, 0, stream);
    if (marker) marker(user, ORB_K_OCTREE, 1, stream);
    if (forked) octree(1, g.nlevels - 1, stream, b.d_err);
    else octree(0, g.nlevels, stream, b.d_err);
    if (marker) marker(user, ORB_K_OCTREE, 0, stream);
    if (forked && (fe = hipStreamWaitEvent(stream, b.ev_join, 0)) != hipSuccess) return fe;
    if (marker) marker(user, ORB_K_DESCRIBE, 1, stream);
    describe(stream);
    if (marker) marker(user, ORB_K_DESCRIBE, 0, stream);
    return hipGetLastError();
}

}  // namespace orbgpu
