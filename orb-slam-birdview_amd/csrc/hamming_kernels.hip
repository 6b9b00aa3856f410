// gfx950 Hamming-distance kernels for ORBmatcher (ORBmatcher.cc).  Two forms of the 256-bit distance
// (DescriptorDistance, ORBmatcher.cc:1647-1663):
//  - k_topk / k_triangulation: 8 x (v_xor_b32 + v_bcnt_u32_b32) per pair on the VALU, for the
//    vocabulary-gated candidate lists (CSR);
//  - k_top2_mfma: the all-pairs top-2 on the matrix cores, bits as +-4 e2m1 (fp4) values so that
//    q . t = 32 dist - 4096 exactly (v_mfma_f32_32x32x64_f8f6f4; bound: the dense FP4 MFMA peak),
//    or, as an A/B form, as +-1 int8 (v_mfma_i32_32x32x32_i8, the I8 peak).
// The selection logic that depends on the order of earlier accepted matches (SearchByBoW's taken set,
// SearchForInitialization's vMatchedDistance) is replayed on the host from these exact top-k lists
// (matcher.hip).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "orbgpu_internal.h"

namespace orbgpu {

namespace {

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}

constexpr int kMaxK = 8;

}  // namespace

/* Top-k per query over a CSR candidate list (or all trains), one wavefront per query.
 * Key = dist << 32 | candidate position: ascending key = ascending distance, then the reference's
 * iteration order (first wins on ties, as the strict '<' updates of ORBmatcher.cc:216-225 do). */
__global__ __launch_bounds__(256) void k_topk(const uint8_t* __restrict__ q, int nq, const uint8_t* __restrict__ t,
                                              int nt, const int2* __restrict__ ranges,
                                              const int* __restrict__ cand_idx, const int* __restrict__ thr, int k,
                                              int* __restrict__ out_dist, int* __restrict__ out_idx,
                                              int* __restrict__ out_nvalid) {
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (qi >= nq) return;
    const uint4* qp = reinterpret_cast<const uint4*>(q + (long long)qi * 32);
    const uint4 qa = qp[0], qb = qp[1];
    int c0 = 0, c1 = nt;
    if (ranges) {
        const int2 r = ranges[qi];
        c0 = r.x;
        c1 = r.y;
    }
    unsigned long long lst[kMaxK];
#pragma unroll
    for (int j = 0; j < kMaxK; j++) lst[j] = ~0ull;
    int nvalid = 0;
    for (int pos = c0 + lane; pos < c1; pos += 64) {
        const int ti = ranges ? cand_idx[pos] : pos;
        const uint4* tp = reinterpret_cast<const uint4*>(t + (long long)ti * 32);
        const int d = hamming256(qa, qb, tp[0], tp[1]);
        if (thr && thr[ti] <= d) continue;
        nvalid++;
        unsigned long long key = ((unsigned long long)d << 32) | (unsigned)(pos - c0);
#pragma unroll
        for (int j = 0; j < kMaxK; j++) {   // sorted insert (compare-swap chain)
            if (j < k && key < lst[j]) {
                const unsigned long long tmp = lst[j];
                lst[j] = key;
                key = tmp;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nvalid += __shfl_xor(nvalid, o);
    int head = 0;
    for (int j = 0; j < k; j++) {
        unsigned long long mine = ~0ull;
#pragma unroll
        for (int s = 0; s < kMaxK; s++)
            if (s == head) mine = lst[s];
        const unsigned long long m = wave_min_u64(mine);
        if (mine == m && m != ~0ull) head++;
        if (lane == 0) {
            int dd = -1, ii = -1;
            if (m != ~0ull) {
                dd = (int)(m >> 32);
                const int pos = (int)(m & 0xFFFFFFFFu) + c0;
                ii = ranges ? cand_idx[pos] : pos;
            }
            out_dist[(long long)qi * k + j] = dd;
            out_idx[(long long)qi * k + j] = ii;
        }
    }
    if (lane == 0 && out_nvalid) out_nvalid[qi] = nvalid;
}

// The window searches' candidate lists built on the device (SearchForInitialization :416-437,
// BirdviewMatch :1680-1700 / :1801-1812): Frame::GetFeaturesInArea(cx, cy, r, lv, lv) with lv = the
// query's octave (:494-547) over F2's grid in its CSR form.  The reference visits cells ix-major, iy
// inner, a cell's keypoints in vector order: that is increasing CSR slot, so a candidate's slot is its
// rank in vIndices2 and (dist, slot) breaks ties as the reference's first minimum does.  One wave per
// item; the rectangle's column ranges are contiguous slot runs.
__global__ __launch_bounds__(256) void k_window_topk(const uint8_t* __restrict__ q, const int* __restrict__ item_q,
                                                     const float2* __restrict__ centre, int nitems,
                                                     const orb_keypoint* __restrict__ kps1,
                                                     const uint8_t* __restrict__ t,
                                                     const orb_keypoint* __restrict__ kps2,
                                                     const int* __restrict__ cell_off,
                                                     const int* __restrict__ cell_idx, WinGrid wg,
                                                     const int* __restrict__ thr, int k, int* __restrict__ out_dist,
                                                     int* __restrict__ out_idx, int* __restrict__ out_nvalid) {
    constexpr int COLS = 64, ROWS = 48;   // Frame.h:39-40
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (qi >= nitems) return;
    const int i1 = item_q[qi];
    const uint4* qp = reinterpret_cast<const uint4*>(q + (long long)i1 * 32);
    const uint4 qa = qp[0], qb = qp[1];
    const int lv = kps1[i1].octave;
    float x, y;
    if (centre) {
        const float2 cc = centre[i1];
        x = cc.x;
        y = cc.y;
    } else {
        x = kps1[i1].x;
        y = kps1[i1].y;
    }
    const float r = wg.r;
    // cell rectangle, the reference's float expressions (-ffp-contract=off: no fused forms)
    const int nMinCellX = max(0, (int)floorf((x - wg.min_x - r) * wg.inv_w));
    const int nMaxCellX = min(COLS - 1, (int)ceilf((x - wg.min_x + r) * wg.inv_w));
    const int nMinCellY = max(0, (int)floorf((y - wg.min_y - r) * wg.inv_h));
    const int nMaxCellY = min(ROWS - 1, (int)ceilf((y - wg.min_y + r) * wg.inv_h));
    const bool empty = nMinCellX >= COLS || nMaxCellX < 0 || nMinCellY >= ROWS || nMaxCellY < 0;
    unsigned long long lst[kMaxK];
#pragma unroll
    for (int j = 0; j < kMaxK; j++) lst[j] = ~0ull;
    int nvalid = 0;
    if (!empty) {
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
            const int s0 = cell_off[ix * ROWS + nMinCellY], s1 = cell_off[ix * ROWS + nMaxCellY + 1];
            for (int s = s0 + lane; s < s1; s += 64) {
                const int ti = cell_idx[s];
                const orb_keypoint kp = kps2[ti];
                if (kp.octave != lv) continue;                                        // :518-525 with min = max = lv
                if (!(fabsf(kp.x - x) < r && fabsf(kp.y - y) < r)) continue;          // :530-533
                const uint4* tp = reinterpret_cast<const uint4*>(t + (long long)ti * 32);
                const int d = hamming256(qa, qb, tp[0], tp[1]);
                if (thr && thr[ti] <= d) continue;
                nvalid++;
                unsigned long long key = ((unsigned long long)d << 32) | (unsigned)s;
#pragma unroll
                for (int j = 0; j < kMaxK; j++) {   // sorted insert (compare-swap chain)
                    if (j < k && key < lst[j]) {
                        const unsigned long long tmp = lst[j];
                        lst[j] = key;
                        key = tmp;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nvalid += __shfl_xor(nvalid, o);
    int head = 0;
    for (int j = 0; j < k; j++) {
        unsigned long long mine = ~0ull;
#pragma unroll
        for (int s = 0; s < kMaxK; s++)
            if (s == head) mine = lst[s];
        const unsigned long long m = wave_min_u64(mine);
        if (mine == m && m != ~0ull) head++;
        if (lane == 0) {
            int dd = -1, ii = -1;
            if (m != ~0ull) {
                dd = (int)(m >> 32);
                ii = cell_idx[(int)(m & 0xFFFFFFFFu)];
            }
            out_dist[(long long)qi * k + j] = dd;
            out_idx[(long long)qi * k + j] = ii;
        }
    }
    if (lane == 0 && out_nvalid) out_nvalid[qi] = nvalid;
}

/* Slices of one (query set, train set) pair's top-2 (k_top2_mfma with gridDim.y > 1) are merged here:
 * keys dist << 16 | train index compose by min (first index on ties) and second = the second-smallest
 * key.  Counts may be read on the device (an extraction batch's d_counts), so a whole batch of frame
 * pairs needs no host round trip. */
__global__ __launch_bounds__(256) void k_top2b_merge(Top2Batch a, int nslices, const uint2* __restrict__ part,
                                                     int* __restrict__ best_o, int* __restrict__ idx_o,
                                                     int* __restrict__ second_o) {
    const int p = blockIdx.y;
    const int2 fr = a.frames ? a.frames[p] : make_int2(0, 0);
    const int nq = a.counts ? a.counts[fr.x] : a.nq, nt = a.counts ? a.counts[fr.y] : a.nt;
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= nq) return;
    const int used = min(nslices, (nt + a.slice - 1) / a.slice);   // slices past nt were never written
    unsigned b = 0xFFFFFFFFu, s2 = 0xFFFFFFFFu;
    for (int s = 0; s < used; s++) {
        const uint2 v = part[((long long)p * nslices + s) * a.out_stride + qi];
        s2 = min(min(s2, v.y), max(b, v.x));
        b = min(b, v.x);
    }
    const long long o = (long long)p * a.out_stride + qi;
    best_o[o] = b == 0xFFFFFFFFu ? 257 : (int)(b >> 16);
    idx_o[o] = b == 0xFFFFFFFFu ? -1 : (int)(b & 0xFFFF);
    second_o[o] = s2 == 0xFFFFFFFFu ? 257 : (int)(s2 >> 16);
}

/* The same all-pairs top-2 on the matrix cores.  With descriptor bits as +-1 int8 values,
 * q . t = 256 - 2 popcount(q ^ t), so a tile of Hamming distances is one 32x32 i8 GEMM over K = 256:
 * eight v_mfma_i32_32x32x32_i8 in one accumulator chain.  A workgroup owns 128 queries (4 waves x 32,
 * the B operand, expanded once into registers as -16 / +16, so the tile's results come out as
 * tile-local keys, see kc) and walks its train slice in tiles of 32 (the A operand: trains expanded to
 * +-1 once per launch by k_expand_pm1, copied into LDS, double-buffered; rows padded to 272 bytes so
 * the 16-byte fragment reads are conflict-free).  The accumulator puts trains on the registers and
 * queries on the lanes (row = (r&3) + 8(r>>2) + 4(lane>>5), column = lane & 31), so the top-2 update is
 * lane-local; the two lane halves are merged at the end.  Running keys: dist << 16 | train index, so
 * min keeps the first index on ties (SearchByBoW's strict `<`).  The accumulators live in VGPRs
 * (-amdgpu-mfma-vgpr-form: no v_accvgpr_read per result). */
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));
constexpr int kMfTr = 32;      // trains per tile (MFMA rows)
constexpr int kMfPitch = 272;  // LDS bytes per expanded train (256 + 16)
constexpr int kMfPitch4 = 144; // the same for the fp4 form (128 + 16: 36 dwords, odd multiple of 4, so the 16 lanes
                               // of a ds_read_b128 group hit 16 distinct 4-bank slots)

__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {   // v_med3_u32
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));   // (not volatile: schedulable)
    return r;
}

// 4 descriptor bits -> 4 bytes: +1 where the bit is set, -1 (0xFF) where it is clear
__device__ __forceinline__ int pm1x4(uint32_t n) {
    const uint32_t s = __umul24(n & 15u, 0x00204081u) & 0x01010101u;   // bit i -> byte i (no carries)
    const uint32_t m = (s << 8) - s;                                    // 0xFF in the set bytes
    return (int)((m & s) | ~m);
}
__device__ __forceinline__ v4i_t pm1x16(uint32_t w) {   // bits 0..15 of w -> 16 int8
    v4i_t r;
    r.x = pm1x4(w);
    r.y = pm1x4(w >> 4);
    r.z = pm1x4(w >> 8);
    r.w = pm1x4(w >> 12);
    return r;
}
/* The pairs' train descriptors expanded to +-1 int8 once per launch (thread = one descriptor dword ->
 * 32 bytes), so k_top2_mfma's train tiles are plain copies: without it every query workgroup of a pair
 * re-expands every train tile (~40 VALU per thread and tile, more than the tile's top-2 updates). */
__global__ __launch_bounds__(256) void k_expand_pm1(Top2Batch a, int max_nt, int slot0) {
    // slot0 + blockIdx.y = expansion slot: one per distinct train frame (a.tx_frames) or, without that list, one
    // per pair
    const int p = slot0 + blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const int row = i >> 3, s = i & 7;
    const int tf = a.tx_frames ? a.tx_frames[p] : (a.frames ? a.frames[p].y : 0);
    const int nt = a.counts ? a.counts[tf] : a.nt;
    if (row >= min(nt, max_nt)) return;
    const uint32_t w = reinterpret_cast<const uint32_t*>(a.t + ((long long)tf * a.t_stride + row) * 32)[s];
    v4i_t* d = reinterpret_cast<v4i_t*>(const_cast<uint8_t*>(a.tx) + ((long long)p * a.tx_stride + row) * 256 + 32 * s);
    d[0] = pm1x16(w);
    d[1] = pm1x16(w >> 16);
}

// 8 bits -> bit 0 of 8 nibbles (bit i -> nibble i)
__device__ __forceinline__ uint32_t spread8_nib(uint32_t b) {
    uint32_t x = b & 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    return (x | (x << 3)) & 0x11111111u;
}
// 32 descriptor bits -> 32 e2m1 (fp4) values, element e = bit e (byte e / 2, low nibble first): X where the bit
// is clear, the negated X where it is set (the sign is nibble bit 3).  X = 0x6 (+4) for the trains, 0xE (-4) for
// the queries, so q t = -16 for equal bits and +16 for different ones.
template <uint32_t X>
__device__ __forceinline__ v4i_t fp4x32(uint32_t w) {
    return v4i_t{(int)(X * 0x11111111u ^ (spread8_nib(w) << 3)), (int)(X * 0x11111111u ^ (spread8_nib(w >> 8) << 3)),
                 (int)(X * 0x11111111u ^ (spread8_nib(w >> 16) << 3)), (int)(X * 0x11111111u ^ (spread8_nib(w >> 24) << 3))};
}
/* The fp4 form of k_expand_pm1: 128 bytes per train (descriptor dword s -> bytes 16 s .. 16 s + 15), at the
 * same slot rows as the int8 form (a.tx rows of 256 bytes, the first half used). */
__global__ __launch_bounds__(256) void k_expand_fp4(Top2Batch a, int max_nt, int slot0) {
    const int p = slot0 + blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const int row = i >> 3, s = i & 7;
    const int tf = a.tx_frames ? a.tx_frames[p] : (a.frames ? a.frames[p].y : 0);
    const int nt = a.counts ? a.counts[tf] : a.nt;
    if (row >= min(nt, max_nt)) return;
    const uint32_t w = reinterpret_cast<const uint32_t*>(a.t + ((long long)tf * a.t_stride + row) * 32)[s];
    v4i_t* d = reinterpret_cast<v4i_t*>(const_cast<uint8_t*>(a.tx) + ((long long)p * a.tx_stride + row) * 128 + 16 * s);
    d[0] = fp4x32<0x6u>(w);
}

// 4 query bits -> 4 bytes of +-S (S = 16 or 32): -S where the bit is set, +S where it is clear
template <int S>
__device__ __forceinline__ int pmSx4(uint32_t n) {
    const uint32_t s = __umul24(n & 15u, 0x00204081u) & 0x01010101u;
    const uint32_t m = (s << 8) - s;                                    // 0xFF in the set bytes
    return (int)((uint32_t)S * 0x01010101u ^ (m & ((uint32_t)(256 - 2 * S) * 0x01010101u)));
}
template <int S>
__device__ __forceinline__ v4i_t pmSx16(uint32_t w) {
    return v4i_t{pmSx4<S>(w), pmSx4<S>(w >> 4), pmSx4<S>(w >> 8), pmSx4<S>(w >> 12)};
}

// the top-2's step (k_top2_mfma top2f): two keys per min3 / med3 / min (1), or one per med3 / min (0, r04 v10)
#ifndef ORBGPU_TOP2_PAIRS
#define ORBGPU_TOP2_PAIRS 1
#endif
constexpr bool TOP2_PAIRS = ORBGPU_TOP2_PAIRS != 0;

// The 16 key bits of an f16 top-2 result, read from the whole register and masked.  hipcc (ROCm 7.2) takes the
// upper half of a 16-bit VALU result (v_min_f16 / v_med3_f16) as zero and folds the zero-extension into the
// key's shift; on gfx950 that half keeps whatever the register held, and builds whose allocator had put a 32-bit
// value there lost second-best keys (wrong seconds in 4-11 of 2,006 queries, deterministic per build; an
// explicit MFMA wait-state pad and keeping operands live changed nothing; this mask fixed every form,
// profiles/r04/v6_hamming_ab.txt).  The asm hides the assumption, so the mask is kept.
__device__ __forceinline__ unsigned f16_bits(_Float16 x) {
    unsigned r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r & 0xFFFFu;
}

/* NS 32-train subtiles per stage (one accumulator chain each).  With the queries scaled to -S / +S,
 * S = 16 NS, and the accumulators seeded with 256 S + subtile * 32 + row, every result is the stage-local key
 * dist * 32 NS + (subtile * 32 + row): the top-2 of a stage's 16 NS keys per lane runs in one med3 / min
 * pass and is merged into the running keys once per stage (NS = 2: one merge per 64 trains instead of
 * two). */
/* FP4: the same top-2 on v_mfma_f32_32x32x64_f8f6f4 with e2m1 operands (the FP4 rate: twice the i8 MFMA's K per
 * instruction in the same cycles, MI355X_MICROARCH.md §Matrix cores): trains +-4, queries -+4, so q . t = 32 dist -
 * 4096 exactly (integers, f32 accumulation), four MFMAs per 32 x 32 tile, 128 expanded bytes per train.  The
 * accumulator is seeded with 2^23 + 4096 + stage row: every result lies in [2^23, 2^24), where an f32's low
 * mantissa bits are the integer itself, so the low 16 bits of its bit pattern are the same key dist << 5 | row as
 * the int8 form's.  The K order inside a fragment does not matter: both operands use one bit -> element map. */
template <bool PRE, int NW, int NS, bool PIPE, int LA = 0, bool FP4 = false>   // PRE: trains pre-expanded by
                                                 // k_expand_pm1 / k_expand_fp4 (a.tx); NW waves of 32 queries; PIPE:
                                                 // stage j's MFMAs beside stage j-1's top-2; LA > 0: each A-fragment
                                                 // read issued LA MFMAs ahead of its MFMA
__global__ __launch_bounds__(NW * 64) void k_top2_mfma(Top2Batch a, uint2* __restrict__ part, int* __restrict__ best_o,
                                                       int* __restrict__ idx_o, int* __restrict__ second_o,
                                                       int vblocks) {
    constexpr int NT = NW * 64, QB = NW * 32, TR = NS * kMfTr;   // threads, queries, trains per stage
    constexpr int TRB = FP4 ? 128 : 256;                         // expanded bytes per train
    constexpr int PIT = FP4 ? kMfPitch4 : kMfPitch;              // their LDS pitch
    constexpr int KS = FP4 ? 4 : 8;                              // MFMAs per 32-train subtile (K = 256)
    constexpr int NCH = TRB / 16 * TR;                           // 16-byte chunks of a stage
    constexpr int CH = NCH >= NT ? NCH / NT : 1;  // chunks each staging thread stages
    constexpr int SACT = NCH / CH;                // staging threads (FP4 with 8 waves: the first four waves)
    constexpr int SC = 16 * NS;        // query scale (int8 form)
    constexpr int KB = 5 + (NS == 2);  // stage-local key: dist << KB | stage row
    constexpr int VG = FP4 ? 9 : NS == 2 ? 5 : 6; // VALU issued after each MFMA of the pipelined stage
    static_assert(CH >= 1 && CH <= 4, "staging chunks");
    static_assert(!FP4 || PRE == false || NS == 1, "fp4 with pre-expanded trains: one subtile per stage");
    using acc_t = typename std::conditional<FP4, v16f_t, v16i_t>::type;
    __shared__ __attribute__((aligned(16))) uint8_t s_t[2][TR * PIT];
    // fp4 without pre-expanded trains: byte -> 8 e2m1 nibbles (+4 where the bit is clear, -4 where set), so a staged
    // train dword costs four LDS lookups instead of ~32 VALU
    __shared__ uint32_t s_lut[FP4 && !PRE ? 256 : 1];
    if (FP4 && !PRE)
        for (int i = threadIdx.x; i < 256; i += NT) s_lut[i] = 0x66666666u ^ (spread8_nib((uint32_t)i) << 3);
    // 1-D grid of (pair, slice, query block), query block fastest.  Blocks are dealt round-robin over the 8
    // XCDs (b and b + 8 share one), so XCD x takes a contiguous run of that sequence: the query blocks of a
    // pair, which all stream the same expanded trains, then share one L2 (dealt round-robin, every pair's
    // 512 KB of C3 trains was fetched into all eight L2s: PMC 1.14 GB per 255-pair launch,
    // profiles/r04/v1_hamming.json)
    // Persistent form (vblocks > gridDim.x): workgroup w runs the virtual blocks w, w + G, w + 2G, ... of a
    // vblocks-block grid (G = gridDim.x, a multiple of 8, so a virtual block keeps its XCD): no per-block launch
    // and drain, one workgroup per slot for the whole launch.
    for (int vb = blockIdx.x; vb < vblocks; vb += gridDim.x) {
    __syncthreads();   // (a previous item's last LDS reads precede this item's staging)
    const int nb = vblocks, xq = nb >> 3, xr = nb & 7, xcd = vb & 7, xj = vb >> 3;
    const int lb = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + xj;
    const int qbi = lb % a.qblocks, rest = lb / a.qblocks;
    const int sli = rest % a.nslices, p = rest / a.nslices;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int2 fr = a.frames ? a.frames[p] : make_int2(0, 0);
    const int nq = a.counts ? a.counts[fr.x] : a.nq, nt = a.counts ? a.counts[fr.y] : a.nt;
    const int qblk = qbi * QB;
    if (qblk >= nq) continue;   // whole workgroup
    const int t0 = sli * a.slice, t1 = min(nt, t0 + a.slice);
    const int h = lane >> 5, c = lane & 31;
    const int qi = qblk + wv * 32 + c;
    // B operand: K-step s = descriptor dword s, lane half h = its bits 16h .. 16h+15 (fp4: K-step s = dwords 2s
    // and 2s + 1, lane half h = dword 2s + h)
    v4i_t qf[KS];
    {
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
        if (qi < nq) {
            const uint4* qp = reinterpret_cast<const uint4*>(a.q + ((long long)fr.x * a.q_stride + qi) * 32);
            q0 = qp[0];
            q1 = qp[1];
        }
        const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const uint32_t hm = h ? 0xFFFFFFFFu : 0u;   // (a select, not qd[2 s + h]: a dynamic index goes to scratch)
        if (FP4) {
#pragma unroll
            for (int s = 0; s < KS; s++) qf[s] = fp4x32<0xEu>(qd[2 * s] ^ ((qd[2 * s] ^ qd[2 * s + 1]) & hm));
        } else {
#pragma unroll
            for (int s = 0; s < KS; s++) qf[s] = pmSx16<SC>(qd[s] >> (16 * h));
        }
    }
    const uint32_t* __restrict__ T = reinterpret_cast<const uint32_t*>(a.t + (long long)fr.y * a.t_stride * 32);
    // PRE: this pair's expanded trains through a buffer descriptor (SGPRs), 32-bit offsets
    const int txs = a.tx_slot ? a.tx_slot[p] : p;   // the pair's expansion slot
    const uint64_t txb = PRE ? reinterpret_cast<uint64_t>(a.tx + (long long)txs * a.tx_stride * TRB) : 0;
    const auto TXR = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(txb >> 32)) << 32) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)txb)),
        0, 0x7FFFFFFF, 0x00020000);
    // staging: thread -> stage row er, chunks ec .. ec + CH - 1 (16 expanded bytes = 16 descriptor bits each)
    const int er = (tid * CH) / (TRB / 16), ec = (tid * CH) % (TRB / 16);
    const bool stager = SACT == NT || tid < SACT;   // (wave-uniform)
    struct Chunk {
        uint32_t w[(CH + 1) / 2];   // !PRE: the descriptor dwords holding the chunks' bits
        v4i_t x[CH];                // PRE: the expanded bytes
    };
    auto fetch = [&](int row) -> Chunk {
        Chunk k;
        if (PRE) {
#pragma unroll
            for (int i = 0; i < CH; i++)
                k.x[i] = stager ? __builtin_bit_cast(v4i_t, __builtin_amdgcn_raw_buffer_load_b128(TXR, row * TRB + 16 * (ec + i), 0, 0))
                                : v4i_t{0, 0, 0, 0};
        } else if (FP4) {   // chunk ec = descriptor dword ec (32 bits -> 16 expanded bytes)
            k.w[0] = stager ? T[(long long)row * 8 + ec] : 0u;
        } else {
#pragma unroll
            for (int i = 0; i < (CH + 1) / 2; i++) k.w[i] = T[(long long)row * 8 + (ec >> 1) + i];
        }
        return k;
    };
    auto stage = [&](int buf, const Chunk& k) {
        if (!stager) return;
        v4i_t* d = reinterpret_cast<v4i_t*>(&s_t[buf][er * PIT + ec * 16]);
        if (FP4 && !PRE) {
            const uint32_t w = k.w[0];
            d[0] = v4i_t{(int)s_lut[w & 255u], (int)s_lut[(w >> 8) & 255u], (int)s_lut[(w >> 16) & 255u], (int)s_lut[w >> 24]};
            return;
        }
#pragma unroll
        for (int i = 0; i < CH; i++) d[i] = PRE ? k.x[i] : pm1x16(k.w[i >> 1] >> (16 * ((ec + i) & 1)));
    };
    unsigned b = 0xFFFFFFFFu, s2 = 0xFFFFFFFFu;
    // the MFMA's initial accumulators: 256 SC + subtile * 32 + row, so that every result is already its
    // stage-local key 256 SC - SC dot + subtile * 32 + row = dist << KB | stage row (dot = 256 - 2 dist: the sum
    // over the 256 bits of (+-1 train bit) x (-+1 query bit)).  A key is < 2^15, so its low half is a finite
    // positive f16 bit pattern ordered like the integer (those below 0x400 are f16 denormals, which gfx950 keeps):
    // the top-2 runs in v_med3_f16 + v_min_f16 (VOP2, full rate: 2.5 cycles per wave instruction against 4.3 for
    // v_min_u32 / v_med3_u32, profiles/r02/valu_rate.txt; compiler builtins the scheduler can interleave with the
    // MFMAs; the file builds with -fno-honor-nans so that v_min_f16 needs no canonicalising v_max_f16).
    acc_t kc[NS];
#pragma unroll
    for (int u = 0; u < NS; u++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int row = 32 * u + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (FP4) kc[u][r] = (float)(8388608 + 4096 * NS + row);   // exact: 2^23 + 4096 NS + row (see above)
            else kc[u][r] = 256 * SC + row;
        }
    const int nst = t1 > t0 ? (t1 - t0 + TR - 1) / TR : 0;   // stages (uniform)
    // e8m0 block scales (byte 0 of a register: 127 = 2^0, 128 = 2^1), from registers (a constant scale operand is
    // read as an f32 inline constant, MI355X builtin note in ck's amd_xdlops.hpp); used by the fp4 NS = 2 form only
    int sc_a = 127, sc_b = 128;
    if (FP4 && NS == 2) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(sc_a) : "v"(sc_a));
        asm volatile("v_mov_b32 %0, %1" : "=v"(sc_b) : "v"(sc_b));
    }
    auto mfma_stage = [&](int buf, acc_t (&acc)[NS]) {
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const uint8_t* A = &s_t[buf][(32 * u + c) * PIT + 16 * h];
            acc[u] = kc[u];
#pragma unroll
            for (int s = 0; s < KS; s++) {   // one chain per subtile: the other waves on the SIMD hide its latency
                const v4i_t av = *reinterpret_cast<const v4i_t*>(A + 32 * s);
                if constexpr (FP4) {
                    const v8i_t a8 = {av[0], av[1], av[2], av[3], 0, 0, 0, 0};
                    const v8i_t b8 = {qf[s][0], qf[s][1], qf[s][2], qf[s][3], 0, 0, 0, 0};
                    // cbsz = blgp = 4: both operands e2m1; zero scales select the unscaled form (4-VGPR operands)
                    if (NS == 1)
                        acc[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[u], 4, 4, 0, 0, 0, 0);
                    else   // block scale 2^1 on the queries: q . t = 64 dist - 8192, keys dist << 6 | row of 64
                        acc[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[u], 4, 4, 0, sc_a, 0, sc_b);
                } else {
                    acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, qf[s], acc[u], 0, 0, 0);
                }
            }
        }
    };
    // a stage's top-2 by med3 / min (2 ops per distance), merged into the running keys dist << 16 | train
    // index once per stage.  A full stage gives every lane 16 NS keys: no tests.
    constexpr unsigned RM = (1u << KB) - 1;
    auto top2f = [&](const acc_t (&acc)[NS], unsigned& lbu, unsigned& lsu, auto keep) {
        const _Float16 inf = __builtin_bit_cast(_Float16, (unsigned short)0x7C00u);
        _Float16 lbh = inf, lsh = inf;
        auto key_of = [&](int u, int r) {
            // (via a scalar: clang's __builtin_bit_cast of an ext_vector element reads element 0)
            const auto kv = acc[u][r];
            const int ki = __builtin_bit_cast(int, kv);
            return keep(u, r) ? __builtin_bit_cast(_Float16, (unsigned short)ki) : inf;
        };
        if constexpr (TOP2_PAIRS) {
            // two keys per step, 3 ops: best' = min3(best, x, y), second' = min(second, med3(best, x, y)) -- the
            // second smallest of {best <= second, x, y} in every order of the four (a stage's keys are distinct)
#pragma unroll
            for (int u = 0; u < NS; u++)
#pragma unroll
                for (int r = 0; r < 16; r += 2) {
                    const _Float16 x = key_of(u, r), y = key_of(u, r + 1);
                    lsh = __builtin_fminf16(lsh, __builtin_amdgcn_fmed3h(lbh, x, y));
                    lbh = __builtin_fminf16(__builtin_fminf16(lbh, x), y);
                }
        } else {
#pragma unroll
            for (int u = 0; u < NS; u++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const _Float16 key = key_of(u, r);
                    lsh = __builtin_amdgcn_fmed3h(lbh, key, lsh);
                    lbh = __builtin_fminf16(lbh, key);
                }
        }
        lbu = f16_bits(lbh);
        lsu = f16_bits(lsh);
    };
    auto reduce_full = [&](const acc_t (&acc)[NS], int tb) {
        unsigned lbt, lst;
        top2f(acc, lbt, lst, [](int, int) { return true; });
        const unsigned gb = ((lbt << (16 - KB)) & 0xFFFF0000u) + (lbt & RM) + (unsigned)tb;
        s2 = umed3(b, gb, s2);
        b = min(b, gb);
        // the second's index is never output: dist << 16 | 0xFFFF orders it after any equal best
        s2 = min(s2, (lst << (16 - KB)) | 0xFFFFu);
    };
    auto reduce_any = [&](const acc_t (&acc)[NS], int tb) {   // the slice's last stage, maybe partial
        if (tb + TR <= t1) {
            reduce_full(acc, tb);
            return;
        }
        unsigned lbt, lst;
        top2f(acc, lbt, lst, [&](int u, int r) { return tb + 32 * u + (r & 3) + 8 * (r >> 2) + 4 * h < t1; });
        constexpr unsigned kInf = 0x7C00u;   // f16 +inf: a lane without keys
        if (lbt != kInf) {   // (only a partial stage leaves a lane without keys)
            const unsigned gb = ((lbt << (16 - KB)) & 0xFFFF0000u) + (lbt & RM) + (unsigned)tb;
            s2 = umed3(b, gb, s2);
            b = min(b, gb);
            if (lst != kInf) s2 = min(s2, (lst << (16 - KB)) | 0xFFFFu);
        }
    };
    if (nst > 0) {
        // rows past the slice load the slice's last row (their keys are masked): no zeroing, no branch
        stage(0, fetch(min(t0 + er, t1 - 1)));
        __syncthreads();
        if (!PIPE) {
            for (int j = 0; j < nst; j++) {
                const int tb = t0 + TR * j;
                const bool more = j + 1 < nst;
                Chunk wn;
                if (more) wn = fetch(min(tb + TR + er, t1 - 1));
                acc_t acc[NS];
                mfma_stage(j & 1, acc);
                reduce_any(acc, tb);
                if (more) stage((j + 1) & 1, wn);
                __syncthreads();
            }
        } else {
            // software-pipelined: stage j's MFMA chains are issued beside stage j-1's top-2, so one wave keeps
            // the matrix pipe and the VALU busy together (every stage but the last is full)
            acc_t accA[NS], accB[NS];
            auto step = [&](int j, acc_t (&accNew)[NS], const acc_t (&accOld)[NS]) {
                // LA > 0: the next stage's rows are fetched and staged unconditionally (after the last stage they
                // are the slice's last row again, written to the buffer no one reads any more): no branch splits
                // the step's scheduling region
                const bool more = LA > 0 || j + 1 < nst;
                Chunk wn;
                if (more) wn = fetch(min(t0 + TR * (j + 1) + er, t1 - 1));
                if (LA > 0) __builtin_amdgcn_sched_barrier(0);   // the global loads issue first, their latency under the step
                mfma_stage(j & 1, accNew);
                reduce_full(accOld, t0 + TR * (j - 1));
                // interleave: the A-fragment reads ahead, then each MFMA followed by a share of the top-2
if (LA == 0) {
#pragma unroll
                    for (int i = 0; i < KS * NS; i++) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one ds_read
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
                        __builtin_amdgcn_sched_group_barrier(0x002, VG, 0);  // VG VALU
                    }
                } else {
                    // the first LA reads up front, then read i + LA after MFMA i: LA reads in flight while the
                    // chain runs (read i -> wait -> MFMA i exposes the LDS latency on every MFMA)
                    __builtin_amdgcn_sched_group_barrier(0x100, LA, 0);
#pragma unroll
                    for (int i = 0; i < KS * NS; i++) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        if (i + LA < KS * NS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, VG, 0);
                    }
                }
                if (more) stage((j + 1) & 1, wn);
                __syncthreads();
            };
            {
                const bool more = 1 < nst;
                Chunk wn;
                if (more) wn = fetch(min(t0 + TR + er, t1 - 1));
                mfma_stage(0, accA);
                if (more) stage(1, wn);
                __syncthreads();
            }
            int j = 1;
            for (; j + 1 < nst; j += 2) {
                step(j, accB, accA);
                step(j + 1, accA, accB);
            }
            if (j < nst) {
                step(j, accB, accA);
                reduce_any(accB, t0 + TR * (nst - 1));
            } else {
                reduce_any(accA, t0 + TR * (nst - 1));
            }
        }
    }
    // the two lane halves hold different train rows of the same query
    const unsigned ob = __shfl_xor(b, 32), os = __shfl_xor(s2, 32);
    s2 = min(min(s2, os), max(b, ob));
    b = min(b, ob);
    if (h == 0 && qi < nq) {
        const long long o = (long long)p * a.out_stride + qi;
        if (a.nslices == 1) {
            best_o[o] = b == 0xFFFFFFFFu ? 257 : (int)(b >> 16);
            idx_o[o] = b == 0xFFFFFFFFu ? -1 : (int)(b & 0xFFFF);
            second_o[o] = s2 == 0xFFFFFFFFu ? 257 : (int)(s2 >> 16);
        } else {
            part[((long long)p * a.nslices + sli) * a.out_stride + qi] = make_uint2(b, s2);
        }
    }
    }   // virtual blocks
}

// k_top2_mfma's configuration (ORBGPU_TOP2, an A/B switch; default "8fx"): '4' / '8' waves per workgroup,
// '1' / '2' subtiles per stage, 'p' software-pipelined stages, 'P' persistent workgroups (one per slot), 'o' the
// expansion of the pairs after the first eighth overlapped with the first eighth's top-2 (Top2Overlap), 'l' / 'L' (with 'p') A-fragment
// reads 2 / 4 MFMAs ahead, 'f' the fp4 form (8 waves, one subtile), 'x' (with 'f') no expansion
// kernel: each stage's train dwords are expanded while staged (k_top2_mfma<false, ..., FP4>; with 'p' too: "8fxp",
// 171-173 us against 157-160, profiles/r04/v14_top2_pairs.txt)
struct Top2Cfg {   // default "8fx": the fp4 form, unpipelined, trains expanded while staged (r04 A/B,
                   // profiles/r04/v9_hamming_ab.txt: 161-162 us; with the expansion kernel 181; pipelined 188; int8 262)
    int waves = 8, stage = 1, la = 0;
    bool pipe = false, persist = false, overlap = false, fp4 = true, noexp = true;
};
static const Top2Cfg& top2_cfg() {
    static const Top2Cfg c = [] {
        Top2Cfg t;
        const char* e = std::getenv("ORBGPU_TOP2");
        if (!e || !*e) return t;
        t.waves = std::strchr(e, '4') ? 4 : 8;
        t.stage = std::strchr(e, '2') ? 2 : 1;
        t.pipe = std::strchr(e, 'p') != nullptr;
        t.persist = std::strchr(e, 'P') != nullptr;
        t.overlap = std::strchr(e, 'o') != nullptr;
        t.la = std::strchr(e, 'L') ? 4 : std::strchr(e, 'l') ? 2 : 0;
        t.fp4 = std::strchr(e, 'f') != nullptr;
        t.noexp = std::strchr(e, 'x') != nullptr;
        if (t.fp4 && !t.noexp) t.stage = 1;   // fp4: one subtile, or two with '2' and 'x' (scaled queries)
        if (t.fp4 && !(t.noexp && t.waves == 4)) t.waves = 8;   // 8 waves, or 4 with '4' and 'x' 
        return t;
    }();
    return c;
}
static int top2_waves() { return top2_cfg().waves; }
bool top2_overlap_enabled() { return top2_cfg().overlap; }
bool top2_fp4_enabled() { return top2_cfg().fp4; }
bool top2_needs_expansion() { return !(top2_cfg().fp4 && top2_cfg().noexp); }
int top2_queries_per_block() { return 32 * top2_cfg().waves; }

int top2_batch_slices(int npairs, int max_nq, int max_nt) {
    npairs = std::max(npairs, 1);
    const int qwaves = std::max(1, (max_nq + 63) / 64);
    int ns = (8192 + npairs * qwaves - 1) / (npairs * qwaves);   // aim for >= 8192 wavefronts
    ns = std::min(ns, std::max(1, (max_nt + 31) / 32));          // >= 32 trains per slice
    return std::max(ns, 1);
}

// Train slice length of one launch: >= 8192 waves, slices of whole 32-train tiles, at most
// top2_batch_slices of them (the partial buffer is sized for that many).  (max_nt == 0: one empty slice of
// one tile width, so that nothing divides by zero.)
static int top2_slice_len(int npairs, int max_nq, int max_nt) {
    const int ns = top2_batch_slices(npairs, max_nq, max_nt);
    const int nw = top2_waves(), qb = (max_nq + 32 * nw - 1) / (32 * nw);
    const int wg = 8192 / nw;
    int want = std::max(1, (wg + qb * npairs - 1) / (qb * npairs));
    want = std::min({want, ns, std::max(1, (max_nt + kMfTr - 1) / kMfTr)});
    return std::max(((max_nt + want - 1) / want + kMfTr - 1) / kMfTr * kMfTr, kMfTr);
}

int top2_launch_slices(int npairs, int max_nq, int max_nt) {
    if (npairs <= 0 || max_nq <= 0 || max_nt < 0) return 0;
    return std::max(1, (max_nt + top2_slice_len(npairs, max_nq, max_nt) - 1) / top2_slice_len(npairs, max_nq, max_nt));
}

hipError_t launch_hamming_top2_batch(const Top2Batch& a0, int npairs, int max_nq, int max_nt, int* d_best,
                                     int* d_best_idx, int* d_second, uint2* d_part, hipStream_t stream,
                                     const Top2Overlap* ov) {
    if (npairs <= 0 || max_nq <= 0) return hipSuccess;
    if (max_nt > 65535) return hipErrorInvalidValue;   // keys hold a 16-bit train index
    Top2Batch a = a0;
    const Top2Cfg& cfg = top2_cfg();
    const int nw = cfg.waves, ns = cfg.stage;
    const int qb = (max_nq + 32 * nw - 1) / (32 * nw);
    a.slice = top2_slice_len(npairs, max_nq, max_nt);
    const int nsu = std::max(1, (max_nt + a.slice - 1) / a.slice);   // 1: k_top2_mfma writes the outputs itself
    a.qblocks = qb;
    a.nslices = nsu;
    const int vblocks = (int)((long long)qb * nsu * npairs);
    // max_nt == 0 (an empty train set, e.g. a previous frame without keypoints): no expansion launch (a
    // zero-sized grid is an error); k_top2_mfma then sees no tiles and writes the no-match sentinels
    if (!(a.tx && max_nt > 0) || (cfg.fp4 && cfg.noexp)) {
        auto kern = nw == 8 ? (ns == 2 ? k_top2_mfma<false, 8, 2, false> : k_top2_mfma<false, 8, 1, false>)
                            : (ns == 2 ? k_top2_mfma<false, 4, 2, false> : k_top2_mfma<false, 4, 1, false>);
        if (cfg.fp4)
            kern = nw == 4 ? k_top2_mfma<false, 4, 1, false, 0, true>
                           : ns == 2 ? k_top2_mfma<false, 8, 2, false, 0, true> : k_top2_mfma<false, 8, 1, false, 0, true>;
        if (cfg.fp4 && cfg.pipe && nw == 8 && ns == 1) kern = k_top2_mfma<false, 8, 1, true, 0, true>;   // "8fxp" (A/B)
        hipLaunchKernelGGL(kern, dim3((unsigned)vblocks), dim3(64 * nw), 0, stream, a, d_part, d_best, d_best_idx,
                           d_second, vblocks);
    } else {
        const bool pp = cfg.pipe;
        auto kern = nw == 8 ? (ns == 2 ? (pp ? k_top2_mfma<true, 8, 2, true> : k_top2_mfma<true, 8, 2, false>)
                                       : (pp ? k_top2_mfma<true, 8, 1, true> : k_top2_mfma<true, 8, 1, false>))
                            : (ns == 2 ? (pp ? k_top2_mfma<true, 4, 2, true> : k_top2_mfma<true, 4, 2, false>)
                                       : (pp ? k_top2_mfma<true, 4, 1, true> : k_top2_mfma<true, 4, 1, false>));
        if (pp && cfg.la && nw == 8)
            kern = ns == 2 ? (cfg.la == 4 ? k_top2_mfma<true, 8, 2, true, 4> : k_top2_mfma<true, 8, 2, true, 2>)
                           : (cfg.la == 4 ? k_top2_mfma<true, 8, 1, true, 4> : k_top2_mfma<true, 8, 1, true, 2>);
        if (cfg.fp4)
            kern = !pp ? k_top2_mfma<true, 8, 1, false, 0, true>
                       : cfg.la ? k_top2_mfma<true, 8, 1, true, 2, true> : k_top2_mfma<true, 8, 1, true, 0, true>;
        auto expand = cfg.fp4 ? k_expand_fp4 : k_expand_pm1;
        int slots = 1 << 30;   // persistent: one workgroup per resident slot (a multiple of 8: virtual blocks keep
        if (cfg.persist) {     // their XCD)
            int dev = 0, ncu = 256, per = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 64 * nw, 0) != hipSuccess || per < 1) per = 1;
            slots = std::max(8, (per * ncu) & ~7);
        }
        const int nslots = a.tx_frames ? a.n_tx_frames : npairs;
        const int gx = (max_nt * 8 + 255) / 256;
        if (ov && ov->nchunks > 1 && nsu == 1 && a.tx_frames && a.tx_slot) {
            // chunk c's expansion (its pairs' train slots) on the side stream, chunk c's top-2 on the launch
            // stream behind it: expansion c + 1 (HBM writes) runs beside top-2 c (matrix cores)
            hipError_t e;
            if ((e = hipEventRecord(ov->ev_fork, stream)) != hipSuccess ||
                (e = hipStreamWaitEvent(ov->s2, ov->ev_fork, 0)) != hipSuccess)
                return e;
            int s0 = 0;
            for (int cix = 0; cix < ov->nchunks; cix++) {
                const int s1 = std::min(ov->slot_end[cix], nslots);
                if (s1 > s0) hipLaunchKernelGGL(expand, dim3(gx, s1 - s0), dim3(256), 0, ov->s2, a, max_nt, s0);
                s0 = std::max(s0, s1);
                if ((e = hipEventRecord(ov->ev[cix], ov->s2)) != hipSuccess) return e;
            }
            for (int cix = 0; cix < ov->nchunks; cix++) {
                const int pb = ov->pair_beg[cix], pe = ov->pair_beg[cix + 1];
                if (pe <= pb) continue;
                if ((e = hipStreamWaitEvent(stream, ov->ev[cix], 0)) != hipSuccess) return e;
                Top2Batch ac = a;
                ac.frames = a.frames + pb;
                ac.tx_slot = a.tx_slot + pb;
                const int vb = qb * (pe - pb);
                const long long oo = (long long)pb * a.out_stride;
                hipLaunchKernelGGL(kern, dim3((unsigned)std::min(vb, slots)), dim3(64 * nw), 0, stream, ac, d_part,
                                   d_best + oo, d_best_idx + oo, d_second + oo, vb);
            }
            return hipGetLastError();
        }
        hipLaunchKernelGGL(expand, dim3(gx, nslots), dim3(256), 0, stream, a, max_nt, 0);
        hipLaunchKernelGGL(kern, dim3((unsigned)std::min(vblocks, slots)), dim3(64 * nw), 0, stream, a, d_part, d_best,
                           d_best_idx, d_second, vblocks);
    }
    if (nsu > 1)
        hipLaunchKernelGGL(k_top2b_merge, dim3((max_nq + 255) / 256, npairs), dim3(256), 0, stream, a, nsu, d_part,
                           d_best, d_best_idx, d_second);
    return hipGetLastError();
}

/* SearchForTriangulation inner loop (ORBmatcher.cc:712-761) for one (idx1, node) item per
 * wavefront: dist <= TH_LOW, epipole distance gate for mono pairs, CheckDistEpipolarLine
 * (:140-157, float with the final comparison in double).  The reference keeps the LAST candidate
 * reaching the running minimum ('dist > bestDist' skips only strictly larger), so the key is
 * dist << 32 | ~pos. */
__global__ __launch_bounds__(256) void k_triangulation(const uint8_t* __restrict__ qdesc,
                                                       const float4* __restrict__ qinfo,
                                                       const uint8_t* __restrict__ tdesc,
                                                       const float4* __restrict__ tinfo,
                                                       const int2* __restrict__ ranges, const int* __restrict__ cand,
                                                       int nitems, TriParams tp, int* __restrict__ best_out) {
    const int it = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (it >= nitems) return;
    const uint4* qp = reinterpret_cast<const uint4*>(qdesc + (long long)it * 32);
    const uint4 qa = qp[0], qb = qp[1];
    const float4 q = qinfo[it];   // x, y, stereo (1 / 0)
    const bool st1 = q.z != 0.f;
    const float* F = tp.F;
    // CheckDistEpipolarLine's float expressions with the contractions the reference's -O3 -march=native
    // build applies (tools/ref_flags_probe.cpp fixes each form)
    const float la = __builtin_fmaf(q.x, F[0], q.y * F[3]) + F[6];
    const float lb = __builtin_fmaf(q.x, F[1], q.y * F[4]) + F[7];
    const float lc = __builtin_fmaf(q.y, F[5], q.x * F[2]) + F[8];
    const float den = __builtin_fmaf(la, la, lb * lb);
    unsigned long long bestKey = ~0ull;
    const int c0 = ranges[it].x, c1 = ranges[it].y;
    for (int pos = c0 + lane; pos < c1; pos += 64) {
        const int j = cand[pos];   // (no map point, stereo if asked: filtered on the host, :725-733)
        const uint4* tq = reinterpret_cast<const uint4*>(tdesc + (long long)j * 32);
        const int dist = hamming256(qa, qb, tq[0], tq[1]);
        if (dist > 50) continue;
        const float4 t = tinfo[j];   // x, y, octave, stereo
        const int oct = (int)t.z;
        const bool st2 = t.w != 0.f;
        if (!st1 && !st2) {
            const float dex = tp.ex - t.x, dey = tp.ey - t.y;
            if (__builtin_fmaf(dex, dex, dey * dey) < 100 * tp.scale2[oct]) continue;
        }
        if (den == 0) continue;
        const float num = __builtin_fmaf(lb, t.y, la * t.x) + lc;
        const float dsqr = num * num / den;
        if (!((double)dsqr < 3.84 * (double)tp.sigma2[oct])) continue;
        const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned)(0x7FFFFFFF - (pos - c0));
        bestKey = key < bestKey ? key : bestKey;
    }
    bestKey = wave_min_u64(bestKey);
    if (lane == 0) {
        int r = -1;
        if (bestKey != ~0ull) r = cand[c0 + (0x7FFFFFFF - (int)(bestKey & 0xFFFFFFFFu))];
        best_out[it] = r;
    }
}

hipError_t launch_hamming_topk(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, const int2* d_ranges,
                               const int* d_cand_idx, const int* d_thr, int k, int* d_dist, int* d_idx, int* d_nvalid,
                               hipStream_t stream) {
    if (nq <= 0) return hipSuccess;
    if (k < 1 || k > kMaxK) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_topk, dim3((nq + 3) / 4), dim3(256), 0, stream, d_q, nq, d_t, nt, d_ranges, d_cand_idx,
                       d_thr, k, d_dist, d_idx, d_nvalid);
    return hipGetLastError();
}

hipError_t launch_window_topk(const uint8_t* d_q, const int* d_item_q, const float2* d_centre, int nitems,
                              const orb_keypoint* d_kps1, const uint8_t* d_t, const orb_keypoint* d_kps2,
                              const int* d_cell_off, const int* d_cell_idx, const WinGrid& wg, const int* d_thr,
                              int k, int* d_dist, int* d_idx, int* d_nvalid, hipStream_t stream) {
    if (nitems <= 0) return hipSuccess;
    if (k < 1 || k > kMaxK) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_window_topk, dim3((nitems + 3) / 4), dim3(256), 0, stream, d_q, d_item_q, d_centre, nitems,
                       d_kps1, d_t, d_kps2, d_cell_off, d_cell_idx, wg, d_thr, k, d_dist, d_idx, d_nvalid);
    return hipGetLastError();
}

hipError_t launch_triangulation(const uint8_t* d_qdesc, const float4* d_qinfo, const uint8_t* d_tdesc,
                                const float4* d_tinfo, const int2* d_ranges, const int* d_cand, int nitems,
                                const TriParams& tp, int* d_best, hipStream_t stream) {
    if (nitems <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_triangulation, dim3((nitems + 3) / 4), dim3(256), 0, stream, d_qdesc, d_qinfo, d_tdesc, d_tinfo,
                       d_ranges, d_cand, nitems, tp, d_best);
    return hipGetLastError();
}

}  // namespace orbgpu
