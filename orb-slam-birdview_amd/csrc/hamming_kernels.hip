// gfx950 Hamming-distance kernels for ORBmatcher's vocabulary-gated searches (ORBmatcher.cc): the 256-bit
// distance (DescriptorDistance, ORBmatcher.cc:1647-1663) as 8 x (v_xor_b32 + v_bcnt_u32_b32) per pair on the VALU,
// over CSR candidate lists (k_topk), the Frame grid's windows (k_window_topk) and SearchForTriangulation's
// epipolar-gated candidates (k_triangulation).  The all-pairs top-2 on the matrix cores is hamming_top2.hip.
// The selection logic that depends on the order of earlier accepted matches (SearchByBoW's taken set,
// SearchForInitialization's vMatchedDistance) is replayed on the host from these exact top-k lists
// (matcher.hip).
#include <algorithm>

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

/* SearchForTriangulation inner loop (ORBmatcher.cc:712-761) for one (idx1, node) item per
 * wavefront: dist <= TH_LOW, epipole distance gate for mono pairs, CheckDistEpipolarLine
 * (:140-157, float with the final comparison in double).  The reference keeps the LAST candidate
 * reaching the running minimum ('dist > bestDist' skips only strictly larger), so the key is
 * dist << 32 | ~pos.  The inputs live in host memory (the call's pinned mirror): the item record is one
 * wave-uniform read, then each lane reads its candidates' records. */
__global__ __launch_bounds__(256) void k_triangulation(const TriItem* __restrict__ items,
                                                       const TriTrain* __restrict__ trains, int nitems,
                                                       int* __restrict__ best_out) {
    const int it = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (it >= nitems) return;
    const TriItem q = items[it];
    const bool st1 = q.stereo != 0;
    // CheckDistEpipolarLine (the reference's contracted float forms, tools/ref_flags_probe.cpp): the line a, b, c
    // comes staged with the query
    const float la = q.la, lb = q.lb, lc = q.lc;
    const float den = __builtin_fmaf(la, la, lb * lb);
    unsigned long long bestKey = ~0ull;
    const int c0 = q.c0, c1 = q.c1;
    for (int pos = c0 + lane; pos < c1; pos += 64) {
        const TriTrain& tr = trains[pos];   // (no map point, stereo if asked: filtered on the host, :725-733)
        const uint4 ta = tr.desc[0], tb = tr.desc[1];
        const int dist = hamming256(q.desc[0], q.desc[1], ta, tb);
        if (dist > 50) continue;
        const int fl = tr.flags;
        if (!st1 && !(fl & 1) && (fl & 2)) continue;   // neither stereo and too close to the epipole (:743-748)
        if (den == 0) continue;
        const float num = __builtin_fmaf(lb, tr.y, la * tr.x) + lc;
        const float dsqr = num * num / den;
        if (!((double)dsqr < 3.84 * (double)tr.sigma2)) continue;
        const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned)(0x7FFFFFFF - (pos - c0));
        bestKey = key < bestKey ? key : bestKey;
    }
    bestKey = wave_min_u64(bestKey);
    if (lane == 0) best_out[it] = bestKey != ~0ull ? c0 + (0x7FFFFFFF - (int)(bestKey & 0xFFFFFFFFu)) : -1;
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

hipError_t launch_triangulation(const TriItem* d_items, const TriTrain* d_trains, int nitems, int* d_best,
                                hipStream_t stream) {
    if (nitems <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_triangulation, dim3((nitems + 3) / 4), dim3(256), 0, stream, d_items, d_trains, nitems, d_best);
    return hipGetLastError();
}

}  // namespace orbgpu
