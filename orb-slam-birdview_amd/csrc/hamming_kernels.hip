// gfx950 Hamming-distance kernels for ORBmatcher (ORBmatcher.cc).  256-bit distance =
// 8 x (v_xor_b32 + v_bcnt_u32_b32): bitwise VALU work, no MFMA.  The selection logic that depends
// on the order of earlier accepted matches (SearchByBoW's taken set, SearchForInitialization's
// vMatchedDistance) is replayed on the host from these exact top-k lists (matcher.cpp).
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

/* Batched all-pairs top-2 over many (query set, train set) pairs in one launch.  Lane = query, one
 * wavefront = 64 queries x one train slice; the train descriptors of the slice are wave-uniform and
 * read through the scalar cache (s_load), so the inner loop is 8 v_xor + 8 v_bcnt (accumulating)
 * and a 3-op top-2 update on keys dist << 16 | train index: min keeps the first index on ties, and
 * second = min(second, max(best, key)) is the second-smallest key.  Slices are merged by
 * k_top2b_merge (keys compose the same way).  Counts may be read on the device (an extraction
 * batch's d_counts), so a whole batch of frame pairs needs no host round trip. */
__global__ __launch_bounds__(256) void k_top2_batch(Top2Batch a, uint2* __restrict__ part, int* __restrict__ best_o,
                                                    int* __restrict__ idx_o, int* __restrict__ second_o) {
    const int p = blockIdx.z, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int2 fr = a.frames ? a.frames[p] : make_int2(0, 0);
    const int nq = a.counts ? a.counts[fr.x] : a.nq, nt = a.counts ? a.counts[fr.y] : a.nt;
    const int qw = (blockIdx.x * 4 + wv) * 64;
    if (qw >= nq) return;   // whole wave (no block barriers below)
    const int qi = qw + lane;
    const int t0 = blockIdx.y * a.slice, t1 = min(nt, t0 + a.slice);
    uint4 qa = make_uint4(0, 0, 0, 0), qb = qa;
    if (qi < nq) {
        const uint4* qp = reinterpret_cast<const uint4*>(a.q + ((long long)fr.x * a.q_stride + qi) * 32);
        qa = qp[0];
        qb = qp[1];
    }
    const uint4* __restrict__ T = reinterpret_cast<const uint4*>(a.t + (long long)fr.y * a.t_stride * 32);
    unsigned b = 0xFFFFFFFFu, s2 = 0xFFFFFFFFu;
#pragma unroll 4
    for (int j = t0; j < t1; j++) {
        const uint4 x = T[2 * j], y = T[2 * j + 1];
        const unsigned d = __popc(qa.x ^ x.x) + __popc(qa.y ^ x.y) + __popc(qa.z ^ x.z) + __popc(qa.w ^ x.w) +
            __popc(qb.x ^ y.x) + __popc(qb.y ^ y.y) + __popc(qb.z ^ y.z) + __popc(qb.w ^ y.w);
        const unsigned key = (d << 16) | (unsigned)j;
        s2 = min(s2, max(b, key));
        b = min(b, key);
    }
    if (qi >= nq) return;
    const long long o = (long long)p * a.out_stride + qi;
    if (gridDim.y == 1) {
        best_o[o] = b == 0xFFFFFFFFu ? 257 : (int)(b >> 16);
        idx_o[o] = b == 0xFFFFFFFFu ? -1 : (int)(b & 0xFFFF);
        second_o[o] = s2 == 0xFFFFFFFFu ? 257 : (int)(s2 >> 16);
    } else {
        part[((long long)p * gridDim.y + blockIdx.y) * a.out_stride + qi] = make_uint2(b, s2);
    }
}

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

int top2_batch_slices(int npairs, int max_nq, int max_nt) {
    const int qwaves = std::max(1, (max_nq + 63) / 64);
    int ns = (8192 + npairs * qwaves - 1) / (npairs * qwaves);   // aim for >= 8192 wavefronts
    ns = std::min(ns, std::max(1, (max_nt + 31) / 32));          // >= 32 trains per slice
    return std::max(ns, 1);
}

hipError_t launch_hamming_top2_batch(const Top2Batch& a0, int npairs, int max_nq, int max_nt, int* d_best,
                                     int* d_best_idx, int* d_second, uint2* d_part, hipStream_t stream) {
    if (npairs <= 0 || max_nq <= 0) return hipSuccess;
    if (max_nt > 65535) return hipErrorInvalidValue;   // keys hold a 16-bit train index
    Top2Batch a = a0;
    const int ns = top2_batch_slices(npairs, max_nq, max_nt);
    a.slice = std::max(1, (max_nt + ns - 1) / ns);
    const int nsu = std::max(1, (max_nt + a.slice - 1) / a.slice);
    hipLaunchKernelGGL(k_top2_batch, dim3((max_nq + 255) / 256, nsu, npairs), dim3(256), 0, stream, a, d_part, d_best,
                       d_best_idx, d_second);
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
__global__ __launch_bounds__(256) void k_triangulation(const uint8_t* __restrict__ desc1,
                                                       const orb_keypoint* __restrict__ kps1,
                                                       const float* __restrict__ ur1,
                                                       const uint8_t* __restrict__ desc2,
                                                       const orb_keypoint* __restrict__ kps2,
                                                       const uint8_t* __restrict__ mp2, const float* __restrict__ ur2,
                                                       const int* __restrict__ item_q, const int2* __restrict__ ranges,
                                                       const int* __restrict__ cand_idx, int nitems, TriParams tp,
                                                       int* __restrict__ best_out) {
    const int it = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (it >= nitems) return;
    const int idx1 = item_q[it];
    const uint4* qp = reinterpret_cast<const uint4*>(desc1 + (long long)idx1 * 32);
    const uint4 qa = qp[0], qb = qp[1];
    const orb_keypoint kp1 = kps1[idx1];
    const bool st1 = ur1[idx1] >= 0;
    const float* F = tp.F;
    const float la = kp1.x * F[0] + kp1.y * F[3] + F[6];
    const float lb = kp1.x * F[1] + kp1.y * F[4] + F[7];
    const float lc = kp1.x * F[2] + kp1.y * F[5] + F[8];
    const float den = la * la + lb * lb;
    unsigned long long bestKey = ~0ull;
    const int c0 = ranges[it].x, c1 = ranges[it].y;
    for (int pos = c0 + lane; pos < c1; pos += 64) {
        const int idx2 = cand_idx[pos];
        if (mp2[idx2]) continue;
        const bool st2 = ur2[idx2] >= 0;
        if (tp.only_stereo && !st2) continue;
        const uint4* tq = reinterpret_cast<const uint4*>(desc2 + (long long)idx2 * 32);
        const int dist = hamming256(qa, qb, tq[0], tq[1]);
        if (dist > 50) continue;
        const orb_keypoint kp2 = kps2[idx2];
        if (!st1 && !st2) {
            const float dex = tp.ex - kp2.x, dey = tp.ey - kp2.y;
            if (dex * dex + dey * dey < 100 * tp.scale2[kp2.octave]) continue;
        }
        if (den == 0) continue;
        const float num = la * kp2.x + lb * kp2.y + lc;
        const float dsqr = num * num / den;
        if (!((double)dsqr < 3.84 * (double)tp.sigma2[kp2.octave])) continue;
        const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned)(0x7FFFFFFF - (pos - c0));
        bestKey = key < bestKey ? key : bestKey;
    }
    bestKey = wave_min_u64(bestKey);
    if (lane == 0) {
        int r = -1;
        if (bestKey != ~0ull) r = cand_idx[c0 + (0x7FFFFFFF - (int)(bestKey & 0xFFFFFFFFu))];
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

hipError_t launch_triangulation(const uint8_t* d_desc1, const orb_keypoint* d_kps1, const float* d_ur1,
                                const uint8_t* d_desc2, const orb_keypoint* d_kps2, const uint8_t* d_mp2,
                                const float* d_ur2, const int* d_item_q, const int2* d_ranges, const int* d_cand_idx,
                                int nitems, const TriParams& tp, int* d_best, hipStream_t stream) {
    if (nitems <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_triangulation, dim3((nitems + 3) / 4), dim3(256), 0, stream, d_desc1, d_kps1, d_ur1, d_desc2,
                       d_kps2, d_mp2, d_ur2, d_item_q, d_ranges, d_cand_idx, nitems, tp, d_best);
    return hipGetLastError();
}

}  // namespace orbgpu
