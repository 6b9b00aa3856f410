// gfx950 Hamming-distance kernels for ORBmatcher (ORBmatcher.cc).  256-bit distance =
// 8 x (v_xor_b32 + v_bcnt_u32_b32): bitwise VALU work, no MFMA.  The selection logic that depends
// on the order of earlier accepted matches (SearchByBoW's taken set, SearchForInitialization's
// vMatchedDistance) is replayed on the host from these exact top-k lists (matcher.cpp).
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

/* All-pairs top-2 (best, its index — first on ties — and second best), thread per query, train
 * descriptors streamed through LDS in 256-row tiles and read as wave-uniform broadcasts.  The
 * train set is split over gridDim.y slices for occupancy; slices are merged by k_top2_merge. */
__global__ __launch_bounds__(256) void k_top2_tiles(const uint8_t* __restrict__ q, int nq,
                                                    const uint8_t* __restrict__ t, int nt, int slice,
                                                    int4* __restrict__ part) {
    __shared__ uint4 s_t[256 * 2];
    const int qi = blockIdx.x * 256 + threadIdx.x;
    const int sl = blockIdx.y;
    const int t0 = sl * slice, t1 = min(nt, t0 + slice);
    uint4 qa = make_uint4(0, 0, 0, 0), qb = qa;
    if (qi < nq) {
        const uint4* qp = reinterpret_cast<const uint4*>(q + (long long)qi * 32);
        qa = qp[0];
        qb = qp[1];
    }
    int best = 257, bidx = -1, second = 257;
    for (int tb = t0; tb < t1; tb += 256) {
        const int n = min(256, t1 - tb);
        __syncthreads();
        if ((int)threadIdx.x < n) {
            const uint4* tp = reinterpret_cast<const uint4*>(t + (long long)(tb + threadIdx.x) * 32);
            s_t[2 * threadIdx.x] = tp[0];
            s_t[2 * threadIdx.x + 1] = tp[1];
        }
        __syncthreads();
        for (int j = 0; j < n; j++) {
            const int d = hamming256(qa, qb, s_t[2 * j], s_t[2 * j + 1]);
            if (d < best) {
                second = best;
                best = d;
                bidx = tb + j;
            } else if (d < second) {
                second = d;
            }
        }
    }
    if (qi < nq) part[(long long)sl * nq + qi] = make_int4(best, bidx, second, 0);
}

__global__ __launch_bounds__(256) void k_top2_merge(const int4* __restrict__ part, int nq, int nslices,
                                                    int* __restrict__ best_o, int* __restrict__ idx_o,
                                                    int* __restrict__ second_o) {
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= nq) return;
    int4 acc = part[qi];
    for (int s = 1; s < nslices; s++) {
        const int4 p = part[(long long)s * nq + qi];
        if (p.x < acc.x) {            // later slice wins only on a strictly smaller distance
            acc.z = min(acc.x, p.z);
            acc.x = p.x;
            acc.y = p.y;
        } else {
            acc.z = min(acc.z, p.x);
        }
    }
    best_o[qi] = acc.x;
    idx_o[qi] = acc.y;
    second_o[qi] = acc.z;
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

int top2_slices(int nq, int nt) {
    const int qblocks = (nq + 255) / 256;
    int nslices = 1;
    while (qblocks * nslices < 1024 && nt / (nslices * 2) >= 256) nslices *= 2;
    return nslices;
}

hipError_t launch_hamming_top2(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int* d_best, int* d_best_idx,
                               int* d_second, int4* d_part, hipStream_t stream) {
    if (nq <= 0) return hipSuccess;
    const int qblocks = (nq + 255) / 256;
    const int nslices = top2_slices(nq, nt);
    const int slice = (nt + nslices - 1) / nslices;
    hipLaunchKernelGGL(k_top2_tiles, dim3(qblocks, nslices), dim3(256), 0, stream, d_q, nq, d_t, nt, slice, d_part);
    hipLaunchKernelGGL(k_top2_merge, dim3(qblocks), dim3(256), 0, stream, d_part, nq, nslices, d_best, d_best_idx,
                       d_second);
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
