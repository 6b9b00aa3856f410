// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:242-307; MapPointBird.cc:87-152 is the
// same) on gfx950, batched over map points: for each map point, the observation
// whose median Hamming distance to all of the point's observations (itself included) is smallest,
// first index on ties.  One wavefront per map point; per row i the distances go into a 257-bin LDS
// histogram (distances are 0..256) and the median vDists[(int)(0.5*(N-1))] is its rank-k value, so
// any number of observations runs in fixed LDS.
#include <vector>

#include "orbgpu_ctx.h"

namespace orbgpu {

__global__ __launch_bounds__(256) void k_distinctive(const int* __restrict__ off, const uint8_t* __restrict__ desc,
                                                     int nmp, int* __restrict__ best_out) {
    __shared__ int s_hist[4][260];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave-uniform: SALU
    const int m = blockIdx.x * 4 + wv;
    if (m >= nmp) return;   // whole wave
    const int b = off[m], N = off[m + 1] - b;
    if (N <= 0) {
        if (lane == 0) best_out[m] = -1;
        return;
    }
    int* hist = s_hist[wv];
    const int k = (int)(0.5 * (N - 1));   // vDists[0.5*(N-1)]: double index truncated
    const uint4* D = reinterpret_cast<const uint4*>(desc + (long long)b * 32);
    int bestMedian = 0x7FFFFFFF, bestIdx = 0;
    for (int i = 0; i < N; i++) {
        for (int t = lane; t < 260; t += 64) hist[t] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint4 a0 = D[2 * i], a1 = D[2 * i + 1];
        for (int j = lane; j < N; j += 64) {
            const uint4 x = D[2 * j], y = D[2 * j + 1];
            const int d = __popc(a0.x ^ x.x) + __popc(a0.y ^ x.y) + __popc(a0.z ^ x.z) + __popc(a0.w ^ x.w) +
                          __popc(a1.x ^ y.x) + __popc(a1.y ^ y.y) + __popc(a1.z ^ y.z) + __popc(a1.w ^ y.w);
            atomicAdd(&hist[d], 1);   // Distances[i][i] = 0 falls out of d(i, i) = 0
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lane l owns bins 5l .. 5l+4 (0..319 >= 257): inclusive counts, then the bin holding rank k
        int c[5], s = 0;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const int bin = 5 * lane + q;
            c[q] = bin < 257 ? hist[bin] : 0;
            s += c[q];
        }
        int x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        int before = x - s, median = 0x7FFFFFFF;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            if (median == 0x7FFFFFFF && before <= k && k < before + c[q]) median = 5 * lane + q;
            before += c[q];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) median = min(median, __shfl_xor(median, o));
        if (median < bestMedian) {   // strict: first index on ties
            bestMedian = median;
            bestIdx = i;
        }
    }
    if (lane == 0) best_out[m] = bestIdx;
}

}  // namespace orbgpu

using namespace orbgpu;

extern "C" int orb_distinctive_descriptors(orb_ctx* h, int nmp, const int* offsets, const uint8_t* desc,
                                           int* best_idx) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    if (!c) return set_error("NULL context", hipSuccess), ORB_ERR_ARG;
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return set_error("hipSetDevice", e), ORB_ERR_HIP;
    if (nmp < 0 || (nmp && (!offsets || !best_idx))) return set_error("orb_distinctive_descriptors: bad arguments",
                                                                      hipSuccess), ORB_ERR_ARG;
    if (nmp == 0) return ORB_OK;
    const int total = offsets[nmp];
    if (total < 0 || (total && !desc)) return ORB_ERR_ARG;
    const size_t A = 256;
    auto al = [&](size_t x) { return (x + A - 1) & ~(A - 1); };
    const size_t need = al((size_t)(nmp + 1) * 4) + al((size_t)std::max(total, 1) * 32) + al((size_t)nmp * 4);
    if (need > c->scratch_cap || !c->d_scratch) {
        if (c->d_scratch) (void)hipFree(c->d_scratch);
        c->d_scratch = nullptr;
        c->scratch_cap = 0;
        if ((e = hipMalloc((void**)&c->d_scratch, need)) != hipSuccess) return set_error("scratch", e), ORB_ERR_NOMEM;
        c->scratch_cap = need;
    }
    int* d_off = reinterpret_cast<int*>(c->d_scratch);
    uint8_t* d_desc = c->d_scratch + al((size_t)(nmp + 1) * 4);
    int* d_best = reinterpret_cast<int*>(d_desc + al((size_t)std::max(total, 1) * 32));
    if ((e = hipMemcpyAsync(d_off, offsets, (size_t)(nmp + 1) * 4, hipMemcpyHostToDevice, c->stream)) != hipSuccess ||
        (total && (e = hipMemcpyAsync(d_desc, desc, (size_t)total * 32, hipMemcpyHostToDevice, c->stream)) !=
                      hipSuccess))
        return set_error("upload", e), ORB_ERR_HIP;
    hipLaunchKernelGGL(k_distinctive, dim3((nmp + 3) / 4), dim3(256), 0, c->stream, d_off, d_desc, nmp, d_best);
    if ((e = hipGetLastError()) != hipSuccess) return set_error("distinctive kernel", e), ORB_ERR_HIP;
    if ((e = hipMemcpyAsync(best_idx, d_best, (size_t)nmp * 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return set_error("download", e), ORB_ERR_HIP;
    return ORB_OK;
}
