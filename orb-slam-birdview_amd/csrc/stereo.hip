// Frame::ComputeStereoMatches (Frame.cc:662-836) on gfx950: the first consumer of the extractor's
// outputs.  Reads the left/right pyramids where the extractor left them in HBM,
// so mvImagePyramid never has to be copied to the host for stereo.
//
//   k_stereo      one wavefront per left keypoint: row-band / octave / disparity-range filtered
//                 Hamming search over the right keypoints (first minimum, as the strict '<' of
//                 :737-741), then the 11x11 centred-L1 window search over 11 offsets (:758-788),
//                 parabola refinement and the disparity checks (:790-819)
//   k_stereo_cut  one workgroup per pair: median of the accepted window distances and the
//                 1.5*1.4*median outlier cut (:822-835)
//
// All window arithmetic is integer (cv::norm NORM_L1 of integer-valued float patches is an exact
// integer); the parabola and depth use the reference's float expressions, uncontracted.
#include <algorithm>
#include <cstdlib>
#include <climits>
#include <cstring>
#include <vector>

#include "orbgpu_ctx.h"

namespace orbgpu {
namespace {

constexpr int kThHigh = 100;                      // ORBmatcher.cc:37
constexpr int kThOrbDist = (kThHigh + 50) / 2;    // Frame.cc:667
constexpr int kWin = 5;                           // :758 w
constexpr int kRange = 5;                         // :765 L

__device__ __forceinline__ const uint8_t* level_base(const Geom* __restrict__ g, const StereoSide& s, int f, int l,
                                                     int& stride) {
    if (l == 0) {
        stride = s.row_stride;
        return s.frames + (long long)f * s.frame_pitch;
    }
    stride = g->L[l].pitch;
    return s.pyr + (long long)f * g->pyr_bytes + g->L[l].pyr_off;
}

__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Exclusive scan of one int per thread over a 256-thread block; s_w holds 4 wave totals.
__device__ __forceinline__ int block256_scan(int v, int* s_w, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    int before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        before += w < wave ? s_w[w] : 0;
        total += s_w[w];
    }
    __syncthreads();
    return before + x - v;
}

}  // namespace

// Right keypoints bucketed by image row (counting sort in LDS, one workgroup per pair): the
// descriptor search of a left keypoint then visits only the rows its band can reach instead of
// every right keypoint.  Order inside a row is irrelevant (the search minimises dist << 16 | iR).
__global__ __launch_bounds__(256) void k_stereo_bucket(const Geom* __restrict__ g, StereoSide R,
                                                       int* __restrict__ rows, int* __restrict__ sorted,
                                                       long long row_stride, long long out_stride) {
    extern __shared__ int s_hist[];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int fR = R.frame0 + p * R.frame_step;
    const int nR = R.counts[fR], H = g->L[0].h;
    const orb_keypoint* kR = R.kps + (long long)fR * R.kp_stride;
    int* rs = rows + (long long)p * row_stride;
    int* srt = sorted + (long long)p * out_stride;
    for (int i = tid; i <= H; i += 256) s_hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < nR; i += 256) atomicAdd(&s_hist[min(max((int)floorf(kR[i].y), 0), H - 1)], 1);
    __syncthreads();
    {   // exclusive scan over the H + 1 rows: a contiguous chunk per thread
        __shared__ int s_w[4];
        const int chunk = (H + 1 + 255) / 256, r0 = min(tid * chunk, H + 1), r1 = min(r0 + chunk, H + 1);
        int local = 0;
        for (int r = r0; r < r1; r++) local += s_hist[r];
        int total;
        int acc = block256_scan(local, s_w, total);
        for (int r = r0; r < r1; r++) {
            const int v = s_hist[r];
            s_hist[r] = acc;
            rs[r] = acc;
            acc += v;
        }
    }
    __syncthreads();
    for (int i = tid; i < nR; i += 256) {
        const int r = min(max((int)floorf(kR[i].y), 0), H - 1);
        srt[atomicAdd(&s_hist[r], 1)] = i;
    }
}

__global__ __launch_bounds__(256) void k_stereo(const Geom* __restrict__ g, StereoSide L, StereoSide R, float mb,
                                                float mbf, float* __restrict__ uright, float* __restrict__ depth,
                                                int* __restrict__ sad, long long out_stride,
                                                const int* __restrict__ rows, const int* __restrict__ sorted,
                                                long long row_stride) {
    __shared__ int s_part[4][64];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;   // wave-uniform: SALU
    const int p = blockIdx.y;
    const int iL = blockIdx.x * 4 + wv;
    const int fL = L.frame0 + p * L.frame_step, fR = R.frame0 + p * R.frame_step;
    const int nL = L.counts[fL], nR = R.counts[fR];
    if (iL >= nL) return;
    const orb_keypoint* kR = R.kps + (long long)fR * R.kp_stride;
    const orb_keypoint kpL = L.kps[(long long)fL * L.kp_stride + iL];
    const uint4* qp = reinterpret_cast<const uint4*>(L.desc + ((long long)fL * L.kp_stride + iL) * 32);
    const uint4 qa = qp[0], qb = qp[1];
    const uint4* dR = reinterpret_cast<const uint4*>(R.desc + (long long)fR * R.kp_stride * 32);
    const float minD = 0, maxD = mbf / mb;   // :692-694 (minZ = mb)
    const float uL = kpL.x, vL = kpL.y;
    const float minU = uL - maxD, maxU = uL - minD;
    const int yL = (int)vL;                  // vRowIndices[vL]: float index truncated (:707)
    const int levelL = kpL.octave;

    // ---- descriptor search over the right keypoints whose row band covers yL (:676-689, :716-745)
    unsigned best = 0xFFFFFFFFu;   // dist << 16 | iR: the first minimum in iR order
    if (maxU >= 0) {
        // a right keypoint reaches rows [floor(y - r), ceil(y + r)], r = 2 * scale <= 2 * scale_max
        const int reach = (int)ceilf(2.0f * g->L[g->nlevels - 1].scale) + 1;
        const int H = g->L[0].h;
        const int* rs = rows + (long long)p * row_stride;
        const int c0 = rs[max(yL - reach, 0)], c1 = rs[min(yL + reach, H - 1) + 1];
        const int* srt = sorted + (long long)p * out_stride;
        (void)nR;
        for (int c = c0 + lane; c < c1; c += 64) {
            const int iR = srt[c];
            const orb_keypoint kr = kR[iR];
            const float r = 2.0f * g->L[kr.octave].scale;
            const int maxr = (int)ceilf(kr.y + r), minr = (int)floorf(kr.y - r);
            if (yL < minr || yL > maxr) continue;
            if (kr.octave < levelL - 1 || kr.octave > levelL + 1) continue;
            if (!(kr.x >= minU && kr.x <= maxU)) continue;
            const int dist = hamming256(qa, qb, dR[2 * iR], dR[2 * iR + 1]);
            if (dist < kThHigh) best = min(best, ((unsigned)dist << 16) | (unsigned)iR);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = min(best, (unsigned)__shfl_xor((int)best, o));

    float outU = -1.0f, outD = -1.0f;
    int outS = -1;
    if (best != 0xFFFFFFFFu && (int)(best >> 16) < kThOrbDist) {
        // ---- sliding-window search at the keypoint's scale (:750-788)
        const int bestIdxR = (int)(best & 0xFFFF);
        const float uR0 = kR[bestIdxR].x;
        const float scaleFactor = 1.0f / g->L[levelL].scale;   // mvInvScaleFactors (ORBextractor.cc:428-429)
        const float scaleduL = roundf(uL * scaleFactor);
        const float scaledvL = roundf(vL * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const float iniu = scaleduR0 + kRange - kWin;
        const float endu = scaleduR0 + kRange + kWin + 1;
        const int cols = g->L[levelL].w;
        if (!(iniu < 0 || endu >= cols)) {
            int sL, sR;
            const uint8_t* PL = level_base(g, L, fL, levelL, sL);
            const uint8_t* PR = level_base(g, R, fR, levelL, sR);
            const int y0 = (int)scaledvL - kWin, xl0 = (int)scaleduL - kWin, xr0 = (int)scaleduR0 - kWin;
            const int cL = PL[(long long)(y0 + kWin) * sL + xl0 + kWin];
            // lane j < 55: offset incR = j/5 - 5, row group j%5 (rows {0-2}, {3-4}, ..., {9-10})
            int acc = 0;
            if (lane < 55) {
                const int inc = lane / 5 - kRange, rg = lane - (lane / 5) * 5;
                const int r0 = rg == 0 ? 0 : 2 * rg + 1, r1 = 2 * rg + 3;
                const int xr = xr0 + inc;
                const int cR = PR[(long long)(y0 + kWin) * sR + xr + kWin];
                for (int yy = r0; yy < r1; yy++) {
                    const uint8_t* rl = PL + (long long)(y0 + yy) * sL + xl0;
                    const uint8_t* rr = PR + (long long)(y0 + yy) * sR + xr;
#pragma unroll
                    for (int xx = 0; xx < 2 * kWin + 1; xx++)   // |(l - cL) - (r - cR)| = |(l + cR) - (r + cL)|
                        acc += abs((rl[xx] + cR) - (rr[xx] + cL));
                }
            }
            s_part[wv][lane] = acc;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane == 0) {
                float vDists[2 * kRange + 1];
                int bestDist = INT_MAX, bestincR = 0;
                for (int k = 0; k < 2 * kRange + 1; k++) {
                    const int* q = &s_part[wv][5 * k];
                    const float dist = (float)(q[0] + q[1] + q[2] + q[3] + q[4]);
                    if (dist < bestDist) {
                        bestDist = (int)dist;
                        bestincR = k - kRange;
                    }
                    vDists[k] = dist;
                }
                if (bestincR != -kRange && bestincR != kRange) {
                    // ---- sub-pixel parabola (:793-801) and disparity checks (:803-819)
                    const float dist1 = vDists[kRange + bestincR - 1];
                    const float dist2 = vDists[kRange + bestincR];
                    const float dist3 = vDists[kRange + bestincR + 1];
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = g->L[levelL].scale * ((float)scaleduR0 + (float)bestincR + deltaR);
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {
                            if (disparity <= 0) {
                                disparity = 0.01f;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            outD = mbf / disparity;
                            outU = bestuR;
                            outS = bestDist;
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        const long long o = (long long)p * out_stride + iL;
        uright[o] = outU;
        depth[o] = outD;
        sad[o] = outS;
    }
}

// Median cut (:822-835): the median of the accepted window distances (values < 2^16: 121 * 510
// at most) by a two-pass 8-bit radix select, thDist = 1.5f*1.4f*median, and every accepted
// keypoint whose distance is >= thDist rejected.  vDistIdx is sorted by (dist, iL), so its element
// cnt/2 has the (cnt/2)-th smallest distance — which is all the cut uses.
__global__ __launch_bounds__(256) void k_stereo_cut(StereoSide L, float* __restrict__ uright,
                                                    float* __restrict__ depth, const int* __restrict__ sad,
                                                    long long out_stride, int* __restrict__ nmatched) {
    __shared__ int s_hist[256];
    __shared__ int s_w[4];
    __shared__ int s_sel[2];
    __shared__ int s_kept;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nL = L.counts[L.frame0 + p * L.frame_step];
    float* ur = uright + (long long)p * out_stride;
    float* dp = depth + (long long)p * out_stride;
    const int* sd = sad + (long long)p * out_stride;
    int cnt = 0, hi = 0, k = 0;
    for (int pass = 0; pass < 2; pass++) {
        s_hist[tid] = 0;
        if (tid == 0) s_kept = 0;
        __syncthreads();
        int mine = 0;
        for (int i = tid; i < nL; i += 256) {
            const int v = sd[i];
            if (v < 0 || (pass == 1 && (v >> 8) != hi)) continue;
            atomicAdd(&s_hist[pass == 0 ? (v >> 8) & 255 : v & 255], 1);
            mine++;
        }
        if (mine) atomicAdd(&s_kept, mine);
        __syncthreads();
        if (pass == 0) {
            cnt = s_kept;
            if (cnt == 0) {   // (the reference reads vDistIdx[0] of an empty vector)
                if (tid == 0) nmatched[p] = 0;
                return;
            }
            k = cnt / 2;
        }
        const int hcount = s_hist[tid];
        int total;
        const int before = block256_scan(hcount, s_w, total);
        if (before <= k && k < before + hcount) {
            s_sel[0] = tid;
            s_sel[1] = k - before;
        }
        __syncthreads();
        if (pass == 0) hi = s_sel[0];
        k = s_sel[1];
        __syncthreads();
    }
    const float median = (float)((hi << 8) | s_sel[0]);
    const float thDist = 1.5f * 1.4f * median;
    if (tid == 0) s_kept = 0;
    __syncthreads();
    int kept = 0;
    for (int i = tid; i < nL; i += 256) {
        const int v = sd[i];
        if (v < 0) continue;
        if ((float)v < thDist) {
            kept++;
        } else {
            ur[i] = -1.0f;
            dp[i] = -1.0f;
        }
    }
    if (kept) atomicAdd(&s_kept, kept);
    __syncthreads();
    if (tid == 0) nmatched[p] = s_kept;
}

size_t stereo_scratch_ints(const Geom& g, int npairs, long long out_stride) {
    return (size_t)npairs * ((size_t)out_stride * 2 + g.L[0].h + 2);   // sad + sorted + row offsets
}

hipError_t launch_stereo(const Geom* d_geom, const Geom& g, const StereoSide& L, const StereoSide& R, int npairs,
                         float mb, float mbf, float* d_uright, float* d_depth, int* d_scratch, long long out_stride,
                         int* d_nmatched, hipStream_t stream) {
    if (npairs <= 0) return hipSuccess;
    const int cap = (int)out_stride;
    const long long row_stride = g.L[0].h + 2;
    int* d_sad = d_scratch;
    int* d_sorted = d_sad + (size_t)npairs * out_stride;
    int* d_rows = d_sorted + (size_t)npairs * out_stride;
    if ((size_t)(g.L[0].h + 1) * 4 > 64 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_stereo_bucket, dim3(npairs), dim3(256), (size_t)(g.L[0].h + 1) * 4, stream, d_geom, R, d_rows,
                       d_sorted, row_stride, out_stride);
    hipLaunchKernelGGL(k_stereo, dim3((cap + 3) / 4, npairs), dim3(256), 0, stream, d_geom, L, R, mb, mbf, d_uright,
                       d_depth, d_sad, out_stride, d_rows, d_sorted, row_stride);
    hipLaunchKernelGGL(k_stereo_cut, dim3(npairs), dim3(256), 0, stream, L, d_uright, d_depth, d_sad, out_stride,
                       d_nmatched);
    (void)g;
    return hipGetLastError();
}

}  // namespace orbgpu

using namespace orbgpu;

#define CTX_GUARD(ctx)                                                              \
    if (!(ctx)) {                                                                   \
        set_error("NULL context", hipSuccess);                                      \
        return ORB_ERR_ARG;                                                         \
    }                                                                               \
    {                                                                               \
        hipError_t _e = hipSetDevice((ctx)->device);                                \
        if (_e != hipSuccess) return set_error("hipSetDevice", _e), ORB_ERR_HIP;    \
    }

static bool same_geometry(const Ctx* a, const Ctx* b) {
    if (!a->have_geom || !b->have_geom) return false;
    const Geom &x = a->geom, &y = b->geom;
    if (x.W != y.W || x.H != y.H || x.nlevels != y.nlevels) return false;
    for (int l = 0; l < x.nlevels; l++)
        if (x.L[l].w != y.L[l].w || x.L[l].h != y.L[l].h || x.L[l].pitch != y.L[l].pitch ||
            x.L[l].pyr_off != y.L[l].pyr_off || x.L[l].scale != y.L[l].scale)
            return false;
    return true;
}

extern "C" {

int orb_compute_stereo_matches(orb_ctx* left, orb_ctx* right, int nL, const orb_keypoint* kpsL, const uint8_t* descL,
                               int nR, const orb_keypoint* kpsR, const uint8_t* descR, float mb, float mbf,
                               float* uright, float* depth, int* nmatched) {
    Ctx* cl = reinterpret_cast<Ctx*>(left);
    Ctx* cr = reinterpret_cast<Ctx*>(right);
    CTX_GUARD(cl);
    if (!cr || nL < 0 || nR < 0 || (nL && (!kpsL || !descL || !uright || !depth)) || (nR && (!kpsR || !descR)))
        return set_error("orb_compute_stereo_matches: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (cl->last_nframes < 1 || cr->last_nframes < 1 || !same_geometry(cl, cr))
        return set_error("orb_compute_stereo_matches: both contexts must have extracted an image of one size",
                         hipSuccess),
               ORB_ERR_ARG;
    if (nL == 0) {
        if (nmatched) *nmatched = 0;
        return ORB_OK;
    }
    hipError_t e;
    if ((e = hipStreamSynchronize(cr->stream)) != hipSuccess) return set_error("sync right", e), ORB_ERR_HIP;
    const int cap = std::max(nL, 1);
    const int scap = std::max(cap, nR);   // slots: sad (left) and sorted right indices share one stride
    // the call's device arena with its pinned host mirror (orbgpu_ctx.h Stage, as the matcher calls): the
    // inputs are packed into the mirror and go up in one DMA, the kernels store mvuRight / mvDepth and the
    // match count straight into the mirror (host-coherent), one synchronisation
    Stage st{cl};
    const size_t o_kL = st.add((size_t)nL * 28), o_dL = st.add((size_t)nL * 32);
    const size_t o_kR = st.add((size_t)std::max(nR, 1) * 28), o_dR = st.add((size_t)std::max(nR, 1) * 32);
    const size_t o_cnt = st.add(16);
    const size_t o_in_end = st.off;
    const size_t o_u = st.add((size_t)cap * 4), o_d = st.add((size_t)cap * 4), o_nm = st.add(4);
    st.end_mirror();
    const size_t o_s = st.add(stereo_scratch_ints(cl->geom, 1, scap) * 4);   // device-only working space
    if (const int r = st.alloc(); r != ORB_OK) return r;
    std::memcpy(st.hi<uint8_t>(o_kL), kpsL, (size_t)nL * 28);
    std::memcpy(st.hi<uint8_t>(o_dL), descL, (size_t)nL * 32);
    if (nR) {
        std::memcpy(st.hi<uint8_t>(o_kR), kpsR, (size_t)nR * 28);
        std::memcpy(st.hi<uint8_t>(o_dR), descR, (size_t)nR * 32);
    }
    st.hi<int>(o_cnt)[0] = nL;
    st.hi<int>(o_cnt)[1] = nR;
    if ((e = st.up(0, o_in_end)) != hipSuccess) return set_error("stereo upload", e), ORB_ERR_HIP;
    orb_keypoint* d_kL = st.di<orb_keypoint>(o_kL);
    uint8_t* d_dL = st.di<uint8_t>(o_dL);
    orb_keypoint* d_kR = st.di<orb_keypoint>(o_kR);
    uint8_t* d_dR = st.di<uint8_t>(o_dR);
    int* d_cnt = st.di<int>(o_cnt);
    float* h_u = st.h<float>(o_u);
    float* h_d = st.h<float>(o_d);
    int* h_nm = st.h<int>(o_nm);
    int* d_s = st.d<int>(o_s);
    StereoSide SL{cl->last_frames, cl->last_frame_pitch, cl->last_row_stride, cl->d_pyr, 0, 0, d_kL, d_dL, d_cnt, 0};
    StereoSide SR{cr->last_frames, cr->last_frame_pitch, cr->last_row_stride, cr->d_pyr, 0, 0, d_kR, d_dR, d_cnt + 1, 0};
    // Left and right extractors on different GPUs (one GPU per camera stream, BASELINE C4): the window
    // search reads the right image and pyramid, so they move to the left device over xGMI first
    // (hipMemcpyPeerAsync: the right frame's level 0 and its pyramid slot, ~2.9 MB at 1280x720).
    // ORBGPU_STEREO_STAGE=1 forces the same staging on one device (tests/test_gpu_stereo.py).
    if (cl->device != cr->device || cl->stereo_stage) {
        const size_t f0 = (size_t)cr->last_frame_pitch, pb = (size_t)cr->geom.pyr_bytes;
        const size_t sneed = ((f0 + 255) & ~(size_t)255) + pb;
        if (sneed > cl->peer_cap || !cl->d_peer) {
            if (cl->d_peer) (void)hipFree(cl->d_peer);
            cl->d_peer = nullptr;
            cl->peer_cap = 0;
            if ((e = hipMalloc((void**)&cl->d_peer, sneed)) != hipSuccess) return set_error("stereo peer staging", e), ORB_ERR_NOMEM;
            cl->peer_cap = sneed;
        }
        if (cl->device != cr->device) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, cl->device, cr->device) == hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(cr->device, 0);   // direct xGMI copies
                if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return set_error("peer access", pe), ORB_ERR_HIP;
                (void)hipGetLastError();
            }
        }
        uint8_t* sf = cl->d_peer;
        uint8_t* sp = cl->d_peer + ((f0 + 255) & ~(size_t)255);
        if ((e = hipMemcpyPeerAsync(sf, cl->device, cr->last_frames, cr->device, f0, cl->stream)) != hipSuccess ||
            (pb && (e = hipMemcpyPeerAsync(sp, cl->device, cr->d_pyr, cr->device, pb, cl->stream)) != hipSuccess))
            return set_error("stereo peer copy", e), ORB_ERR_HIP;
        SR.frames = sf;
        SR.pyr = sp;
    }
    if (cl->prof_on) Ctx::marker(cl, ORB_K_STEREO, 1, cl->stream);
    e = launch_stereo(cl->d_geom, cl->geom, SL, SR, 1, mb, mbf, h_u, h_d, d_s, scap, h_nm, cl->stream);
    if (cl->prof_on) Ctx::marker(cl, ORB_K_STEREO, 0, cl->stream);
    if (e != hipSuccess) return set_error("stereo kernels", e), ORB_ERR_HIP;
    if ((e = hipStreamSynchronize(cl->stream)) != hipSuccess) return set_error("stereo sync", e), ORB_ERR_HIP;
    std::memcpy(uright, h_u, (size_t)nL * 4);
    std::memcpy(depth, h_d, (size_t)nL * 4);
    if (nmatched) *nmatched = *h_nm;
    return ORB_OK;
}

int orb_stereo_batch_device(orb_ctx* h, int npairs, float mb, float mbf, float* d_uright, float* d_depth,
                            int* d_nmatched) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (npairs <= 0 || !d_uright || !d_depth || !d_nmatched)
        return set_error("orb_stereo_batch_device: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (!c->last_kps || c->last_nframes < 2 * npairs)
        return set_error("orb_stereo_batch_device: the last batch holds fewer than 2*npairs frames", hipSuccess),
               ORB_ERR_ARG;
    const int cap = c->last_kp_cap;
    const size_t need = stereo_scratch_ints(c->geom, npairs, cap) * 4 + 256;
    hipError_t e;
    if (need > c->scratch_cap || !c->d_scratch) {
        if (c->d_scratch) (void)hipFree(c->d_scratch);
        c->d_scratch = nullptr;
        c->scratch_cap = 0;
        if ((e = hipMalloc((void**)&c->d_scratch, need)) != hipSuccess) return set_error("stereo scratch", e), ORB_ERR_NOMEM;
        c->scratch_cap = need;
    }
    StereoSide SL{c->last_frames, c->last_frame_pitch, c->last_row_stride, c->d_pyr, 0, 2, c->last_kps, c->last_desc,
                  c->last_counts, cap};
    StereoSide SR = SL;
    SR.frame0 = 1;
    if (c->prof_on) Ctx::marker(c, ORB_K_STEREO, 1, c->stream);
    e = launch_stereo(c->d_geom, c->geom, SL, SR, npairs, mb, mbf, d_uright, d_depth, (int*)c->d_scratch, cap,
                      d_nmatched, c->stream);
    if (c->prof_on) Ctx::marker(c, ORB_K_STEREO, 0, c->stream);
    if (e != hipSuccess) return set_error("stereo kernels", e), ORB_ERR_HIP;
    return ORB_OK;
}

}  // extern "C"
