// The all-pairs Hamming top-2 on the matrix cores: for every query descriptor of a (query set, train set) pair,
// the smallest distance, its train index (first on ties) and the second-smallest distance -- the brute-force
// inner loop of ORBmatcher::SearchByBoW (ORBmatcher.cc:205-226: the strict '<' updates of bestDist1 /
// bestDist2 over one vocabulary node's features; DescriptorDistance :1647-1663).
//
// Distances as an fp4 GEMM.  Descriptor bits become e2m1 values, trains +-4 and queries -+4 (the sign is
// the bit), so q . t = 16 (#different - #equal) = 32 dist - 4096 exactly, and a 32 x 32 tile of distances over
// K = 256 bits is four v_mfma_scale_f32_32x32x64_f8f6f4 (both operands e2m1, unit scales: DESIGN.md §4.6).
// The accumulator starts at 2^23 + 4096 + row, so every result lies in [2^23, 2^24), where an f32's mantissa
// is the integer itself: the low 16 bits of its bit pattern are the tile-local key dist << 5 | row, a finite
// positive f16 (< 2^15) ordered like the integer, and the top-2 runs in f16 min / min3 / med3 (built with
// -fno-honor-nans: no canonicalising ops).
//
// This translation unit holds only the top-2 and its merge (the -fno-honor-nans flag stays off the
// geometry-checking matcher kernels, hamming_kernels.hip).
#include <algorithm>

#include "orbgpu_internal.h"

namespace orbgpu {

namespace {

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));

// Shape (r05 A/B, profiles/r05/hamming_ab.txt): 4 waves x 2 chains, stages of two 32-train tiles, the next stage's
// dwords fetched at the start of the current one, one chain's MFMAs interleaved with the other chain's top-2 (124
// VGPRs, 4 waves per SIMD).  Measured on one box: one tile per stage 143-145 us, two 137-141, four 142 (130
// VGPRs), 8 waves x 2 chains 149-152, fetching two stages ahead 138-139 (equal); the interleaved forms 130-136
// against 131-143 without (two accumulator sets, tile T + 1's MFMAs beside tile T's top-2: 151 VGPRs, 135-136;
// chain-staggered, one set: 130-131).  Diagnostic builds (profiles/r05/hamming_ab.txt): without the MFMAs 92 us,
// with the top-2 cut to one min 85 us, with neither (staging, barriers, fragment reads) 46-47 us: the MFMA and
// top-2 phases still mostly add up.
constexpr int kTile = 32;            // trains per MFMA tile (rows)
constexpr int kTps = 2;              // tiles per stage (one barrier per stage)
constexpr int kTr = kTile * kTps;    // trains per stage
constexpr int kChains = 2;           // query fragments per wave: two independent 32-column MFMA chains
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kQb = kWaves * 32 * kChains;   // queries per workgroup (256)
constexpr int kPitch = 144;          // LDS bytes per expanded train (128 + 16: 36 dwords, so the 16 lanes of a
                                     // ds_read_b128 group hit 16 distinct 4-bank slots)
constexpr int kStageBytes = kTr * kPitch;
constexpr float kSeed = 8388608.f + 4096.f;   // 2^23 + 4096: q . t + seed in [2^23, 2^23 + 8192]

// Descriptor bits -> e2m1 values by byte permutation: output dword j, byte k is tbl[(w >> (8k + 2j)) & 3], the
// two fp4 values of bits 8k + 2j (low nibble) and 8k + 2j + 1.  Queries and trains share this bit -> element
// map (the order of K inside an MFMA does not matter when both operands use the same one).
//   trains:  bit clear -> 0x6 (+4), set -> 0xE (-4):  tbl bytes {66, 6E, E6, EE}
//   queries: bit clear -> 0xE (-4), set -> 0x6 (+4):  tbl bytes {EE, E6, 6E, 66}
constexpr uint32_t kTblTrain = 0xEEE66E66u;
constexpr uint32_t kTblQuery = 0x666EE6EEu;

__device__ __forceinline__ v4i_t expand_fp4(uint32_t w, uint32_t tbl) {
    constexpr uint32_t m = 0x03030303u;
    return v4i_t{(int)__builtin_amdgcn_perm(tbl, tbl, w & m), (int)__builtin_amdgcn_perm(tbl, tbl, (w >> 2) & m),
                 (int)__builtin_amdgcn_perm(tbl, tbl, (w >> 4) & m), (int)__builtin_amdgcn_perm(tbl, tbl, (w >> 6) & m)};
}

// The 16 key bits of an f16 result, read from the whole register and masked.  hipcc (ROCm 7.2) takes the upper
// half of a 16-bit VALU result as zero; on gfx950 it keeps whatever the register held (r04: wrong second
// distances in builds whose allocator had put a 32-bit value there).  The asm hides the assumption.
__device__ __forceinline__ unsigned f16_bits(_Float16 x) {
    unsigned r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r & 0xFFFFu;
}
__device__ __forceinline__ _Float16 f16_of(unsigned bits) { return __builtin_bit_cast(_Float16, (unsigned short)bits); }

constexpr unsigned kInf16 = 0x7C00u;   // f16 +inf: no key

}  // namespace

/* One workgroup: 256 queries (4 waves x 2 chains x 32) of one pair against one train slice, in stages of 64 trains.
 * Per stage every thread expands two train descriptor dwords (v_perm, no table) into LDS (double-buffered, one
 * barrier); per 32-train tile each wave reads the A fragments once (four ds_read_b128) and issues them against both
 * of its query fragments (eight MFMAs, two accumulator chains), each chain's four interleaved with the other
 * chain's top-2.  Each chain's 16 keys per lane go through a two-stream top-2 (min / min3 / med3),
 * and the tile's (best, second) is merged into the running state in the same f16 key space: best replaced only
 * when the tile's distance is strictly smaller (an earlier tile wins a tie), its tile base kept beside it, so the
 * first index wins as the reference's strict '<' does; second = min3(second, tile second, max(best, tile best)). */
__global__ __launch_bounds__(kThreads) void k_top2_mfma(Top2Batch a, uint2* __restrict__ part, int* __restrict__ best_o,
                                                        int* __restrict__ idx_o, int* __restrict__ second_o) {
    __shared__ __attribute__((aligned(16))) uint8_t s_t[2][kStageBytes];
    // 1-D grid of (pair, slice, query block), query block fastest.  Blocks are dealt round-robin over the 8 XCDs
    // (b and b + 8 share one), so XCD x takes a contiguous run of that sequence: the query blocks of a pair, which
    // all stream the same trains, share one L2.
    const int nb = gridDim.x, vb = blockIdx.x, xq = nb >> 3, xr = nb & 7, xcd = vb & 7, xj = vb >> 3;
    const int lb = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + xj;
    const int qbi = lb % a.qblocks, rest = lb / a.qblocks;
    const int sli = rest % a.nslices, p = rest / a.nslices;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int2 fr = a.frames ? a.frames[p] : make_int2(0, 0);
    const int nq = a.counts ? a.counts[fr.x] : a.nq, nt = a.counts ? a.counts[fr.y] : a.nt;
    const int qblk = qbi * kQb;
    if (qblk >= nq) return;   // whole workgroup
    const int t0 = sli * a.slice, t1 = min(nt, t0 + a.slice);
    const int h = lane >> 5, c = lane & 31;
    // B operands: chain u's column c is query qblk + 64 wv + 32 u + c; K-step s = descriptor dwords 2s, 2s + 1,
    // lane half h = dword 2s + h (the A fragments below read the same dword of the train)
    v4i_t qf[kChains][4];
#pragma unroll
    for (int u = 0; u < kChains; u++) {
        const int qi = qblk + 64 * wv + 32 * u + c;
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
        if (qi < nq) {
            const uint4* qp = reinterpret_cast<const uint4*>(a.q + ((long long)fr.x * a.q_stride + qi) * 32);
            q0 = qp[0];
            q1 = qp[1];
        }
        const uint32_t qd[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const uint32_t hm = h ? 0xFFFFFFFFu : 0u;   // (a select, not qd[2 s + h]: a dynamic index goes to scratch)
#pragma unroll
        for (int s = 0; s < 4; s++) qf[u][s] = expand_fp4(qd[2 * s] ^ ((qd[2 * s] ^ qd[2 * s + 1]) & hm), kTblQuery);
    }
    // the slice's packed trains through a buffer descriptor (base and size in SGPRs): rows past t1 read as 0 (their
    // keys are masked), so the last stage needs no clamp (the stage offset goes in voffset: soffset is not
    // range-checked)
    const uint64_t tbase = reinterpret_cast<uint64_t>(a.t + ((long long)fr.y * a.t_stride + t0) * 32);
    const auto TR = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(tbase >> 32)) << 32) |
                                (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)tbase)),
        0, max(t1 - t0, 0) * 32, 0x00020000);
    // staging: thread -> stage rows (tid >> 3) + k * kThreads / 8, descriptor dword tid & 7 (16 expanded bytes each)
    constexpr int kSper = kTr * 8 / kThreads;   // dwords each thread stages
    static_assert(kSper >= 1 && kSper * kThreads == kTr * 8, "staging map");
    const int soff = (tid >> 3) * kPitch + (tid & 7) * 16;
    struct Fetched {
        uint32_t w[kSper];
    };
    auto fetch = [&](int j) -> Fetched {
        Fetched f;
#pragma unroll
        for (int k = 0; k < kSper; k++)
            f.w[k] = __builtin_amdgcn_raw_buffer_load_b32(TR, tid * 4 + k * kThreads * 4 + j * (kTr * 32), 0, 0);
        return f;
    };
    auto stage = [&](int buf, const Fetched& f) {
#pragma unroll
        for (int k = 0; k < kSper; k++)
            *reinterpret_cast<v4i_t*>(&s_t[buf][soff + k * (kThreads / 8) * kPitch]) = expand_fp4(f.w[k], kTblTrain);
    };
    // accumulator seed: 2^23 + 4096 + row, row = the accumulator element's train row in the tile
    v16f_t seed;
#pragma unroll
    for (int r = 0; r < 16; r++) seed[r] = kSeed + (float)((r & 3) + 8 * (r >> 2) + 4 * h);
    // running state per chain: best key (f16 bits dist << 5 | row), its stage base, second key
    _Float16 rb[kChains], rs[kChains];
    int rst[kChains];
#pragma unroll
    for (int u = 0; u < kChains; u++) {
        rb[u] = f16_of(kInf16);
        rs[u] = f16_of(kInf16);
        rst[u] = 0;
    }
    // a chain's stage top-2 in two independent streams (rows r = 0..7 and 8..15, keys taken in pairs), merged,
    // then folded into the running state
    auto top2 = [&](const v16f_t& acc, int u, int tb, auto keep) {
        auto key = [&](int r) {
            const float kv = acc[r];   // (via a scalar: clang's bit_cast of an ext_vector element reads element 0)
            const int ki = __builtin_bit_cast(int, kv);
            return keep(r) ? __builtin_bit_cast(_Float16, (unsigned short)ki) : f16_of(kInf16);
        };
        _Float16 b2[2], s2[2];
#pragma unroll
        for (int st = 0; st < 2; st++) {
            const _Float16 x0 = key(8 * st), x1 = key(8 * st + 1);
            b2[st] = __builtin_fminf16(x0, x1);
            s2[st] = __builtin_fmaxf16(x0, x1);
#pragma unroll
            for (int r = 8 * st + 2; r < 8 * st + 8; r += 2) {
                // second smallest of {best <= second, x, y}: min(second, med3(best, x, y)) (a stage's keys are distinct)
                const _Float16 x = key(r), y = key(r + 1);
                s2[st] = __builtin_fminf16(s2[st], __builtin_amdgcn_fmed3h(b2[st], x, y));
                b2[st] = __builtin_fminf16(__builtin_fminf16(b2[st], x), y);
            }
        }
        const _Float16 sb = __builtin_fminf16(b2[0], b2[1]);
        const _Float16 ss = __builtin_fminf16(__builtin_fminf16(s2[0], s2[1]), __builtin_fmaxf16(b2[0], b2[1]));
        // running merge: the stage's best replaces the running one only at a strictly smaller distance (its key
        // below the running key with the row bits cleared)
        const bool take = sb < f16_of(f16_bits(rb[u]) & 0xFFE0u);
        rs[u] = __builtin_fminf16(__builtin_fminf16(rs[u], ss), __builtin_fmaxf16(rb[u], sb));
        rb[u] = take ? sb : rb[u];
        rst[u] = take ? tb : rst[u];
    };
    const int nst = t1 > t0 ? (t1 - t0 + kTr - 1) / kTr : 0;   // stages (uniform)
    // chain-staggered: one chain's four MFMAs interleaved with the other chain's top-2, so a single accumulator per
    // chain suffices (no second set): phase (t, 1) = MFMAs of chain 1, tile t + top-2 of chain 0, tile t; phase
    // (t, 0) = MFMAs of chain 0, tile t + 1 + top-2 of chain 1, tile t.  A tile's A fragments are read once and
    // serve both phases that use them.
    auto frags = [&](int buf, int tile, v8i_t (&a8)[4]) {
        const uint8_t* A = &s_t[buf][(kTile * tile + c) * kPitch + 16 * h];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const v4i_t av = *reinterpret_cast<const v4i_t*>(A + 32 * s);
            a8[s] = v8i_t{av[0], av[1], av[2], av[3], 0, 0, 0, 0};
        }
    };
    auto mfma_chain = [&](const v8i_t (&a8)[4], int u, v16f_t& acc) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const v8i_t b8 = {qf[u][s][0], qf[u][s][1], qf[u][s][2], qf[u][s][3], 0, 0, 0, 0};
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8[s], b8, s == 0 ? seed : acc, 4, 4, 0, 0, 0, 0);
        }
    };
    auto inter4 = [&]() {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);   // eight VALU
        }
    };
    auto all = [](int) { return true; };
    if (nst > 0) {
        stage(0, fetch(0));
        __syncthreads();
        v16f_t acc0, acc1;
        v8i_t fa[4], fb[4];
        frags(0, 0, fa);
        mfma_chain(fa, 0, acc0);
        for (int j = 0; j + 1 < nst; j++) {
            const Fetched wn = fetch(j + 1);
            const int tb = t0 + kTr * j;
            mfma_chain(fa, 1, acc1);   // tile 2j, chain 1
            top2(acc0, 0, tb, all);
            inter4();
            frags(j & 1, 1, fb);
            mfma_chain(fb, 0, acc0);   // tile 2j + 1, chain 0
            top2(acc1, 1, tb, all);
            inter4();
            mfma_chain(fb, 1, acc1);   // tile 2j + 1, chain 1
            top2(acc0, 0, tb + kTile, all);
            inter4();
            stage((j + 1) & 1, wn);
            __syncthreads();
            frags((j + 1) & 1, 0, fa);
            mfma_chain(fa, 0, acc0);   // tile 2j + 2, chain 0
            top2(acc1, 1, tb + kTile, all);
            inter4();
        }
        const int j = nst - 1, tb = t0 + kTr * j;
        auto masked = [&](int tb_) {
            return [=](int r) { return tb_ + (r & 3) + 8 * (r >> 2) + 4 * h < t1; };
        };
        mfma_chain(fa, 1, acc1);
        top2(acc0, 0, tb, masked(tb));
        top2(acc1, 1, tb, masked(tb));
        frags(j & 1, 1, fb);
        mfma_chain(fb, 0, acc0);
        mfma_chain(fb, 1, acc1);
        top2(acc0, 0, tb + kTile, masked(tb + kTile));
        top2(acc1, 1, tb + kTile, masked(tb + kTile));
    }
    // per chain: running keys -> dist << 16 | train index; the two lane halves hold different train rows of the
    // same query
#pragma unroll
    for (int u = 0; u < kChains; u++) {
        const unsigned kb = f16_bits(rb[u]), ks = f16_bits(rs[u]);
        unsigned b = kb == kInf16 ? 0xFFFFFFFFu : ((kb >> 5) << 16) | (unsigned)(rst[u] + (int)(kb & 31u));
        // the second's index is never output: dist << 16 | 0xFFFF orders it after any equal best
        unsigned s2 = ks == kInf16 ? 0xFFFFFFFFu : ((ks >> 5) << 16) | 0xFFFFu;
        const unsigned ob = __shfl_xor(b, 32), os = __shfl_xor(s2, 32);
        s2 = min(min(s2, os), max(b, ob));
        b = min(b, ob);
        const int qi = qblk + 64 * wv + 32 * u + c;
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
    }
}

/* Slices of one (query set, train set) pair's top-2 (k_top2_mfma with nslices > 1) are merged here: keys
 * dist << 16 | train index compose by min (first index on ties) and second = the second-smallest key.  Counts
 * may be read on the device (an extraction batch's d_counts), so a whole batch of frame pairs needs no host round
 * trip. */
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

// Train slices: a launch aims at >= kTargetBlocks workgroups (two rounds of four per CU); slices are whole 32-train
// stages of >= 64 trains.  top2_batch_slices is the partial buffer's capacity (the callers size it), the launch
// uses top2_launch_slices <= that many.  (max_nt == 0: one empty slice of one stage, nothing divides by zero.)
constexpr int kTargetBlocks = 8192 / kWaves;   // 8192 waves
int top2_batch_slices(int npairs, int max_nq, int max_nt) {
    npairs = std::max(npairs, 1);
    const int qb = std::max(1, (max_nq + kQb - 1) / kQb);
    int ns = (kTargetBlocks + npairs * qb - 1) / (npairs * qb);
    ns = std::min(ns, std::max(1, (max_nt + 63) / 64));
    return std::max(ns, 1);
}

static int top2_slice_len(int npairs, int max_nq, int max_nt) {
    const int ns = top2_batch_slices(npairs, max_nq, max_nt);
    return std::max(((max_nt + ns - 1) / ns + kTr - 1) / kTr * kTr, kTr);
}

int top2_launch_slices(int npairs, int max_nq, int max_nt) {
    if (npairs <= 0 || max_nq <= 0 || max_nt < 0) return 0;
    const int len = top2_slice_len(npairs, max_nq, max_nt);
    return std::max(1, (max_nt + len - 1) / len);
}

hipError_t launch_hamming_top2_batch(const Top2Batch& a0, int npairs, int max_nq, int max_nt, int* d_best,
                                     int* d_best_idx, int* d_second, uint2* d_part, hipStream_t stream) {
    if (npairs <= 0 || max_nq <= 0) return hipSuccess;
    if (max_nt > 65535) return hipErrorInvalidValue;   // keys hold a 16-bit train index
    Top2Batch a = a0;
    a.slice = top2_slice_len(npairs, max_nq, max_nt);
    const int nsu = std::max(1, (max_nt + a.slice - 1) / a.slice);   // 1: k_top2_mfma writes the outputs itself
    a.qblocks = (max_nq + kQb - 1) / kQb;
    a.nslices = nsu;
    const long long blocks = (long long)a.qblocks * nsu * npairs;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    // (max_nt == 0, e.g. a previous frame without keypoints: k_top2_mfma sees no stage and writes the sentinels)
    hipLaunchKernelGGL(k_top2_mfma, dim3((unsigned)blocks), dim3(kThreads), 0, stream, a, d_part, d_best, d_best_idx,
                       d_second);
    if (nsu > 1)
        hipLaunchKernelGGL(k_top2b_merge, dim3((max_nq + 255) / 256, npairs), dim3(256), 0, stream, a, nsu, d_part,
                           d_best, d_best_idx, d_second);
    return hipGetLastError();
}

}  // namespace orbgpu
