// DBoW2 vocabulary transform on gfx950: Frame::ComputeBoW / KeyFrame::ComputeBoW
// (Frame.cc:562-569, KeyFrame.cc:74-83) call TemplatedVocabulary::transform(features, BowVector&,
// FeatureVector&, 4) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1139-1210), whose per-feature
// part is a k-ary tree descent with a Hamming distance at every level (:1240-1277).  That descent
// runs here, one lane per feature; the (word, weight, node) triples are assembled into the
// BowVector / FeatureVector maps on the host in feature order (orb_vocab_bow), as the reference
// accumulates them.
//
// The vocabulary is read with the reference's binary loader semantics (:1466-1510) — including its
// while(!f.eof()) quirk, which appends a duplicate of the last record as an extra child of its
// parent (it never wins the strict '<' of the descent) — and laid out for the device with every
// node's children contiguous (child ids + child descriptors in child order).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "orbgpu_ctx.h"

struct orb_vocab {
    int device;
    int k, L, scoring, weighting, nnodes, nwords;
    int* d_cbeg = nullptr;        // per node: first child slot
    int* d_ccnt = nullptr;        // per node: #children (0 = leaf)
    int* d_child = nullptr;       // per child slot: node id
    uint8_t* d_cdesc = nullptr;   // per child slot: 32-byte descriptor
    int* d_word = nullptr;        // per node: word id (-1 for internal nodes)
    float* d_weight = nullptr;    // per node: weight (stored as float in the file)
};

namespace orbgpu {

constexpr int kVocabMaxDepth = 64;   // descent bound: every lane exits even on a malformed tree

__global__ __launch_bounds__(256) void k_vocab_transform(const int* __restrict__ cbeg, const int* __restrict__ ccnt,
                                                         const int* __restrict__ child,
                                                         const uint8_t* __restrict__ cdesc,
                                                         const int* __restrict__ word, const float* __restrict__ weight,
                                                         const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                         int n_fixed, long long slot_stride, int nid_level,
                                                         int* __restrict__ word_out, float* __restrict__ weight_out,
                                                         uint32_t* __restrict__ node_out) {
    const int f = blockIdx.y;
    const int n = counts ? counts[f] : n_fixed;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const long long slot = (long long)f * slot_stride + i;
    const uint4* fp = reinterpret_cast<const uint4*>(desc + slot * 32);
    const uint4 a = fp[0], b = fp[1];
    int node = 0;
    uint32_t nid = 0;   // nid_level <= 0: the root (:1250); also if a leaf comes first (uninitialised upstream)
    for (int level = 1; level <= kVocabMaxDepth; level++) {
        const int c0 = cbeg[node], nc = ccnt[node];
        if (nc <= 0) break;
        const uint4* cd = reinterpret_cast<const uint4*>(cdesc + (long long)c0 * 32);
        int best = 0, bd = 257;
        for (int j = 0; j < nc; j++) {
            const uint4 x = cd[2 * j], y = cd[2 * j + 1];
            const int d = __popc(a.x ^ x.x) + __popc(a.y ^ x.y) + __popc(a.z ^ x.z) + __popc(a.w ^ x.w) +
                          __popc(b.x ^ y.x) + __popc(b.y ^ y.y) + __popc(b.z ^ y.z) + __popc(b.w ^ y.w);
            if (d < bd) {   // first minimum (strict '<', :1262-1266)
                bd = d;
                best = j;
            }
        }
        node = child[c0 + best];
        if (level == nid_level) nid = (uint32_t)node;
        if (ccnt[node] == 0) break;   // isLeaf()
    }
    word_out[slot] = word[node];
    weight_out[slot] = weight[node];
    node_out[slot] = nid;
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

static void vocab_free(orb_vocab* v) {
    if (!v) return;
    (void)hipSetDevice(v->device);
    void* bufs[] = {v->d_cbeg, v->d_ccnt, v->d_child, v->d_cdesc, v->d_word, v->d_weight};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    delete v;
}

extern "C" {

int orb_vocab_load(orb_ctx* h, const char* path, orb_vocab** out) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!path || !out) return set_error("orb_vocab_load: bad arguments", hipSuccess), ORB_ERR_ARG;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return set_error("orb_vocab_load: cannot open the vocabulary file", hipSuccess), ORB_ERR_ARG;
    unsigned int nb_nodes = 0, size_node = 0;
    int hdr[4];
    if (std::fread(&nb_nodes, 4, 1, f) != 1 || std::fread(&size_node, 4, 1, f) != 1 || std::fread(hdr, 4, 4, f) != 4 ||
        size_node != 4 + 32 + 4 + 1 || nb_nodes == 0 || nb_nodes > (1u << 26)) {
        std::fclose(f);
        return set_error("orb_vocab_load: not a DBoW2 binary vocabulary of 32-byte descriptors", hipSuccess),
               ORB_ERR_ARG;
    }
    // TemplatedVocabulary::loadFromBinaryFile (:1466-1510), eof quirk included
    const int nn = (int)nb_nodes + 1;
    std::vector<int> parent(nn, 0), word(nn, -1);
    std::vector<float> weight(nn, 0.f);
    std::vector<uint8_t> desc((size_t)nn * 32, 0);
    std::vector<std::vector<int>> children(nn);
    std::vector<char> buf(size_node, 0);
    int nid = 1, nwords = 0;
    for (;;) {
        const size_t got = std::fread(buf.data(), 1, size_node, f);
        if (nid >= nn) break;
        int par;
        std::memcpy(&par, buf.data(), 4);
        if (par < 0 || par >= nn) {
            std::fclose(f);
            return set_error("orb_vocab_load: parent index out of range", hipSuccess), ORB_ERR_ARG;
        }
        parent[nid] = par;
        children[par].push_back(nid);
        std::memcpy(&desc[(size_t)nid * 32], buf.data() + 4, 32);
        std::memcpy(&weight[nid], buf.data() + 36, 4);
        if (buf[40]) word[nid] = nwords++;
        nid += 1;
        if (got < size_node) break;
    }
    std::fclose(f);
    // device layout: children contiguous
    std::vector<int> cbeg(nn), ccnt(nn), child;
    std::vector<uint8_t> cdesc;
    child.reserve(nn);
    cdesc.reserve((size_t)nn * 32);
    for (int n = 0; n < nn; n++) {
        cbeg[n] = (int)child.size();
        ccnt[n] = (int)children[n].size();
        for (int ch : children[n]) {
            child.push_back(ch);
            cdesc.insert(cdesc.end(), &desc[(size_t)ch * 32], &desc[(size_t)ch * 32] + 32);
        }
    }
    if (child.empty()) {
        child.push_back(0);
        cdesc.resize(32, 0);
    }
    orb_vocab* v = new (std::nothrow) orb_vocab();
    if (!v) return ORB_ERR_NOMEM;
    v->device = c->device;
    v->k = hdr[0];
    v->L = hdr[1];
    v->scoring = hdr[2];
    v->weighting = hdr[3];
    v->nnodes = nn;
    v->nwords = nwords;
    hipError_t e;
    if ((e = hipMalloc((void**)&v->d_cbeg, nn * 4)) != hipSuccess || (e = hipMalloc((void**)&v->d_ccnt, nn * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&v->d_child, child.size() * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&v->d_cdesc, cdesc.size())) != hipSuccess ||
        (e = hipMalloc((void**)&v->d_word, nn * 4)) != hipSuccess ||
        (e = hipMalloc((void**)&v->d_weight, nn * 4)) != hipSuccess) {
        vocab_free(v);
        return set_error("orb_vocab_load: device allocation", e), ORB_ERR_NOMEM;
    }
    if ((e = hipMemcpy(v->d_cbeg, cbeg.data(), nn * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(v->d_ccnt, ccnt.data(), nn * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(v->d_child, child.data(), child.size() * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(v->d_cdesc, cdesc.data(), cdesc.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(v->d_word, word.data(), nn * 4, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(v->d_weight, weight.data(), nn * 4, hipMemcpyHostToDevice)) != hipSuccess) {
        vocab_free(v);
        return set_error("orb_vocab_load: upload", e), ORB_ERR_HIP;
    }
    *out = v;
    return ORB_OK;
}

void orb_vocab_destroy(orb_vocab* v) { vocab_free(v); }

int orb_vocab_info(const orb_vocab* v, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords) {
    if (!v) return ORB_ERR_ARG;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (nnodes) *nnodes = v->nnodes;
    if (nwords) *nwords = v->nwords;
    return ORB_OK;
}

int orb_vocab_transform(orb_ctx* h, const orb_vocab* v, const uint8_t* desc, int n, int levelsup, int* word_id,
                        float* weight, uint32_t* node_id) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!v || v->device != c->device || n < 0 || (n && (!desc || !word_id || !weight || !node_id)))
        return set_error("orb_vocab_transform: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (n == 0) return ORB_OK;
    // one DMA up (descriptors) through the context's pinned staging; the results come back by the kernel's
    // own stores to it
    Stage st{c};
    st.zc = 1;   // the descriptors are read once per tree level from L2 after the first touch (Stage::zc)
    const size_t o_desc = st.add((size_t)n * 32), o_w = st.add((size_t)n * 4), o_wt = st.add((size_t)n * 4),
                 o_nd = st.add((size_t)n * 4), o_end = st.off;
    const int r = st.alloc();
    if (r != ORB_OK) return r;
    std::memcpy(st.hi<uint8_t>(o_desc), desc, (size_t)n * 32);
    hipError_t e = st.up(o_desc, o_w);
    if (e != hipSuccess) return set_error("vocab upload", e), ORB_ERR_HIP;
    hipLaunchKernelGGL(k_vocab_transform, dim3((n + 255) / 256, 1), dim3(256), 0, c->stream, v->d_cbeg, v->d_ccnt,
                       v->d_child, v->d_cdesc, v->d_word, v->d_weight, st.di<uint8_t>(o_desc), nullptr, n, 0,
                       v->L - levelsup, st.h<int>(o_w), st.h<float>(o_wt), st.h<uint32_t>(o_nd));
    if ((e = hipGetLastError()) != hipSuccess) return set_error("vocab kernel", e), ORB_ERR_HIP;
    // the kernel writes [word | weight | node] straight into the pinned mirror: no D2H command
    (void)o_end;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return set_error("vocab sync", e), ORB_ERR_HIP;
    std::memcpy(word_id, st.h<int>(o_w), (size_t)n * 4);
    std::memcpy(weight, st.h<float>(o_wt), (size_t)n * 4);
    std::memcpy(node_id, st.h<uint32_t>(o_nd), (size_t)n * 4);
    return ORB_OK;
}

int orb_vocab_transform_batch_device(orb_ctx* h, const orb_vocab* v, int nframes, int levelsup, int* d_word,
                                     float* d_weight, uint32_t* d_node) {
    Ctx* c = reinterpret_cast<Ctx*>(h);
    CTX_GUARD(c);
    if (!v || v->device != c->device || nframes <= 0 || !d_word || !d_weight || !d_node)
        return set_error("orb_vocab_transform_batch_device: bad arguments", hipSuccess), ORB_ERR_ARG;
    if (!c->last_desc || c->last_nframes < nframes)
        return set_error("orb_vocab_transform_batch_device: no such frames in the last batch", hipSuccess),
               ORB_ERR_ARG;
    const int cap = c->last_kp_cap;
    hipLaunchKernelGGL(k_vocab_transform, dim3((cap + 255) / 256, nframes), dim3(256), 0, c->stream, v->d_cbeg,
                       v->d_ccnt, v->d_child, v->d_cdesc, v->d_word, v->d_weight, c->last_desc, c->last_counts, 0,
                       (long long)cap, v->L - levelsup, d_word, d_weight, d_node);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? ORB_OK : (set_error("vocab kernel", e), ORB_ERR_HIP);
}

int orb_vocab_bow(const orb_vocab* v, int n, const int* word_id, const float* weight, const uint32_t* node_id,
                  int* bow_words, double* bow_values, int* nbow, uint32_t* fv_nodes, int* fv_off, int* fv_idx,
                  int* nfv) {
    if (!v || n < 0 || !nbow || !nfv || !fv_off || (n && (!word_id || !weight || !node_id || !bow_words ||
                                                          !bow_values || !fv_nodes || !fv_idx)))
        return ORB_ERR_ARG;
    // TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup) (:1139-1210).
    // std::map order = ascending word / node id, and within a word / node the features in input order:
    // sorting (id, feature) keys gives the same order and the same summation order as the map inserts.
    const bool tf = v->weighting == 0 || v->weighting == 1;   // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    const bool must = v->scoring != 5;                        // DotProductScoring does not normalise
    const bool l1 = v->scoring != 1;                          // L2Scoring normalises with L2
    int b = 0, j = 0, o = 0;
    fv_off[0] = 0;
    if (v->nwords > 0) {   // if(empty()) return; (:1146-1149)
        std::vector<unsigned long long> kw, kn;
        kw.reserve(n);
        kn.reserve(n);
        for (int i = 0; i < n; i++)
            if ((double)weight[i] > 0) {   // not stopped
                kw.push_back(((unsigned long long)(uint32_t)word_id[i] << 32) | (uint32_t)i);
                kn.push_back(((unsigned long long)node_id[i] << 32) | (uint32_t)i);
            }
        std::sort(kw.begin(), kw.end());
        std::sort(kn.begin(), kn.end());
        for (size_t a = 0; a < kw.size();) {
            const uint32_t w = (uint32_t)(kw[a] >> 32);
            double acc = (double)weight[(uint32_t)kw[a]];
            size_t e = a + 1;
            for (; e < kw.size() && (uint32_t)(kw[e] >> 32) == w; e++)
                if (tf) acc += (double)weight[(uint32_t)kw[e]];   // bow[word] += w, in feature order
            bow_words[b] = (int)w;
            bow_values[b] = acc;
            b++;
            a = e;
        }
        if (tf && b > 0 && !must)
            for (int i = 0; i < b; i++) bow_values[i] /= (double)b;
        if (must) {   // BowVector::normalize (BowVector.cpp:61-86), in map order
            double norm = 0.0;
            if (l1) {
                for (int i = 0; i < b; i++) norm += std::fabs(bow_values[i]);
            } else {
                for (int i = 0; i < b; i++) norm += bow_values[i] * bow_values[i];
                norm = std::sqrt(norm);
            }
            if (norm > 0.0)
                for (int i = 0; i < b; i++) bow_values[i] /= norm;
        }
        for (size_t a = 0; a < kn.size(); a++) {   // FeatureVector::addFeature (FeatureVector.cpp:31-45)
            const uint32_t nd = (uint32_t)(kn[a] >> 32);
            if (a == 0 || (uint32_t)(kn[a - 1] >> 32) != nd) {
                if (a) fv_off[++j] = o;
                fv_nodes[j] = nd;
            }
            fv_idx[o++] = (int)(uint32_t)kn[a];
        }
        if (!kn.empty()) fv_off[++j] = o;
    }
    *nbow = b;
    *nfv = j;
    return ORB_OK;
}

}  // extern "C"
