// liborbgpu context (the object behind the opaque orb_ctx*).
#pragma once
#include <algorithm>
#include <array>
#include <cstring>
#include <string>
#include <vector>

#include "orbgpu_internal.h"

namespace orbgpu {

void set_error(const char* what, hipError_t e);

struct ProfPair {
    int id;
    hipEvent_t b, e;
};

struct Ctx {
    orb_params p{};
    int device = 0;
    int num_cu = 256;
    bool fast_stamps = false;     // ORBGPU_FAST_STAMPS=1: the kernels record phase timestamps (diagnostic)
    bool stereo_stage = false;    // ORBGPU_STEREO_STAGE=1: stereo stages the right side as for a peer GPU (test)
    unsigned long long* d_stamps = nullptr;
    size_t stamps_cap = 0;
    hipStream_t stream = nullptr;
    // the host path's second stream and fork / join events (Ctx::run_extract latency mode; ORBGPU_FORK=1: on.  Off by
    // default: 0.1154-0.1198 ms per C3 frame forked against 0.1074 ms in one stream, profiles/r04/v3_host_path.txt)
    bool fork = false;
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;

    // ORBextractor tables (ORBextractor.cc:410-470)
    float scale[ORBGPU_MAX_LEVELS]{}, inv_scale[ORBGPU_MAX_LEVELS]{}, sigma2[ORBGPU_MAX_LEVELS]{},
        inv_sigma2[ORBGPU_MAX_LEVELS]{};
    int n_per_level[ORBGPU_MAX_LEVELS]{};
    int umax[16]{};
    bool umax_ok = false;
    int gk[8]{};

    // geometry of the current image size
    bool have_geom = false;
    Geom geom{};
    int rcoef_off[ORBGPU_MAX_LEVELS]{};
    Geom* d_geom = nullptr;
    size_t geom_cap = 0;
    ResizeCoef* d_rcoef = nullptr;
    size_t rcoef_cap = 0;
    ChainJob* d_chain = nullptr;   // the one-launch pyramid's jobs (small batches)
    size_t chain_cap = 0;
    ChainPlan chain{};
    std::vector<ChainJob> chain_jobs_host;   // (the dataflow launch's chain tasks index them)
    ChainJob* d_chain2 = nullptr;  // the small-batch plan (levels past kSmallChainBase in one launch)
    size_t chain2_cap = 0;
    ChainPlan chain_small{};
    CellDesc* d_cells = nullptr;
    size_t cells_cap = 0;

    // extractor work buffers (capacities in elements)
    uint8_t* d_pyr = nullptr;
    size_t pyr_cap = 0;
    uint32_t* d_cands = nullptr;
    size_t cands_cap = 0;
    uint32_t* d_candFirst = nullptr;
    size_t candfirst_cap = 0;
    uint32_t* d_keys = nullptr;
    size_t keys_cap = 0;
    uint16_t* d_knode = nullptr;
    size_t knode_cap = 0;
    uint32_t* d_lvlKps = nullptr;
    size_t lvlkps_cap = 0;
    int* d_lvlCount = nullptr;
    size_t lvlc_cap = 0;
    int* d_err = nullptr;
    size_t err_cap = 0;

    // host-image path (orb_extract)
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    // streamed upload (k_upload_stream; off by default, ORBGPU_UPLOAD=1 turns it on; off = the pageable
    // hipMemcpy2DAsync): the image's pinned host-coherent staging copy and the per-band flags the host raises (call
    // sequence numbers)
    bool upload_stream = false;
    uint8_t* h_img = nullptr;
    size_t himg_cap = 0;
    uint32_t* h_flags = nullptr;
    uint32_t upload_seq = 0;
    // orb_extract's outputs [count | flag | pad | keypoints | descriptors]: host-coherent pinned memory the
    // kernels write directly (no download)
    void* h_pinned = nullptr;
    size_t pinned_cap = 0;

    // orb_search_for_triangulation's host lists, kept across calls (capacity reused: a call is ~30 us, and its
    // dozens of small allocations were a measurable part of it)
    std::vector<int> tri_item_q, tri_train_of, tri_best, tri_match, tri_ranges;
    std::vector<int> tri_hist[30];
    // orb_hamming_top2_frames_device: the pair list on the device (re-uploaded only when it changes), the list it
    // holds, and two pinned staging slots used in turn
    int* d_pairs = nullptr;
    size_t dpairs_cap = 0;
    std::vector<int> pairs_last;
    int* h_pairs[2] = {nullptr, nullptr};
    size_t pairs_cap[2] = {0, 0};
    hipEvent_t pairs_ev[2] = {nullptr, nullptr};
    int pairs_slot = 0;
    // matcher scratch arena (bytes)
    uint8_t* d_scratch = nullptr;
    size_t scratch_cap = 0;
    // pinned mirror of the matcher arena: a call's inputs are packed here at the device offsets and go up
    // in one DMA, its outputs come back in one (matcher.hip Stage)
    uint8_t* h_mstage = nullptr;
    size_t mstage_cap = 0;
    // the right extractor's frame + pyramid when it runs on another GPU (orb_compute_stereo_matches)
    uint8_t* d_peer = nullptr;
    size_t peer_cap = 0;

    // last batch (for the mvImagePyramid view and debug reads)
    const uint8_t* last_frames = nullptr;
    long long last_frame_pitch = 0;
    int last_row_stride = 0;
    int last_nframes = 0;
    const orb_keypoint* last_kps = nullptr;   // outputs of the last batch (stereo matching reads them)
    const uint8_t* last_desc = nullptr;
    const int* last_counts = nullptr;
    int last_kp_cap = 0;
    unsigned level_cache_valid = 0;
    std::vector<uint8_t> level_host[ORBGPU_MAX_LEVELS];

    // profiling
    bool prof_on = false;
    // Replay of the per-batch launch sequence as a HIP graph (ORBGPU_GRAPH=0 disables): captured on the
    // first batch with a given set of buffers / arguments and re-instantiated when any of them changes
    bool use_graph = true;
    unsigned geom_serial = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    std::array<uintptr_t, 24> gkey{};
    hipEvent_t prof_open[ORB_K_COUNT]{};
    std::vector<ProfPair> prof_pairs;

    // the small-batch dataflow launch (k_extract_flow): batches of at most flow_max_frames frames take it
    // (ORBGPU_FLOW=1; 0, the default, keeps the per-kernel launches); its task list per (geometry, frame count), the
    // counters it waits on
    int flow_max_frames = 0;
    int flow_blocks = 0;            // workgroups per launch (ORBGPU_FLOW_BLOCKS; 0: the default, kFlowDefaultBlocks)
    FlowTask* d_flow = nullptr;
    size_t flow_cap = 0;
    int* d_flow_ctr = nullptr;
    size_t flow_ctr_cap = 0;
    FlowPlan flow{};
    ChainPlan flow_chain_plan{};
    FlowArgs* d_flow_args = nullptr;   // the last uploaded arguments (h_flow_args mirrors them)
    FlowArgs h_flow_args{};
    bool flow_args_valid = false;
    bool flow_stamps = false;       // ORBGPU_FLOW_STAMPS=1: per-task timestamps (orb_debug_fast_stamps returns them)
    unsigned long long* d_flow_stamps = nullptr;
    size_t flow_stamps_cap = 0;
    unsigned flow_serial = 0;       // geom_serial the plan was built for
    bool flow_ok = false;           // flow holds a plan for (flow_serial, flow.nframes)

    int ensure_geometry(int W, int H);
    int ensure_flow(int nframes);
    int ensure_frames(int nframes);
    ExtractBuffers buffers() const;
    // err: the overflow flag the kernels raise (default d_err); err_host: a host-coherent word k_describe
    // copies it to (orb_extract, whose kernels write their outputs straight into pinned memory)
    int run_extract(const uint8_t* d_frames, int nframes, long long frame_pitch, int row_stride, orb_keypoint* d_kps,
                    uint8_t* d_desc, int* d_counts, int kp_cap, int* err = nullptr, bool latency = false,
                    int* err_host = nullptr);
    static void marker(void* user, int id, int begin, hipStream_t s);
};

// The context's device scratch arena (Ctx::d_scratch): reserve the total first, then take() pieces.
struct Arena {
    Ctx* c;
    size_t off = 0;
    static size_t align(size_t x) { return (x + 255) & ~(size_t)255; }
    hipError_t reserve(size_t bytes) {
        if (bytes <= c->scratch_cap && c->d_scratch) return hipSuccess;
        if (c->d_scratch) (void)hipFree(c->d_scratch);
        c->d_scratch = nullptr;
        c->scratch_cap = 0;
        hipError_t e = hipMalloc((void**)&c->d_scratch, bytes);
        if (e == hipSuccess) c->scratch_cap = bytes;
        return e;
    }
    template <class T>
    T* take(size_t n) {
        off = align(off);
        T* p = (T*)(c->d_scratch + off);
        off += std::max<size_t>(n, 1) * sizeof(T);
        return p;
    }
};

// A host call's device arena and its pinned host mirror (Ctx::h_mstage): regions are laid out once
// with add(), inputs are written into the mirror at the device offsets, one DMA takes the input span up
// (or the kernels read the mirror itself, zc = 1), and the kernels store their outputs straight into the mirror
// (host-coherent), so nothing is downloaded.  Regions added after end_mirror() are device-only working space:
// the pinned mirror is not sized for them.
struct Stage {
    Ctx* c;
    size_t off = 0;
    size_t mirror_end = 0;   // 0: every region has a host mirror
    // the call's input mode.  r04 per call (profiles/r04/v3_matcher_zc.txt): the single-kernel calls with small
    // inputs (SearchForTriangulation, ComputeBoW) gain from reading the pinned mirror (zc = 1: no DMA before the
    // kernel); the searches whose kernels re-read their inputs many times (the BoW searches, the window search:
    // every candidate's descriptor; stereo) lose, so they keep the DMA (zc = 0)
    int zc = 0;
    size_t add(size_t bytes) {
        off = Arena::align(off);
        const size_t o = off;
        off += std::max<size_t>(bytes, 1);
        return o;
    }
    void end_mirror() { mirror_end = Arena::align(off); }
    int alloc() {
        const size_t need = Arena::align(off) + 4096;
        Arena a{c};
        hipError_t e = a.reserve(need);
        if (e != hipSuccess) return set_error("matcher scratch", e), ORB_ERR_NOMEM;
        const size_t hneed = (mirror_end ? mirror_end : Arena::align(off)) + 4096;
        if (hneed > c->mstage_cap || !c->h_mstage) {
            if (c->h_mstage) (void)hipHostFree(c->h_mstage);
            c->h_mstage = nullptr;
            c->mstage_cap = 0;
            const size_t cap = std::max<size_t>(hneed, 1 << 20);
            // mapped + coherent explicitly: the matcher kernels store their results straight into this mirror
            // and the host reads them after the stream synchronisation, with no D2H copy
            if ((e = hipHostMalloc((void**)&c->h_mstage, cap, hipHostMallocMapped | hipHostMallocCoherent)) !=
                hipSuccess)
                return set_error("matcher pinned staging", e), ORB_ERR_NOMEM;
            c->mstage_cap = cap;
        }
        return ORB_OK;
    }
    template <class T>
    T* h(size_t o) const { return reinterpret_cast<T*>(c->h_mstage + o); }   // outputs (host view)
    template <class T>
    T* d(size_t o) const { return reinterpret_cast<T*>(c->d_scratch + o); }
    template <class T>
    T* hi(size_t o) const { return reinterpret_cast<T*>(c->h_mstage + o); }   // inputs, written by the host
    template <class T>
    T* di(size_t o) const {   // inputs, as the kernels read them
        return zc ? reinterpret_cast<T*>(c->h_mstage + o) : d<T>(o);
    }
    hipError_t up(size_t from, size_t to) const {
        if (zc) return hipSuccess;   // the kernels read the pinned mirror itself
        return to > from ? hipMemcpyAsync(c->d_scratch + from, c->h_mstage + from, to - from, hipMemcpyHostToDevice,
                                          c->stream)
                         : hipSuccess;
    }
    hipError_t down(size_t from, size_t to) const {
        return to > from ? hipMemcpyAsync(c->h_mstage + from, c->d_scratch + from, to - from, hipMemcpyDeviceToHost,
                                          c->stream)
                         : hipSuccess;
    }
};

}  // namespace orbgpu
