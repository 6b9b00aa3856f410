// liborbgpu context (the object behind the opaque orb_ctx*).
#pragma once
#include <string>
#include <array>
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
    CellDesc* d_cells = nullptr;
    size_t cells_cap = 0;

    // extractor work buffers (capacities in elements)
    uint8_t* d_pyr = nullptr;
    size_t pyr_cap = 0;
    uint32_t* d_cands = nullptr;
    size_t cands_cap = 0;
    int* d_cellCount = nullptr;
    size_t cellc_cap = 0;
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
    // host-path outputs in one allocation, [count | 12 B pad | keypoints | descriptors], so that one
    // download brings all of them back
    uint8_t* d_hout = nullptr;
    size_t hout_cap = 0;
    void* h_pinned = nullptr;     // pinned staging for orb_extract's single download (count, flag, keypoints, descriptors)
    size_t pinned_cap = 0;

    std::vector<int> pairs_upload_host;   // staging for orb_hamming_top2_frames_device pair lists / slots
    // matcher scratch arena (bytes)
    uint8_t* d_scratch = nullptr;
    size_t scratch_cap = 0;
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

    int ensure_geometry(int W, int H);
    int ensure_frames(int nframes);
    ExtractBuffers buffers() const;
    // err: the overflow flag the kernels raise (default d_err; orb_extract passes a word of its output
    // block so that one download brings it back)
    int run_extract(const uint8_t* d_frames, int nframes, long long frame_pitch, int row_stride, orb_keypoint* d_kps,
                    uint8_t* d_desc, int* d_counts, int kp_cap, int* err = nullptr);
    static void marker(void* user, int id, int begin, hipStream_t s);
};

}  // namespace orbgpu
