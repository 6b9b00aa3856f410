// Internal types shared by the host side and the gfx950 kernels of liborbgpu.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/orbgpu.h"

namespace orbgpu {

constexpr int kEdgeThreshold = 19;    // ORBextractor.cc:74
constexpr int kMinBorder = kEdgeThreshold - 3;   // :773
constexpr int kPatchSize = 31;        // :72
constexpr int kHalfPatch = 15;        // :73
constexpr int kMaxDim = 4096;         // candidate coordinates are packed in 12 bits
constexpr int kFastTilePitch = 80;    // 16-bit elements per FAST tile row (ROI <= 66 px, prefilter window <= 74)
constexpr int kFastMaxRoi = 66;
constexpr int kOctreeThreads = 512;
constexpr int kCandRec = 8;           // dwords per cell in d_candFirst: [corner count | first kCandFirst corners]
constexpr int kCandFirst = kCandRec - 1;
constexpr int kDescWin = 43;          // unblurred window: radius 18 (BRIEF) + 3 (blur taps)
constexpr int kDescWinPitch = 48;       // 12 dwords: window rows are loaded as aligned dwords
constexpr int kDescBlur = 37;         // blurred window: radius 18
constexpr int kDescBlurPitch = 40;
constexpr int kRtPitch = 44;          // k_describe row-pass sums RT[column][row], u16, 43 rows + 1 (even: the
                                      // MFMA row pass stores four rows of a column as one 8-byte write)
constexpr int kDescTapTiles = 3;      // k_describe MFMA row pass: 16-column tiles of RT (37 columns used)
constexpr int kRsTileW = 128;         // k_resize_tiled<TH>: output tile 128 x TH, 4 px per thread
constexpr int kRsPitch = 272;         // LDS source tile: up to 272 bytes (from a 16-B aligned column) x (2*TH + 8) rows
constexpr int rs_rows(int th) { return 2 * th + 8; }

// Per-level geometry (host-computed once per image size; lives in device memory).
struct LevelGeom {
    int w, h;            // level size (ComputePyramid, ORBextractor.cc:1112)
    int pitch;           // row pitch of the stored level (levels >= 1)
    int rs_tiled;        // bit i: k_resize_tiled<16 << i>'s LDS tile holds every source span (else k_resize)
    long long pyr_off;   // byte offset of the level inside a frame's pyramid slot (levels >= 1)
    int maxBX, maxBY;    // maxBorderX/Y (:775-776)
    int nCols, nRows, wCell, hCell;   // cell grid (:781-787)
    int cell_base;       // first cell of the level within a frame
    int cell_cap;        // candidate slots per cell: ceil(wCell/2)*ceil(hCell/2) (NMS independent set)
    int cand_base;       // first candidate slot of the level within a frame
    int cand_cap;        // candidate slots of the level
    int nfeat;           // mnFeaturesPerLevel (:435-446)
    int kp_cap, kp_base; // octree output slots
    int nIni;            // DistributeOctTree root count (:543)
    float hX;            // root width (:545)
    float scale;         // mvScaleFactor
    float patch_size;    // (int)(PATCH_SIZE*scale) (:837)
    int rs_span_rows;    // k_resize_tiled: the largest source span (rows) of a tile: its LDS tile height
    int rs_chunks;       // k_resize_tiled: the most 16-byte source chunks of a tile (rows x chunks per row), so
                         // the launch issues ceil(rs_chunks / 256) loads per thread, not the worst case's
};

struct Geom {
    int nlevels, W, H;
    int ncells;          // cells per frame
    int ncand;           // candidate slots per frame
    int nkpcap;          // octree output slots per frame
    long long pyr_bytes; // pyramid bytes per frame (levels >= 1)
    int iniTh, minTh;
    int variant;         // ORB_VARIANT_* bits (orb_params.variant): the OpenCV arithmetic variant
    int node_cap;        // octree LDS node capacity
    int max_level_cand;  // max cand_cap over levels (octree key scratch per level)
    int fast_rows;       // k_fast_wave per-wave LDS carve (max over levels): ROI rows,
    int fast_drows;      //   detection-domain rows,
    int fast_list;       //   prefilter-survivor list entries (domain pixels)
    int fast_wave_bytes; //   bytes per wave (lead pad | 16-bit tile | survivor list)
    int fast_compact;    //   every cell <= 36 px wide: compact tile pitch (48 elements; else kFastTilePitch)
    int umax[16];        // ORBextractor.cc:454-469
    int gk[8];           // 7-tap Gaussian, sigma 2, 8-bit fixed point (getGaussianKernel x 256)
    LevelGeom L[ORBGPU_MAX_LEVELS];
    // k_describe's row pass as int8 MFMA (v_mfma_i32_16x16x64_i8): the B fragments of the banded tap matrix
    // T[k][c] = gk[k - sh - c] (0 <= k - sh - c <= 6, else 0) for window shift sh, column tile tc and lane l:
    // bytes e = 0..15 of desc_taps[(sh * kDescTapTiles + tc) * 64 + l] are T[16 (l >> 4) + e][16 tc + (l & 15)]
    int4 desc_taps[4 * kDescTapTiles * 64];
};

// Per-cell descriptor of the FAST grid (host-built once per image size; k_fast_wave reads one per
// wavefront with a single scalar load instead of decoding the cell from the level tables).
struct CellDesc {
    int lv;        // level | valid << 8
    int iniX, iniY;
    int rwrh;      // ROI width | height << 16 (clipped, ORBextractor.cc:791-806)
    int out_off;   // first candidate slot of the cell within a frame
    int xoyo;      // output coordinate offsets (3 + cj*wCell) | (3 + ci*hCell) << 16 (:822-823)
    int pitch;     // level row pitch (levels >= 1)
    int pyr_off;   // level offset in a frame's pyramid slot (levels >= 1)
    // lane mappings of k_fast_wave, precomputed so the kernel divides nothing (a wave-uniform 32-bit
    // division costs ~15 VALU instructions, one of them a transcendental v_rcp):
    int roi;       // ROI load: dwords per row nw | rows per round (64 / nw) << 8 | first dword (iniX >> 2) << 16
    int m_nw;      // recip20(nw)
    int runs;      // prefilter: 16-pixel runs per row nruns | rows per round (64 / nruns) << 8
    int m_runs;    // recip20(nruns)
    int pad[4];    // 64 bytes: one scalar dwordx16 load
};
// q = x / n for x < 2^20 / n, from m = recip20(n) (host and device)
__host__ __device__ inline uint32_t recip20(uint32_t n) { return ((1u << 20) + n - 1) / n; }

// cv::resize INTER_LINEAR coefficient tables (OpenCV 3.2 imgwarp.cpp), one entry per dst column/row.
struct ResizeCoef {
    int s0, s1;          // source column/row indices (clamped)
    int c0, c1;          // 11-bit fixed-point weights (saturate_cast<short>(w*2048))
};

// One workgroup of k_pyramid_chain (the few-launch pyramid of small batches): an output tile of
// `level`, computed from level `base` (the frame, or a level an earlier launch wrote) through the
// region reg[k] = (x0, x1, y0, y1) of every level k = base .. level - 1 its pixels depend on (levels
// above base: x0 and x1 - x0 multiples of 4, so every stage writes dwords).
struct ChainJob {
    int level, base, pad0, pad1;
    int4 reg[ORBGPU_MAX_LEVELS];
};
// Plan of k_pyramid_chain, host-built once per image size (orbgpu_abi.hip build_chain): the levels in
// segments of up to kChainSeg, one launch each; a segment's jobs are contiguous, in level order.  LDS
// carve per launch = two region buffers (ping-pong) + the stages' coefficient slots.
constexpr int kChainSeg = 4;
struct ChainSegment {
    int job0 = 0, njobs = 0;
    int buf_bytes = 0, coef_entries = 0, lds_bytes = 0;
};
struct ChainPlan {
    int nseg = 0;           // 0: the plan does not fit (per-level launches only)
    int first_base = 0;     // levels 1..first_base are per-level launches before the segments
    ChainSegment seg[ORBGPU_MAX_LEVELS];
};
// Batches of up to kChainMaxFrames frames in the batch path (C5 at one frame per GPU) compute levels 1..3 with one
// launch each and levels 4..7 from level 3 in one k_pyramid_chain launch (r05, profiles/r05/c5b1_pyramid_ab.txt: C5
// one frame per step, four in flight, 171 M features/s against 164-169 with seven per-level launches; chaining from
// level 2 157-159, level 1 137, level 4 167-174: the chained launch's per-tile level walk is long, so only the small
// top levels pay for their launches)
constexpr int kSmallChainBase = 3;
constexpr int kChainMaxFrames = 2;
struct RcoefOff {   // per-level offsets into the coefficient table (a kernel argument)
    int o[ORBGPU_MAX_LEVELS];
};   // batches up to this many frames take the one-launch pyramid

// The small-batch dataflow launch (k_extract_flow, extract_kernels.hip): one persistent launch of 1024-thread
// workgroups that take (stage, level, frame) tasks from a device ticket in a host-built topological order and wait
// only on the per-(frame, level) counters of what each task reads: level l's FAST / octree / describe start as soon
// as level l exists, independent of the other levels (ComputeKeyPointsOctTree loops per level, ORBextractor.cc:
// 765-853; operator() per level, :1076-1103).  Tasks: a resize task = up to 4 output tiles of one level (a 256-thread
// quarter each), a FAST task = up to 16 cells (a wave each), an octree task = one (frame, level) (the block), a
// describe task = up to 16 keypoint slots of one level (a wave each).
enum FlowKind : int { kFlowResize = 0, kFlowFast = 1, kFlowOctree = 2, kFlowDescribe = 3, kFlowChain = 4 };
struct FlowTask {   // 32 B (one scalar dwordx8 load)
    int klf;       // kind | level << 8 | frame << 16
    int sig;       // counter raised when the task is done (-1: none)
    int a, b;      // resize: first tile, tiles; FAST: first cell of the level, cells; describe: first keypoint slot
                   // (frame-local), slots
    int dep, nd;   // wait until counters dep .. dep + nd - 1 each reach tgt (nd = 0: no wait)
    int tgt;
    int seg;       // chain task: its segment of the chain plan (a = first ChainJob, b = jobs, one per quarter)
};
struct FlowPlan {
    int ntasks = 0;
    int nframes = 0;
    int nctr = 0;          // counter words (zeroed once; the launch's last workgroup re-zeroes them)
    int lds_bytes = 0;     // dynamic LDS of the launch
    int lds_keys = 0;      // octree keys kept in LDS
    int rs_quarter = 0;    // LDS bytes of one resize quarter (source tile + coefficient slots)
    int blocks = 0;        // workgroups of the launch
};
// counter layout: [0] ticket, [16] workgroups done, [32] octrees done, [48] timeout flag, then per frame f at
// kFlowCtrBase + 4 nl f: resize tasks done [nl], FAST tasks done [nl], octree done [nl], octree error bits [nl]
constexpr int kFlowCtrBase = 64;
constexpr int kFlowThreads = 1024;
constexpr int kFlowDefaultBlocks = 64;   // workgroups per frame of a dataflow launch (a quarter of the CUs: four
                                         // launches in flight, one per hardware queue, fill the chip)
// build the task list of nframes frames for geometry g (extract_kernels.hip); false: the geometry does not take the
// dataflow launch (a level whose resize is not LDS-tiled)
// chain (optional): the few-launch pyramid's plan and its jobs (host copy); when given, the pyramid runs as chain-job
// tasks (a level's tiles straight from its segment's base level, so the levels of a segment need no wait on each
// other) instead of per-level resize tasks
bool build_flow(const Geom& g, int nframes, int blocks, const ChainPlan* chain, const std::vector<ChainJob>* jobs,
                std::vector<FlowTask>& tasks, FlowPlan& plan);

// The dataflow launch's arguments, read by the kernel from device memory (the caller uploads them when they change)
struct FlowArgs {
    const Geom* g;
    const ResizeCoef* rcoef;
    RcoefOff roff;
    const CellDesc* cells;
    const uint8_t* frames;
    long long framePitch;
    int rowStride;
    uint8_t* pyr;
    uint32_t* cands;
    uint32_t* candFirst;
    uint32_t* keys;
    uint16_t* knode;
    uint32_t* lvlKps;
    int* lvlCount;
    int* err;        // the host-visible overflow flags [2] (written once, by the workgroup finishing the last octree)
    int* errHost;    // host-coherent copy of them (orb_extract), or NULL
    orb_keypoint* outK;
    uint8_t* outD;
    int* outN;
    int kpCap;
    const FlowTask* tasks;
    int ntasks;
    int nframes;
    int* ctr;
    int ldsKeys;
    int rsQuarter;
    unsigned long long* stamps;   // ORBGPU_FLOW_STAMPS=1 (diagnostic): per task [ticket taken, wait over, done, id]
    const ChainJob* chainJobs;    // the chain plan's jobs (chain tasks), and its segments
    ChainSegment chainSeg[ORBGPU_MAX_LEVELS];
};

// Kernel launchers (extract_kernels.hip / hamming_kernels.hip / hamming_top2.hip).
struct ExtractBuffers {
    const Geom* d_geom;
    const ResizeCoef* d_rcoef;     // per level: w_l x-coefs then h_l y-coefs, at rcoef_off[l]
    const CellDesc* d_cells;       // ncells FAST cell descriptors
    int rcoef_off[ORBGPU_MAX_LEVELS];
    const ChainJob* d_chain;       // k_pyramid_chain jobs (chain.njobs per frame)
    ChainPlan chain;
    uint8_t* d_pyr;                // nframes * pyr_bytes
    uint32_t* d_cands;             // nframes * ncand: a cell's corners from the (kCandFirst+1)th on, at its slots
    uint32_t* d_candFirst;         // nframes * ncells * kCandRec: a cell's corner count and first corners (32 B per
                                   // cell: the octree reads most cells' corners with two coalesced loads)
    uint32_t* d_keys;              // nframes * nlevels * max_level_cand
    uint16_t* d_knode;             // same
    uint32_t* d_lvlKps;            // nframes * nkpcap
    int* d_lvlCount;               // nframes * nlevels
    int* d_err;                    // 2 ints: internal overflow flags (the level-0 branch of a forked launch sets [1])
    int* err_host;                 // host-coherent copy of it written by k_describe (the host path), or NULL
    int zero_err;                  // FAST zeroes d_err (0: the caller did)
    unsigned long long* d_stamps;  // phase timestamps (ORBGPU_FAST_STAMPS=1 diagnostic): 8 per (frame, cell),
                                   // 32 per (frame, level), 8 per keypoint slot
    // Forked launch (one frame in flight, the host path): level 0's FAST -> octree branch runs on fork_s2
    // beside the pyramid and levels 1.. on the launch stream, joined before k_describe (NULL: one stream)
    hipStream_t fork_s2;
    hipEvent_t ev_fork, ev_join;
    // the dataflow launch (NULL d_flow: the per-kernel launches); its plan matches this call's nframes
    const FlowTask* d_flow;
    int* d_flow_ctr;
    ChainPlan flow_chain;          // the plan the dataflow tasks were built with (nseg 0: per-level resize tasks)
    const FlowArgs* d_flow_args;   // this call's arguments (flow_args()), already in device memory
    unsigned long long* d_flow_stamps;   // ORBGPU_FLOW_STAMPS=1: 4 per task (diagnostic), else NULL
    FlowPlan flow;
};
FlowArgs flow_args(const ExtractBuffers& b, const uint8_t* d_frames, long long frame_pitch, int row_stride, int nframes,
                   orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int kp_cap);

typedef void (*KernelMarker)(void* user, int kernel_id, int begin, hipStream_t stream);

hipError_t launch_extract(const Geom& g, const ExtractBuffers& b, const uint8_t* d_frames, long long frame_pitch,
                          int row_stride, int nframes, orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                          int kp_cap, hipStream_t stream, KernelMarker marker, void* user);

// d_ranges: per query [begin, end) into d_cand_idx, or NULL = all trains.
hipError_t launch_hamming_topk(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, const int2* d_ranges,
                               const int* d_cand_idx, const int* d_thr, int k, int* d_dist, int* d_idx,
                               int* d_nvalid, hipStream_t stream);


// Batched all-pairs top-2 (k_top2_mfma, hamming_top2.hip): pair p = (query frame frames[p].x, train frame
// frames[p].y) of descriptor arrays q / t with q_stride / t_stride descriptors per frame; counts[frame] on the
// device, or nq / nt for every pair when counts == NULL (frames == NULL: one pair, frame 0).
struct Top2Batch {
    const uint8_t* q;
    const uint8_t* t;
    long long q_stride, t_stride;
    const int* counts;
    int nq, nt;
    const int2* frames;
    int slice;
    long long out_stride;   // outputs / partials of pair p at p * out_stride + query
    // set by launch_hamming_top2_batch: query blocks per pair and train slices per pair of the 1-D grid
    int qblocks, nslices;
};
int top2_batch_slices(int npairs, int max_nq, int max_nt);   // partial buffer: npairs * slices * out_stride uint2
int top2_launch_slices(int npairs, int max_nq, int max_nt);   // slices one launch uses (1 = direct write)
hipError_t launch_hamming_top2_batch(const Top2Batch& a, int npairs, int max_nq, int max_nt, int* d_best,
                                     int* d_best_idx, int* d_second, uint2* d_part, hipStream_t stream);

// Window candidates from the Frame grid (orb_window_match_grid): per item the query feature, its
// window centre and the grid geometry; ranks (dist, grid slot) like k_topk ranks (dist, list position).
struct WinGrid {
    float min_x, min_y, inv_w, inv_h, r;
};
hipError_t launch_window_topk(const uint8_t* d_q, const int* d_item_q, const float2* d_centre, int nitems,
                              const orb_keypoint* d_kps1, const uint8_t* d_t, const orb_keypoint* d_kps2,
                              const int* d_cell_off, const int* d_cell_idx, const WinGrid& wg, const int* d_thr,
                              int k, int* d_dist, int* d_idx, int* d_nvalid, hipStream_t stream);

// SearchForTriangulation's staged inputs, read by k_triangulation straight from the pinned mirror (over PCIe):
// one record per query (item) holding everything its wave needs, and the candidate trains' records in
// candidate order, so a wave's reads are two dependent round trips (its item record, then its candidates').
// Everything that depends on the keyframe pair rather than on a (query, candidate) pair is evaluated on the host
// while staging, with the reference build's float forms (tools/ref_flags_probe.cpp): the query's epipolar line
// (CheckDistEpipolarLine's a, b, c, ORBmatcher.cc:143-145) and the candidate's epipole test (:743-748) and
// sigma^2 (:156).  So one launch can serve several keyframe pairs (the batch call).
struct TriItem {          // 64 B
    uint4 desc[2];
    float la, lb, lc;     // a = x F00 + y F10 + F20, b = x F01 + y F11 + F21, c = x F02 + y F12 + F22 (contracted)
    int c0, c1;           // the item's candidates: train records [c0, c1)
    int stereo;           // mvuRight >= 0
    int pad[2];
};
struct TriTrain {         // 48 B
    uint4 desc[2];
    float x, y;           // KF2 keypoint
    float sigma2;         // pKF2->mvLevelSigma2[octave]
    int flags;            // bit 0: stereo (mvuRight >= 0); bit 1: inside the epipole radius (dex^2 + dey^2 < 100 scale)
};
static_assert(sizeof(TriItem) == 64 && sizeof(TriTrain) == 48, "k_triangulation's record layout");
// One work item per query with candidates; returns per item the best train record (or -1).
hipError_t launch_triangulation(const TriItem* d_items, const TriTrain* d_trains, int nitems, int* d_best,
                                hipStream_t stream);

// Frame::ComputeStereoMatches (stereo.hip).  One side of a rectified pair: its pyramid (level 0 in
// `frames`, levels >= 1 in `pyr`) and extraction outputs, for pair p at frame frame0 + p*frame_step.
struct StereoSide {
    const uint8_t* frames;
    long long frame_pitch;
    int row_stride;
    const uint8_t* pyr;
    int frame0, frame_step;
    const orb_keypoint* kps;   // pair p: kps + (frame0 + p*frame_step) * kp_stride
    const uint8_t* desc;       // same slots, 32 B each
    const int* counts;         // counts[frame]
    long long kp_stride;
};
size_t stereo_scratch_ints(const Geom& g, int npairs, long long out_stride);
hipError_t launch_stereo(const Geom* d_geom, const Geom& g, const StereoSide& L, const StereoSide& R, int npairs,
                         float mb, float mbf, float* d_uright, float* d_depth, int* d_scratch, long long out_stride,
                         int* d_nmatched, hipStream_t stream);

// glibc sinf/cosf (glibc_trig.h) over n angles, for the trig pin test (orb_debug_sincosf)
hipError_t launch_debug_sincosf(const float* d_x, int n, float* d_s, float* d_c, hipStream_t stream);
// The host path's streamed image upload (k_upload_stream): band b copied once h_flags[b] == seq.
hipError_t launch_upload_stream(const uint8_t* h_img, const uint32_t* h_flags, uint32_t seq, uint8_t* d_img, int pitch,
                                int h, int nbands, int band_rows, uint32_t* h_fail, hipStream_t stream);

// OpenCV 3.2 resize INTER_LINEAR coefficients for sw -> dw (orbgpu_abi.hip), appended to `out`
void resize_coefs(int sw, int dw, std::vector<ResizeCoef>& out, bool vertical);
size_t octree_lds_bytes(int node_cap);
void fast_wave_layout(Geom& g);   // fills fast_rows/drows/list/wave_bytes from the level grids
void build_cells(const Geom& g, std::vector<CellDesc>& cells);

}  // namespace orbgpu
