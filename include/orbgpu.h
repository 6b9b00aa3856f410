/*
 * orbgpu.h — C-ABI of the MI355X-native ORB front-end (gfx950 HIP kernels).
 *
 * Drop-in boundary for the ORB front-end of donglinb/ORB-SLAM-BIRDVIEW.  Each entry point names the
 * reference interface it replaces; the C++ mirror classes ORB_SLAM2::ORBextractor / ORBmatcher
 * (orb-slam-birdview_amd/csrc/host/) and the Python binding (orbgpu/) are thin layers over it.
 *
 *  - Plain pointers and sizes only: no HIP, torch or OpenCV types in any signature.
 *  - Nothing throws across the ABI; every function returns an orb_status (0 = OK).
 *  - A context owns one HIP stream on one device; entry points call hipSetDevice on entry, so a
 *    context may be driven from any host thread (Frame.cc:124-127 spawns fresh threads per frame),
 *    but one context must not be used by two threads at once (same contract as the reference's
 *    one-extractor-per-thread, ORBextractor.h:85 mvImagePyramid is instance state).
 *  - There is no CPU fallback: if the HIP runtime or device is unavailable, orb_create fails.
 */
#ifndef ORBGPU_H
#define ORBGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBGPU_ABI_VERSION 2
#define ORBGPU_MAX_LEVELS 16

/* OpenCV arithmetic variant (orb_params.variant / orb_bird_params.variant, bit flags).  The reference
 * links whichever OpenCV 2.4.3-3.4 the build machine has (CMakeLists.txt:31-37) and calls its resize
 * (ORBextractor.cc:1120) and GaussianBlur (:1085-1086); those versions differ in the last bits, and the
 * octree sort (:684) breaks size ties by heap address.  0 is the pinned default (OpenCV 3.2 x86-64 SSE2
 * without IPP; ties by node creation sequence; BRIEF offsets contracted to FMA as GCC -march=native
 * builds them).  The bit values equal the oracle's ORACLE_* flags (oracle/orb_oracle.h). */
#define ORB_VARIANT_DEFAULT        0
#define ORB_VARIANT_TIE_REVERSE    1  /* :684 tie: a later-created node counts as the SMALLER pointer      */
#define ORB_VARIANT_RESIZE_GENERIC 2  /* resize vertical pass = generic FixedPtCast (b0*H0+b1*H1+2^21)>>22 */
#define ORB_VARIANT_BLUR_HALFUP    4  /* GaussianBlur column pass rounds half-up everywhere (no SSE2 body) */
#define ORB_VARIANT_NO_FMA         8  /* BRIEF sample offsets (:119-120) uncontracted (no -march=native FMA) */
#define ORB_VARIANT_MASK          15

typedef enum {
    ORB_OK = 0,
    ORB_ERR_ARG = -1,        /* bad argument / NULL pointer                                     */
    ORB_ERR_HIP = -2,        /* HIP runtime error (message via orb_last_error)                   */
    ORB_ERR_CAPACITY = -3,   /* caller buffer too small; *n receives the required count          */
    ORB_ERR_GEOMETRY = -4,   /* image too small for the pyramid (reference: division by zero UB), a side
                                above 4096 pixels (candidates pack 12-bit coordinates), or a level whose
                                octree node tables exceed one CU's LDS (N per level above ~2,550, i.e.
                                nfeatures above ~11,700 at scale 1.2 / 8 levels) */
    ORB_ERR_NOMEM = -5,      /* device allocation failed                                         */
    ORB_ERR_INTERNAL = -6    /* a kernel reported an overflow of an internal bound               */
} orb_status;

/* Bit-compatible with cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id;}
 * (28 bytes), so the OpenCV-side adapter can memcpy. */
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} orb_keypoint;

/* ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * replaces ORBextractor::ORBextractor, reference src/ORBextractor.cc:410-470 / include/ORBextractor.h:52-53 */
typedef struct {
    int nfeatures;
    float scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;
    int device;       /* HIP device ordinal                                     */
    int max_width;    /* capacity hints (contexts grow on demand for host input) */
    int max_height;
    int max_batch;    /* frames per batched launch (device-resident path)       */
    int variant;      /* ORB_VARIANT_* bits (0 = pinned default); unknown bits: ORB_ERR_ARG */
} orb_params;

typedef struct orb_ctx orb_ctx;

int  orb_abi_version(void);
const char* orb_last_error(void);      /* thread-local message for the last failure */
int  orb_device_count(void);

orb_ctx* orb_create(const orb_params* p, int* status);
void     orb_destroy(orb_ctx* ctx);

/* GetLevels/GetScaleFactor(s)/GetInverseScaleFactors/GetScaleSigmaSquares/GetInverseScaleSigmaSquares
 * (include/ORBextractor.h:63-83) + mnFeaturesPerLevel (ORBextractor.cc:435-446) + umax (:454-469).
 * Any pointer may be NULL. Arrays hold nlevels entries (umax: 16). */
int orb_scale_tables(const orb_ctx* ctx, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2,
                     int* n_per_level, int* umax16);

/* ORBextractor::operator()(InputArray image, InputArray mask, vector<KeyPoint>&, OutputArray)
 * — reference src/ORBextractor.cc:1043-1105.  Host gray image in (mask ignored, as in the reference,
 * include/ORBextractor.h:58); keypoints (level-0 coordinates, level-major order) and n x 32
 * descriptors out.  Empty image (w==0 || h==0 || img==NULL) returns ORB_OK leaving *n and the
 * outputs untouched (:1046-1047).  If *n would exceed cap, returns ORB_ERR_CAPACITY with *n set. */
int orb_extract(orb_ctx* ctx, const uint8_t* img, int w, int h, size_t stride,
                orb_keypoint* kps, int cap, int* n, uint8_t* desc);

/* public std::vector<cv::Mat> mvImagePyramid (include/ORBextractor.h:85), read by
 * Frame::ComputeStereoMatches (Frame.cc:669,759): host view of level `level` of the last
 * orb_extract, copied lazily device->host into context-owned memory (valid until the next call). */
int orb_get_level(orb_ctx* ctx, int level, const uint8_t** data, int* w, int* h, size_t* stride);

/* ---- device-resident batched path (bench, multi-camera streams). Asynchronous on the context
 * stream; call orb_sync before reading outputs. d_frames: nframes gray frames, frame f at
 * d_frames + f*frame_pitch, rows `row_stride` apart (w <= row_stride < 16 MiB).  Outputs: frame f's keypoints at
 * d_kps + f*kp_cap, descriptors at d_desc + f*kp_cap*32, count in d_counts[f].
 * kp_cap must be >= orb_batch_kp_cap(ctx, w, h). ---- */
int orb_batch_kp_cap(orb_ctx* ctx, int w, int h);
int orb_extract_batch_device(orb_ctx* ctx, const uint8_t* d_frames, int nframes, int w, int h,
                             size_t frame_pitch, size_t row_stride,
                             orb_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int kp_cap);
int orb_sync(orb_ctx* ctx);

/* device memory helpers (so callers need no HIP headers) */
void* orb_device_alloc(orb_ctx* ctx, size_t bytes);
int   orb_device_free(orb_ctx* ctx, void* p);
int   orb_memcpy_h2d(orb_ctx* ctx, void* dst, const void* src, size_t bytes);
int   orb_memcpy_d2h(orb_ctx* ctx, void* dst, const void* src, size_t bytes);
int   orb_memset_device(orb_ctx* ctx, void* dst, int value, size_t bytes);

/* ---- per-kernel timing with HIP events on the context stream (bench roofline) ---- */
enum { ORB_K_RESIZE = 0, ORB_K_FAST = 1, ORB_K_OCTREE = 2, ORB_K_DESCRIBE = 3, ORB_K_HAMMING = 4,
       ORB_K_STEREO = 5, ORB_K_FLOW = 6 /* the small-batch dataflow launch: every stage in one kernel */,
       ORB_K_COUNT = 7 };
int orb_profile_enable(orb_ctx* ctx, int on);   /* clears accumulated times */
int orb_profile_read(orb_ctx* ctx, double* ms_total /*ORB_K_COUNT*/, int* launches /*ORB_K_COUNT*/);

/* ---- debug views of intermediate device buffers (parity tests pinpoint the failing stage) ---- */
/* FAST candidates of `level` for frame `frame` of the last batch, in vToDistributeKeys order
 * (ORBextractor.cc:820-825): 3 ints (x, y, score) each, coords relative to minBorder. */
int orb_debug_candidates(orb_ctx* ctx, int frame, int level, int* out, int cap);
/* Octree output of `level` (DistributeOctTree list order): 3 ints (x, y, score), level coords. */
int orb_debug_level_keypoints(orb_ctx* ctx, int frame, int level, int* out, int cap);
int orb_debug_level_image(orb_ctx* ctx, int frame, int level, uint8_t* out, int* w, int* h);
/* Phase timestamps of the last FAST launch (diagnostic; only with ORBGPU_FAST_STAMPS=1 in the
 * environment at orb_create): 8 s_memtime values per (frame, cell) item.  With ORBGPU_FLOW_STAMPS=1 instead,
 * the last dataflow launch's: 4 values per task in ticket order (100 MHz s_memrealtime when its ticket was
 * taken, when its wait ended, when it was done; then kind | level << 8 | frame << 16 | workgroup << 32).
 * Returns the count copied. */
int orb_debug_fast_stamps(orb_ctx* ctx, uint64_t* out, int cap);
/* The BRIEF rotation's sin/cos as the kernels compute them (glibc sinf/cosf restated, ORBextractor.cc:113)
 * for n host angles (radians, 0 <= x < 120): s[i] = sinf(x[i]), c[i] = cosf(x[i]).  Pin test only. */
int orb_debug_sincosf(orb_ctx* ctx, const float* x, int n, float* s, float* c);

/* =========================== Birdview stream (Frame.cc:318-342) ===========================
 * The reference runs OpenCV's cv::ORB (HARRIS_SCORE, not ORBextractor) plus cv::cornerSubPix on the
 * birdview image.  orb_bird mirrors cv::ORB::create(nfeatures, scaleFactor, nlevels, edgeThreshold,
 * firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31, fastThreshold) — Frame.cc:329 uses
 * ORB::create(2000): {2000, 1.2f, 8, 31, 20}.  One HIP stream per object; one host thread at a time. */
typedef struct {
    int nfeatures;
    float scaleFactor;
    int nlevels;
    int edgeThreshold;
    int fastThreshold;
    int device;
    int variant;      /* ORB_VARIANT_RESIZE_GENERIC | ORB_VARIANT_BLUR_HALFUP apply (cv::ORB's own pyramid
                         resize and descriptor blur, orb.cpp); other bits: ORB_ERR_ARG */
} orb_bird_params;

typedef struct orb_bird orb_bird;

orb_bird* orb_bird_create(const orb_bird_params* p, int* status);
void      orb_bird_destroy(orb_bird* b);

/* cv::ORB::detect(image, keypoints, mask) — Frame.cc:330 (OpenCV 3.2 ORB_Impl::detectAndCompute,
 * computeKeyPoints).  mask may be NULL (no mask).  Keypoints in level-0 coordinates, reference order.
 * Empty image: *n = 0.  cap too small: ORB_ERR_CAPACITY with *n set. */
int orb_bird_detect(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, const uint8_t* mask,
                    size_t mask_stride, orb_keypoint* kps, int cap, int* n);
/* cv::ORB::compute(image, keypoints, descriptors) — Frame.cc:342.  kps in/out: border-culled
 * (runByImageBorder, edgeThreshold) and level-sorted in place, *n updated; desc receives *n x 32. */
int orb_bird_compute(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, orb_keypoint* kps, int* n,
                     uint8_t* desc);
/* cv::cornerSubPix(image, pts (n x float2, in/out), Size(win_w, win_h), Size(-1,-1),
 * TermCriteria(EPS+MAX_ITER, max_iter, eps)) — Frame.cc:336-337.  Only Size(5,5) is built. */
int orb_corner_subpix(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, float* pts, int n, int win_w,
                      int win_h, int max_iter, double eps);
/* Frame.cc:320-342 fused: footprint-masked detect, cornerSubPix(5x5, 40, 0.001), compute — one upload,
 * one pyramid.  mask (birdviewMask) is not modified: the footprint is zeroed in the device copy. */
int orb_bird_extract(orb_bird* b, const uint8_t* img, int w, int h, size_t stride, const uint8_t* mask,
                     size_t mask_stride, orb_keypoint* kps, int cap, int* n, uint8_t* desc);
/* Same, image and mask already in device memory (bench / multi-stream callers). */
int orb_bird_extract_device(orb_bird* b, const uint8_t* d_img, int w, int h, size_t stride, const uint8_t* d_mask,
                            size_t mask_stride, orb_keypoint* kps, int cap, int* n, uint8_t* desc);
/* Frame.cc:320-327: zero the vehicle footprint (+15 px boundary) of a birdview mask in place (host). */
int orb_bird_footprint_mask(uint8_t* mask, int w, int h, size_t stride);
/* debug: last detect's level-l candidates after mask / border / NMS, raster order, level coordinates;
 * response = Harris response, class_id = FAST score.  Returns the count (or -count-1 if cap is too small). */
int orb_bird_debug_candidates(orb_bird* b, int level, orb_keypoint* out, int cap);
int orb_bird_debug_level(orb_bird* b, int level, uint8_t* out, int* w, int* h);

/* =========================== ORBmatcher =========================== */

/* static int ORBmatcher::DescriptorDistance(const cv::Mat&, const cv::Mat&)  ORBmatcher.cc:1647-1663
 * (host helper: a single pair is never worth a kernel launch). */
int orb_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* Top-k smallest Hamming distances per query on the GPU (the inner loop of every ORBmatcher search).
 * Candidates of query i: cand_idx[cand_off[i] .. cand_off[i+1]) (CSR, in the reference's iteration
 * order), or all trains 0..nt-1 if cand_off == NULL.  A candidate t is skipped when
 * train_thr != NULL and train_thr[t] <= dist (covers vbMatched2 / vMatchedDistance / invalid
 * MapPoints).  Results sorted by (dist, candidate position): out_dist/out_idx[i*k + j], -1 padded;
 * out_nvalid[i] = number of candidates that passed the filter (tells whether the list is complete).
 * Host pointers, synchronous. */
int orb_hamming_topk(orb_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt,
                     const int* cand_off, const int* cand_idx, const int* train_thr, int k,
                     int* out_dist, int* out_idx, int* out_nvalid);

/* Device-pointer variant of the all-pairs (cand_off == NULL, no filter) top-2: best distance,
 * its train index (first on ties) and second-best distance per query. Asynchronous. */
int orb_hamming_top2_device(orb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                            int* d_best, int* d_best_idx, int* d_second);

/* Batched device form over the descriptor slots of an extraction batch (orb_extract_batch_device's
 * d_desc / d_counts / kp_cap): pair p matches the descriptors of frame q_frames[p] against those of
 * frame t_frames[p] (host arrays), all pairs in one launch, counts read on the device.  Outputs at
 * d_best / d_best_idx / d_second[p * kp_cap + i].  kp_cap <= 65535.  Asynchronous.  This is the
 * brute-force SearchByBoW inner loop of BASELINE config C4 (one vocabulary node holding everything). */
int orb_hamming_top2_frames_device(orb_ctx* ctx, const uint8_t* d_desc, const int* d_counts, int kp_cap, int npairs,
                                   const int* q_frames, const int* t_frames, int* d_best, int* d_best_idx,
                                   int* d_second);

/* Train slices one top-2 launch splits each pair into for these sizes (orb_hamming_top2_device passes
 * npairs = 1; the frames form passes kp_cap for both maxima).  1 = the MFMA kernel writes best / index /
 * second itself; more = per-slice partial results merged by a second kernel.  Host only (test / tuning). */
int orb_hamming_top2_slices(int npairs, int max_nq, int max_nt);

/* Operand width of the all-pairs top-2's matrix-core form: 4 = +-4 e2m1 fp4 (v_mfma_scale_f32_32x32x64_f8f6f4,
 * bound by the dense FP4 peak; the only form since round 5).  Host only (bench / tests). */
int orb_hamming_top2_mfma_bits(void);

/* DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>, FeatureVector.h:21) as CSR.  The three
 * FeatureVector matchers below return ORB_ERR_ARG (before any GPU work) for a CSR whose offsets do not start at
 * 0 or decrease, whose indices leave [0, n) of their side, or whose node ids do not ascend strictly. */
typedef struct {
    int nnodes;
    const uint32_t* node_ids;   /* ascending */
    const int* offsets;         /* nnodes + 1 */
    const int* indices;
} orb_featvec;

/* int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
 * ORBmatcher.cc:159-288.  mp_kf[i]!=0 <=> KF feature i has a non-bad MapPoint; angles are
 * mvKeysUn (KF) / mvKeys (F) angles.  match_f[iF] = KF feature index whose MapPoint was assigned
 * to F feature iF, or -1.  *nmatches receives the return value of the reference function. */
int orb_search_by_bow_kf_f(orb_ctx* ctx, float nnratio, int check_ori,
                           int n_kf, const uint8_t* desc_kf, const float* angle_kf, const uint8_t* mp_kf,
                           orb_featvec fv_kf, int n_f, const uint8_t* desc_f, const float* angle_f,
                           orb_featvec fv_f, int* match_f, int* nmatches);

/* int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
 * ORBmatcher.cc:522-655.  match12[i1] = KF2 feature index whose MapPoint was assigned, or -1. */
int orb_search_by_bow_kf_kf(orb_ctx* ctx, float nnratio, int check_ori,
                            int n1, const uint8_t* desc1, const float* angle1, const uint8_t* mp1,
                            orb_featvec fv1, int n2, const uint8_t* desc2, const float* angle2,
                            const uint8_t* mp2, orb_featvec fv2, int* match12, int* nmatches);

/* The BoW searches over several keyframes in one call (one staging, one ranking launch, then each keyframe's
 * replay in the reference's order): the loops of Tracking::Relocalization (Tracking.cc:1931-1938,
 * SearchByBoW(pKF, mCurrentFrame, ...) per candidate keyframe) and LoopClosing::ComputeSim3 (LoopClosing.cc:252-265,
 * SearchByBoW(mpCurrentKF, pKF, ...) per loop candidate), whose iterations are independent.  Entry p's outputs are
 * exactly the single call's for the same inputs.
 *   orb_search_by_bow_kf_f_batch:  KF = kfs[p] (n, desc, angle, mp = its map-point flags, fv) against one Frame;
 *                                  match = match_f (n_f ints), *nmatches = the return value.
 *   orb_search_by_bow_kf_kf_batch: KF1 against KF2 = kf2s[p] (mp = KF2's map-point flags); match = match12 (n1 ints).
 * ORB_ERR_ARG for a malformed entry (nothing runs). */
typedef struct orb_bow_kf {
    int n;
    const uint8_t* desc;
    const float* angle;
    const uint8_t* mp;
    orb_featvec fv;
    int* match;
    int* nmatches;
} orb_bow_kf;
int orb_search_by_bow_kf_f_batch(orb_ctx* ctx, float nnratio, int check_ori, int n_f, const uint8_t* desc_f,
                                 const float* angle_f, orb_featvec fv_f, int nkf, const orb_bow_kf* kfs);
int orb_search_by_bow_kf_kf_batch(orb_ctx* ctx, float nnratio, int check_ori, int n1, const uint8_t* desc1,
                                  const float* angle1, const uint8_t* mp1, orb_featvec fv1, int nkf,
                                  const orb_bow_kf* kf2s);

/* int ORBmatcher::SearchForTriangulation(KeyFrame*, KeyFrame*, cv::Mat F12,
 *     vector<pair<size_t,size_t>>&, const bool bOnlyStereo)   ORBmatcher.cc:657-823
 * Keypoints are mvKeysUn; has_mp[i] <=> GetMapPoint(i) != NULL; uright = mvuRight; F12 row-major
 * 3x3; (ex, ey) the epipole of KF1's centre in KF2 (:662-668, computed by the caller from poses);
 * scale2/sigma2_2 = pKF2->mvScaleFactors / mvLevelSigma2.  pairs_out: 2 ints per pair (ascending
 * idx1), *npairs = count (ORB_ERR_CAPACITY if > cap).  ORB_ERR_ARG for a malformed FeatureVector CSR (see
 * orb_featvec; the call stages at most offsets[nnodes] records per side). */
int orb_search_for_triangulation(orb_ctx* ctx, int check_ori, int only_stereo,
                                 int n1, const uint8_t* desc1, const orb_keypoint* kps1, const uint8_t* has_mp1,
                                 const float* uright1, orb_featvec fv1,
                                 int n2, const uint8_t* desc2, const orb_keypoint* kps2, const uint8_t* has_mp2,
                                 const float* uright2, orb_featvec fv2,
                                 const float* F12, float ex, float ey, const float* scale2, const float* sigma2_2,
                                 int nlevels2, int* pairs_out, int cap, int* npairs);

/* SearchForTriangulation of one keyframe (KF1) against several (KF2s) in one call: LocalMapping::CreateNewMapPoints
 * (LocalMapping.cc:247-278) calls SearchForTriangulation(mpCurrentKeyFrame, pKF2, F12, ..., false) once per
 * neighbour keyframe.  pairs[p] carries what the single call takes for KF2 = pair p (its outputs included);
 * the result for pair p is exactly orb_search_for_triangulation's for the same inputs, all pairs sharing one
 * staging, one launch and one synchronisation.  The reference loop adds map points to KF1 between neighbours
 * (:449), and SearchForTriangulation skips KF1 features that have one (:694-696); with check_ori = 0 (the
 * LocalMapping call) every query is decided independently, so a caller that drops, while it walks the pairs in
 * order, the matches of pair p whose idx1 received a map point from pairs < p gets the sequential result exactly.
 * ORB_ERR_ARG for a malformed pair (nothing runs); ORB_ERR_CAPACITY if any pair's list overflowed (every pair's
 * *npairs holds its full count, the lists are filled up to cap). */
typedef struct orb_tri_pair {
    int n2;
    const uint8_t* desc2;
    const orb_keypoint* kps2;
    const uint8_t* has_mp2;
    const float* uright2;
    orb_featvec fv2;
    const float* F12;            /* row-major 3x3 */
    float ex, ey;                /* KF1's centre projected in KF2 */
    const float* scale2;         /* pKF2->mvScaleFactors */
    const float* sigma2_2;       /* pKF2->mvLevelSigma2 */
    int nlevels2;
    int* pairs_out;              /* 2 ints per pair */
    int cap;
    int* npairs;
} orb_tri_pair;
int orb_search_for_triangulation_batch(orb_ctx* ctx, int check_ori, int only_stereo,
                                       int n1, const uint8_t* desc1, const orb_keypoint* kps1, const uint8_t* has_mp1,
                                       const float* uright1, orb_featvec fv1, int npairs, const orb_tri_pair* pairs);

/* int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<Point2f>& vbPrevMatched,
 *     vector<int>& vnMatches12, int windowSize)  ORBmatcher.cc:405-520 (level0_only = 1), and
 * int ORBmatcher::BirdviewMatch(const Frame&, const Frame&, vector<int>&, int)  :1790-1899
 * (level0_only = 0).  Candidates per query = Frame::GetFeaturesInArea (CSR), computed by the caller
 * (orb_features_in_area restates it).  match12 out. */
int orb_window_match(orb_ctx* ctx, float nnratio, int check_ori, int level0_only,
                     int n1, const uint8_t* desc1, const orb_keypoint* kps1,
                     int n2, const uint8_t* desc2, const orb_keypoint* kps2,
                     const int* cand_off, const int* cand_idx, int* match12, int* nmatches);

/* The Frame grid as the reference holds it (Frame.h:211 mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS], filled by
 * Frame::AssignFeaturesToGrid, Frame.cc:378-413) flattened column-major: the keypoints of cell (ix, iy)
 * are cell_idx[cell_off[ix * 48 + iy] .. cell_off[ix * 48 + iy + 1]) in the cell vector's order; the cell
 * arithmetic of Frame::GetFeaturesInArea (:494-547) uses min_x / min_y and the inverse cell sizes.  The
 * birdview grid (GetFeaturesInAreaBirdview, :891-945) is the same with min_x = min_y = 0. */
typedef struct orb_frame_grid {
    float min_x, min_y;          /* mnMinX, mnMinY */
    float inv_w, inv_h;          /* mfGridElementWidthInv, mfGridElementHeightInv */
    const int* cell_off;         /* 64 * 48 + 1 */
    const int* cell_idx;         /* cell_off[64 * 48] entries */
} orb_frame_grid;

/* The window searches with the candidate lists computed on the GPU from F2's grid: the same matches
 * as orb_window_match with cand = GetFeaturesInArea(centre, window, octave1, octave1) per query.
 * centres: n1 (x, y) pairs (SearchForInitialization's vbPrevMatched, BirdviewMatch's vPrevMatched), or
 * NULL = each query's own keypoint position (BirdviewMatch(const Frame&, const Frame&, ...), :1803-1808).
 * level0_only: queries with octave > 0 are skipped (:420-423, :1683-1685).  match12 out. */
int orb_window_match_grid(orb_ctx* ctx, float nnratio, int check_ori, int level0_only,
                          int n1, const uint8_t* desc1, const orb_keypoint* kps1, const float* centres,
                          float window, int n2, const uint8_t* desc2, const orb_keypoint* kps2,
                          orb_frame_grid grid2, int* match12, int* nmatches);

/* Frame::GetFeaturesInArea over the 64x48 Frame grid (Frame.cc:378-412, 494-560): host helper the
 * C++ mirror uses to build window candidate lists. Returns count or -(needed)-1. */
int orb_features_in_area(int n, const orb_keypoint* kps_un, float min_x, float max_x, float min_y, float max_y,
                         float x, float y, float r, int min_level, int max_level, int* out, int cap);

/* ======================= Frame::ComputeStereoMatches ======================= */

/* void Frame::ComputeStereoMatches()  Frame.cc:662-836, for one rectified pair.  `left` / `right` are
 * the contexts that extracted the left / right image last (orb_extract; the reference's
 * mpORBextractorLeft/Right, whose mvImagePyramid the window search reads), same image size.  They may sit
 * on different GPUs (one GPU per camera stream): the right image and pyramid are then copied to the left
 * device with hipMemcpyPeerAsync and the search runs there.  kpsL/descL = mvKeys/mDescriptors (nL),
 * kpsR/descR = mvKeysRight/mDescriptorsRight (nR);
 * mb = baseline, mbf = baseline * fx.  uright / depth (nL each) receive mvuRight / mvDepth
 * (-1 = no match); *nmatched = number of left keypoints with a depth.  Synchronous. */
int orb_compute_stereo_matches(orb_ctx* left, orb_ctx* right, int nL, const orb_keypoint* kpsL, const uint8_t* descL,
                               int nR, const orb_keypoint* kpsR, const uint8_t* descR, float mb, float mbf,
                               float* uright, float* depth, int* nmatched);

/* Device-resident batched form: frames (2p, 2p+1) of the last orb_extract_batch_device on ctx are
 * the (left, right) images of pair p.  Outputs at d_uright/d_depth[p * kp_cap + i] (kp_cap of that
 * batch) and d_nmatched[p].  Asynchronous on the context stream. */
int orb_stereo_batch_device(orb_ctx* ctx, int npairs, float mb, float mbf, float* d_uright, float* d_depth,
                            int* d_nmatched);

/* ======================= DBoW2 vocabulary transform ======================= */

typedef struct orb_vocab orb_vocab;

/* TemplatedVocabulary::loadFromBinaryFile (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1466-1510)
 * of an ORB vocabulary (ORBvoc.bin format: header nb_nodes, size_node = 41, k, L, scoring,
 * weighting; records parent:int32 | desc[32] | weight:float | isLeaf:u8), onto ctx's device. */
int  orb_vocab_load(orb_ctx* ctx, const char* path, orb_vocab** out);
void orb_vocab_destroy(orb_vocab* v);
int  orb_vocab_info(const orb_vocab* v, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords);

/* Per-feature part of TemplatedVocabulary::transform (:1240-1277): word id, word weight and the node
 * `levelsup` levels above the leaf (FeatureVector key) of each of n descriptors, on the GPU.  Host
 * pointers, synchronous. */
int orb_vocab_transform(orb_ctx* ctx, const orb_vocab* v, const uint8_t* desc, int n, int levelsup, int* word_id,
                        float* weight, uint32_t* node_id);

/* Same for frames 0..nframes-1 of the last orb_extract_batch_device on ctx: outputs at
 * [f * kp_cap + i] (device pointers), counts from that batch.  Asynchronous. */
int orb_vocab_transform_batch_device(orb_ctx* ctx, const orb_vocab* v, int nframes, int levelsup, int* d_word,
                                     float* d_weight, uint32_t* d_node);

/* Host assembly of TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
 * (:1139-1210) from the per-feature triples, in feature order: BowVector as nbow (word, value)
 * pairs ascending by word; FeatureVector as nfv nodes ascending with CSR fv_off (nfv+1) / fv_idx.
 * Every output array needs room for n entries (fv_off n+1). */
int orb_vocab_bow(const orb_vocab* v, int n, const int* word_id, const float* weight, const uint32_t* node_id,
                  int* bow_words, double* bow_values, int* nbow, uint32_t* fv_nodes, int* fv_off, int* fv_idx,
                  int* nfv);

/* ============ MapPoint::ComputeDistinctiveDescriptors, batched ============ */

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:242-307; MapPointBird.cc:87-152): for each
 * of nmp map points, the descriptors of its observations from non-bad keyframes (observation order)
 * are desc[offsets[m] .. offsets[m+1]) (32 B each); best_idx[m] receives the index (within the point's
 * list) of the descriptor with the least median distance to the others — first on ties — or -1 for
 * an empty list (the reference returns without touching mDescriptor).  Host pointers, synchronous. */
int orb_distinctive_descriptors(orb_ctx* ctx, int nmp, const int* offsets, const uint8_t* desc, int* best_idx);

#ifdef __cplusplus
}
#endif
#endif
