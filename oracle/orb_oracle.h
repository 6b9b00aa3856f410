/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of the reference ORB front-end of donglinb/ORB-SLAM-BIRDVIEW:
 *   src/ORBextractor.cc  (pyramid, per-cell FAST + fallback, DistributeOctTree, IC_Angle,
 *                         GaussianBlur + computeOrbDescriptor)
 *   src/ORBmatcher.cc    (DescriptorDistance, SearchByBoW x2, SearchForTriangulation,
 *                         SearchForInitialization / BirdviewMatch, ComputeThreeMaxima)
 * and of the OpenCV-3.2 primitives those files call (resize INTER_LINEAR, FAST 9/16 + NMS,
 * GaussianBlur 7x7 sigma 2, fastAtan2, cvRound) as pinned in SURVEY.md Appendix A.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * PARITY STATUS: pinned against every known-answer constant derivable from the reference
 * (umax table, features-per-level, pyramid sizes, pattern checksum, DescriptorDistance KATs,
 * ThreeMaxima edge cases, rotation-bin quirk).  The reference ships no tests, fixtures or golden
 * vectors, and cannot be built here (needs OpenCV, absent), so the OpenCV-primitive arithmetic
 * is "parity unpinned" beyond those constants.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bit-compatible with cv::KeyPoint (28 bytes). */
typedef struct {
    float x, y, size, angle, response;
    int octave, class_id;
} OracleKeyPoint;

/* flags */
#define ORACLE_TIE_REVERSE_SEQ   1  /* octree sort tie: later-created = SMALLER "pointer"   */
#define ORACLE_RESIZE_GENERIC    2  /* VResize uses generic FixedPtCast instead of 3.x >>4  */
#define ORACLE_BLUR_ALL_HALFUP   4  /* column pass rounds half-up everywhere (no SSE body)  */
#define ORACLE_NO_FMA            8  /* BRIEF offsets uncontracted (reference built without FMA) */
#define ORACLE_TRIG_CR          16  /* BRIEF cos/sin correctly rounded instead of glibc cosf/sinf */
#define ORACLE_TIE_LITERAL      32  /* DistributeOctTree as the reference runs it: std::list nodes,
                                       pair<int, node*> sort by heap address (glibc malloc, this process) */

void* oracle_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int flags);
void  oracle_destroy(void* h);
/* Runs ORBextractor::operator() (ORBextractor.cc:1043-1105). Returns #keypoints, or -1 if the
 * image is empty (outputs untouched, :1046-1047), -2 if the geometry is degenerate. */
int   oracle_run(void* h, const uint8_t* img, int w, int hgt, int stride);
int   oracle_level_size(void* h, int level, int* w, int* hgt);
int   oracle_get_level(void* h, int level, uint8_t* out);            /* pyramid ROI, w*h bytes */
int   oracle_get_blurred(void* h, int level, uint8_t* out);          /* 7x7 blurred level      */
/* FAST candidates in vToDistributeKeys order, coords relative to minBorder (ORBextractor.cc:820-825).
 * out: 3 ints per candidate (x, y, score). Returns count (or -count-1 if cap too small). */
int   oracle_get_candidates(void* h, int level, int* out, int cap);
/* Level keypoints after DistributeOctTree + border shift + IC angle (level coordinates). */
int   oracle_get_level_keypoints(void* h, int level, OracleKeyPoint* out, int cap);
int   oracle_get_output(void* h, OracleKeyPoint* kps, uint8_t* desc, int cap);
void  oracle_tables(void* h, float* scale, float* invScale, float* sigma2, float* invSigma2,
                    int* nPerLevel, int* umax16);

/* ---- primitives / known-answer helpers ---- */
float oracle_fast_atan2(float y, float x);
int   oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);
void  oracle_three_maxima(const int* histo_sizes, int L, int* ind1, int* ind2, int* ind3);
int   oracle_rot_bin(float angle1, float angle2);   /* the matchers' round(rot*(1/30)) bin */
int   oracle_fast_roi(const uint8_t* roi, int w, int h, int stride, int threshold, int* out, int cap);
void  oracle_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, int flags);
void  oracle_blur(const uint8_t* src, int w, int hgt, uint8_t* dst, int flags);
void  oracle_pattern(int* out1024);
/* glibc sinf/cosf as restated in glibc_sincosf.inc (ORBextractor.cc:113), n angles */
void  oracle_sincosf(const float* x, int n, float* s, float* c);

/* ---- CPU baseline timing: extract `nframes` frames (contiguous w*h each), round-robin over
 * `nthreads` threads (one frame per thread at a time), `iters` passes.  Returns wall seconds;
 * total_kps (optional) receives the keypoint total of one pass. ---- */
double oracle_time_extract(const uint8_t* frames, int nframes, int w, int h, int nfeatures,
                           float scaleFactor, int nlevels, int iniTh, int minTh,
                           int nthreads, int iters, long long* total_kps);

/* ---- CPU baseline protocol ---- */
/* single thread: `warmup` frames, then `timed` frames each timed (frame_ms[timed]); stage_ms6 = total ms of
 * the timed frames per stage: pyramid, FAST+NMS, octree, IC angle, blur, BRIEF */
int    oracle_bench_single(const uint8_t* frames, int nframes, int w, int h, int nfeatures, int warmup, int timed,
                           double* frame_ms, double* stage_ms6, long long* total_kps);
/* frame-parallel: nthreads extractors, `warmup` frames each off the clock, then `total` frames; seconds */
double oracle_bench_parallel(const uint8_t* frames, int nframes, int w, int h, int nfeatures, int nthreads, int warmup,
                             int total, long long* total_kps);
/* Hamming over frame pairs (desc/angles: `stride` slots per frame, counts per frame): mode 0 = SearchByBoW(KF,F)
 * with one node holding every feature, 1 = all-pairs top-2; seconds for `iters` passes, *evals = sum nq*nt */
double oracle_bench_hamming(const uint8_t* desc, const float* angles, const int* counts, int stride, int npairs,
                            const int* qf, const int* tf, int mode, int nthreads, int iters, long long* evals);

/* ---- matchers (ORBmatcher.cc). FeatureVector = CSR over ascending node ids. ---- */
typedef struct {
    int nnodes;
    const uint32_t* node_ids;   /* ascending */
    const int* offsets;         /* nnodes+1   */
    const int* indices;         /* feature indices per node, in FeatureVector order */
} OracleFeatVec;

/* SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)  ORBmatcher.cc:159-288
 * mp_kf[i] != 0  <=> KF feature i has a MapPoint that is not bad.
 * out match_f[iF] = KF feature index whose MapPoint was assigned, or -1. */
int oracle_search_by_bow_kf_f(float nnratio, int checkOri,
                              int n_kf, const uint8_t* desc_kf, const float* angle_kf,
                              const uint8_t* mp_kf, OracleFeatVec fv_kf,
                              int n_f, const uint8_t* desc_f, const float* angle_f,
                              OracleFeatVec fv_f, int* match_f);

/* SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)  ORBmatcher.cc:522-655
 * out match12[i1] = KF2 feature index whose MapPoint was assigned, or -1. */
int oracle_search_by_bow_kf_kf(float nnratio, int checkOri,
                               int n1, const uint8_t* desc1, const float* angle1,
                               const uint8_t* mp1, OracleFeatVec fv1,
                               int n2, const uint8_t* desc2, const float* angle2,
                               const uint8_t* mp2, OracleFeatVec fv2, int* match12);

/* SearchForTriangulation  ORBmatcher.cc:657-823 (+ CheckDistEpipolarLine :140-157).
 * has_mp[i] != 0 <=> GetMapPoint(i) non-NULL.  F12 row-major 3x3 float.
 * pairs_out: 2 ints per pair (idx1, idx2), ascending idx1. Returns #pairs. */
int oracle_search_for_triangulation(int checkOri, int onlyStereo,
                                    int n1, const uint8_t* desc1, const OracleKeyPoint* kps1,
                                    const uint8_t* has_mp1, const float* uright1, OracleFeatVec fv1,
                                    int n2, const uint8_t* desc2, const OracleKeyPoint* kps2,
                                    const uint8_t* has_mp2, const float* uright2, OracleFeatVec fv2,
                                    const float* F12, float ex, float ey,
                                    const float* scaleFactors2, const float* levelSigma2_2,
                                    int* pairs_out, int cap);

/* SearchForInitialization (ORBmatcher.cc:405-520) when level0_only=1;
 * BirdviewMatch(const Frame&, const Frame&, ...) (:1790-1899) when level0_only=0.
 * cand_off/cand_idx: Frame::GetFeaturesInArea result per query (CSR).
 * match12 out (-1 = none). Returns nmatches. */
int oracle_window_match(float nnratio, int checkOri, int level0_only,
                        int n1, const uint8_t* desc1, const OracleKeyPoint* kps1,
                        int n2, const uint8_t* desc2, const OracleKeyPoint* kps2,
                        const int* cand_off, const int* cand_idx, int* match12);

/* Frame::GetFeaturesInArea (Frame.cc:494-547) over the Frame grid (Frame.cc:378-412, 549-560).
 * Returns #indices written (or -needed-1 if cap too small). */
int oracle_features_in_area(int n, const OracleKeyPoint* kpsUn,
                            float minX, float maxX, float minY, float maxY,
                            float x, float y, float r, int minLevel, int maxLevel,
                            int* out, int cap);

/* Frame::ComputeStereoMatches (Frame.cc:662-836) on the pyramids of two oracle extractors that ran on
 * the rectified left / right images.  Writes mvuRight / mvDepth (N each, -1 = no match); returns the
 * number of left keypoints with a depth. */
int oracle_stereo_matches(void* left, void* right, int N, const OracleKeyPoint* kpsL, const uint8_t* descL, int Nr,
                          const OracleKeyPoint* kpsR, const uint8_t* descR, float mb, float mbf, float* mvuRight,
                          float* mvDepth);

/* DBoW2 vocabulary (TemplatedVocabulary.h): binary loader (:1466-1510), per-feature descent
 * (:1240-1277) and the BowVector / FeatureVector transform (:1139-1210).  NULL on a bad file. */
void* oracle_vocab_load(const char* path);
void  oracle_vocab_destroy(void* h);
int   oracle_vocab_info(void* h, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords);
void  oracle_vocab_transform_each(void* h, const uint8_t* desc, int n, int levelsup, int* word_id, double* weight,
                                  uint32_t* nid);
int   oracle_vocab_transform(void* h, const uint8_t* desc, int n, int levelsup, int* bow_words, double* bow_values,
                             int* nbow, uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* nfv);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307): index of the chosen descriptor of N. */
int oracle_distinctive_descriptor(const uint8_t* desc, int N);

/* ---- Birdview stream (Frame.cc:318-342): OpenCV 3.2 cv::ORB(HARRIS) detect/compute + cornerSubPix,
 * restated in cvorb_oracle.inc.  PARITY UNPINNED (OpenCV absent, no reference fixture). ---- */
void* oracle_cvorb_create(int nfeatures, float scaleFactor, int nlevels, int edgeThreshold, int fastThreshold);
void  oracle_cvorb_destroy(void* h);
/* OpenCV arithmetic variant of the cv::ORB pyramid resize and descriptor blur (ORACLE_RESIZE_GENERIC,
 * ORACLE_BLUR_ALL_HALFUP; other bits ignored) */
void  oracle_cvorb_set_flags(void* h, int flags);
/* cv::ORB::detect(img, kps, mask); mask may be NULL.  Returns n (or -n-1 if cap too small). */
int   oracle_cvorb_detect(void* h, const uint8_t* img, int w, int hgt, int stride, const uint8_t* mask, int mstride,
                          OracleKeyPoint* out, int cap);
/* last detect(): level-l FAST candidates after the mask and border filters, raster order, Harris response */
int   oracle_cvorb_candidates(void* h, int level, OracleKeyPoint* out, int cap);
int   oracle_cvorb_level(void* h, int level, uint8_t* out, int* w, int* hgt);
/* cv::ORB::compute(img, kps, desc): kps in/out (border-culled, level-sorted); returns the new n */
int   oracle_cvorb_compute(void* h, const uint8_t* img, int w, int hgt, int stride, OracleKeyPoint* kps, int n,
                           uint8_t* desc);
/* cv::cornerSubPix(img, pts(2n floats, in/out), Size(winW,winH), Size(-1,-1), EPS|ITER(maxIter, eps)) */
void  oracle_corner_subpix(const uint8_t* img, int w, int hgt, int stride, float* pts, int n, int winW, int winH,
                           int maxIter, double eps);
void  oracle_bird_footprint_mask(uint8_t* mask, int w, int hgt, int stride);   /* Frame.cc:320-327 */
/* Frame.cc:320-342 end to end (mask gets the footprint applied to a copy; NULL = no mask) */
int   oracle_bird_extract(void* h, const uint8_t* img, int w, int hgt, int stride, const uint8_t* mask, int mstride,
                          OracleKeyPoint* out, int cap, uint8_t* desc);

#ifdef __cplusplus
}
#endif
#endif
