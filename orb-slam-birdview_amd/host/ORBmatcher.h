/*
 * ORB_SLAM2::ORBmatcher — C++ mirror of the reference's descriptor matchers
 * (include/ORBmatcher.h:37-119, src/ORBmatcher.cc) over liborbgpu's C-ABI.
 *
 * The reference methods take Frame& / KeyFrame* and read a handful of their members; the mirror
 * takes a FeatureSet naming exactly those members (INTEGRATION.md shows the two-line adapter from a
 * Frame / KeyFrame).  Results keep the reference's meaning, with MapPoint* replaced by the index of
 * the feature that owns it:
 *   SearchByBoW(KF, F, v)     v[iF]  = KF feature whose MapPoint the reference assigns, or -1
 *   SearchByBoW(KF1, KF2, v)  v[i1]  = KF2 feature whose MapPoint the reference assigns, or -1
 * Distances and candidate filtering run on the GPU; the order-dependent acceptance (taken sets,
 * vMatchedDistance, rotation histogram) is replayed in the reference's iteration order, so match
 * indices are identical to the reference's.  GPU failures throw ORB_SLAM2::OrbGpuError.
 */
#ifndef ORBGPU_HOST_ORBMATCHER_H
#define ORBGPU_HOST_ORBMATCHER_H

#include <map>
#include <utility>
#include <vector>

#include "ORBextractor.h"

// The matcher lives in ORB_SLAM2 like the reference's.  When integrated next to the reference's own
// ORB_SLAM2::ORBmatcher (which keeps the projection-based searches), build with
// -DORBGPU_MATCHER_NAMESPACE=orbgpu_host.
#ifndef ORBGPU_MATCHER_NAMESPACE
#define ORBGPU_MATCHER_NAMESPACE ORB_SLAM2
#endif

namespace ORBGPU_MATCHER_NAMESPACE {

using ORB_SLAM2::DescriptorMat;
using ORB_SLAM2::KeyPoint;
using ORB_SLAM2::OrbGpuError;
using ORB_SLAM2::Point2f;

// DBoW2::FeatureVector (Thirdparty/DBoW2/DBoW2/FeatureVector.h: std::map<NodeId, std::vector<unsigned int>>)
typedef std::map<unsigned int, std::vector<unsigned int> > FeatureVector;

#define ORBGPU_FRAME_GRID_ROWS 48   // Frame.h:39
#define ORBGPU_FRAME_GRID_COLS 64   // Frame.h:40

// Frame::mGrid + GetFeaturesInArea (Frame.cc:378-412, 494-560).  The birdview grid
// (Frame.cc:877-940) is the same structure with minX = minY = 0 and its own cell sizes.
class FrameGrid {
public:
    FrameGrid() = default;
    // Frame grid: cells of (maxX-minX)/64 x (maxY-minY)/48 over mvKeysUn
    FrameGrid(const KeyPoint* keysUn, int n, float minX, float maxX, float minY, float maxY);
    // birdview grid: GridElementWidthInv/HeightInv given directly, origin (0, 0)
    static FrameGrid Birdview(const KeyPoint* keysBird, int n, float widthInv, float heightInv);
    std::vector<size_t> GetFeaturesInArea(float x, float y, float r, int minLevel = -1, int maxLevel = -1) const;

private:
    void assign(const KeyPoint* keys, int n);
    const KeyPoint* keys_ = nullptr;
    float minX_ = 0, minY_ = 0, invW_ = 0, invH_ = 0;
    std::vector<std::vector<size_t> > cells_;   // [ix * ROWS + iy]
};

// The members of a Frame / KeyFrame that ORBmatcher reads, as zero-copy views (cv::KeyPoint and
// orb_keypoint share one 28-byte layout; a continuous n x 32 CV_8U Mat is n*32 bytes).  Pointers
// may be NULL where a method does not read the member (see each method).
struct FeatureSet {
    int n = 0;                                        // N (Frame::N / KeyFrame::N / mvKeysBird.size())
    const KeyPoint* keys = nullptr;                   // Frame::mvKeys / KeyFrame::mvKeysUn / mvKeysBird
    const uint8_t* descriptors = nullptr;             // mDescriptors / mDescriptorsBird, row-major n x 32
    const FeatureVector* featVec = nullptr;           // mFeatVec
    const uint8_t* hasMapPoint = nullptr;             // per feature: MapPoint != NULL (&& !isBad() where read)
    const float* uRight = nullptr;                    // mvuRight
    const float* scaleFactors = nullptr;              // mvScaleFactors
    const float* levelSigma2 = nullptr;               // mvLevelSigma2
    int nlevels = 0;                                  // mnScaleLevels (length of the two tables above)
    const FrameGrid* grid = nullptr;                  // mGrid / mGridBirdview
    int N() const { return n; }
};
// Tags standing for the reference's Frame& and KeyFrame* arguments (so the overloads keep the
// reference's names: SearchByBoW(KeyFrame*, Frame&) vs SearchByBoW(KeyFrame*, KeyFrame*)).
struct FrameData : FeatureSet {};
struct KeyFrameData : FeatureSet {};

class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true);

    // Computes the Hamming distance between two ORB descriptors (ORBmatcher.cc:1647-1663)
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b);

    // ORBmatcher.cc:159-288.  KF: keys (mvKeysUn), descriptors, featVec, hasMapPoint (MP && !isBad);
    // F: keys (mvKeys), descriptors, featVec.
    int SearchByBoW(const KeyFrameData& KF, const FrameData& F, std::vector<int>& vpMapPointMatches);
    // ORBmatcher.cc:522-655.  Both: keys (mvKeysUn), descriptors, featVec, hasMapPoint (MP && !isBad).
    int SearchByBoW(const KeyFrameData& KF1, const KeyFrameData& KF2, std::vector<int>& vpMatches12);

    // ORBmatcher.cc:405-520.  F1: keys (mvKeysUn), descriptors; F2: keys, descriptors, grid.
    int SearchForInitialization(const FrameData& F1, const FrameData& F2, std::vector<Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10);

    // ORBmatcher.cc:657-823.  Both: keys (mvKeysUn), descriptors, featVec, hasMapPoint (GetMapPoint != NULL),
    // uRight; KF2: scaleFactors, levelSigma2.  F12 row-major 3x3; (ex, ey) = epipole of KF1's camera
    // centre in KF2 (:662-668, computed by the caller from the poses).
    int SearchForTriangulation(const KeyFrameData& KF1, const KeyFrameData& KF2, const float F12[9], float ex, float ey,
                               std::vector<std::pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo);
    // KF1 against several KF2s in one call (LocalMapping.cc:247-278's neighbour loop; orb_search_for_triangulation_batch):
    // vvMatchedPairs[p] == SearchForTriangulation(KF1, *neighbours[p].KF2, ...) for the same inputs.  Returns the total.
    struct TriangulationNeighbour {
        const KeyFrameData* KF2;
        float F12[9];
        float ex, ey;
    };
    int SearchForTriangulation(const KeyFrameData& KF1, const std::vector<TriangulationNeighbour>& neighbours,
                               std::vector<std::vector<std::pair<size_t, size_t> > >& vvMatchedPairs, const bool bOnlyStereo);

    // ORBmatcher.cc:1667-1789 (window around vPrevMatched, level-0 only, updates vPrevMatched) and
    // :1790-1899 (window around each keypoint).  F1: keys (mvKeysBird), descriptors;
    // F2: keys, descriptors, grid (FrameGrid::Birdview).
    int BirdviewMatch(const FrameData& F1, const FrameData& F2, std::vector<int>& vnMatches12,
                      std::vector<Point2f>& vPrevMatched, int windowSize = 10);
    int BirdviewMatch(const FrameData& F1, const FrameData& F2, std::vector<int>& vnMatches12, int windowSize = 10);

    static const int TH_LOW;
    static const int TH_HIGH;
    static const int HISTO_LENGTH;

protected:
    int window_match(bool level0_only, const FeatureSet& F1, const FeatureSet& F2, const std::vector<Point2f>* centres,
                     int windowSize, std::vector<int>& vnMatches12);
    float mfNNratio;
    bool mbCheckOrientation;
};

// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307), batched over map points:
// observations[m] = the descriptors (32 B each, observation order, bad keyframes skipped) of map
// point m.  Returns per point the index of the descriptor the reference copies into mDescriptor, or
// -1 for an empty list (the reference then leaves mDescriptor untouched).
std::vector<int> ComputeDistinctiveDescriptors(const std::vector<std::vector<const uint8_t*> >& observations);

}  // namespace ORBGPU_MATCHER_NAMESPACE

#endif
