// Test infrastructure: model of the reference's ORB_SLAM2::ORBmatcher declaration (include/ORBmatcher.h:
// 37-119), reduced to the constructor, the data members and the six methods that
// orb-slam-birdview_amd/adapter/ORBmatcher_gpu.cc defines, with the reference's exact signatures.
#ifndef ORBGPU_TEST_SLAM_API_ORBMATCHER_H
#define ORBGPU_TEST_SLAM_API_ORBMATCHER_H
#include <utility>
#include <vector>

#include <opencv2/core/core.hpp>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {

using std::pair;
using std::vector;

class ORBmatcher {
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);
    int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10);
    int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                               std::vector<pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo);
    // the declarations a maintainer adds to include/ORBmatcher.h for the batched forms
    int SearchByBoW(const std::vector<KeyFrame*>& vpKFs, Frame& F, std::vector<std::vector<MapPoint*> >& vvpMapPointMatches,
                    std::vector<int>& vnMatches);
    int SearchByBoW(KeyFrame* pKF1, const std::vector<KeyFrame*>& vpKF2, std::vector<std::vector<MapPoint*> >& vvpMatches12,
                    std::vector<int>& vnMatches);
    int SearchForTriangulation(KeyFrame* pKF1, const std::vector<KeyFrame*>& vpKF2, const std::vector<cv::Mat>& vF12,
                               std::vector<std::vector<pair<size_t, size_t> > >& vvMatchedPairs, const bool bOnlyStereo);
    int BirdviewMatch(Frame& F1, Frame& F2, vector<int>& vnMatches12, vector<cv::Point2f>& vPrevMatched,
                      int windowSize = 10);
    int BirdviewMatch(const Frame& F1, const Frame& F2, vector<int>& vnMatches12, int windowSize = 10);

protected:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2

#endif
