// Test infrastructure: model of ORB_SLAM2::Frame holding only the members the ported ORBmatcher searches
// read (include/Frame.h: N, mvKeys, mvKeysUn, mDescriptors, mFeatVec, mvKeysBird, mDescriptorsBird,
// GetFeaturesInArea, GetFeaturesInAreaBirdview).  The grid lookups follow Frame.cc:494-547 / :891-945
// through the oracle's restatement (oracle_features_in_area): the model is test-only.
#ifndef ORBGPU_TEST_SLAM_API_FRAME_H
#define ORBGPU_TEST_SLAM_API_FRAME_H
#include <stddef.h>

#include <vector>

#include <opencv2/core/core.hpp>

#include "../../../oracle/orb_oracle.h"
#include "Thirdparty/DBoW2/DBoW2/FeatureVector.h"

namespace ORB_SLAM2 {

class Frame {
public:
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    // image bounds of the 64 x 48 grid (Frame.cc:156-157: mnMinX .. mnMaxX, mnMinY .. mnMaxY)
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    // birdview stream (Frame.h:167-168); its grid covers [0, birdW) x [0, birdH) (Frame.cc:877-890)
    std::vector<cv::KeyPoint> mvKeysBird;
    cv::Mat mDescriptorsBird;
    float birdW = 0, birdH = 0;

    std::vector<size_t> GetFeaturesInArea(const float& x, const float& y, const float& r, const int minLevel = -1,
                                          const int maxLevel = -1) const {
        return area(mvKeysUn, mnMinX, mnMaxX, mnMinY, mnMaxY, x, y, r, minLevel, maxLevel);
    }
    std::vector<size_t> GetFeaturesInAreaBirdview(const float& x, const float& y, const float& r, const int minLevel = -1,
                                                  const int maxLevel = -1) const {
        return area(mvKeysBird, 0.f, birdW, 0.f, birdH, x, y, r, minLevel, maxLevel);
    }

private:
    static std::vector<size_t> area(const std::vector<cv::KeyPoint>& k, float x0, float x1, float y0, float y1, float x,
                                    float y, float r, int minLevel, int maxLevel) {
        std::vector<int> out(k.size() + 1);
        const int n = oracle_features_in_area((int)k.size(), reinterpret_cast<const OracleKeyPoint*>(k.data()), x0, x1,
                                              y0, y1, x, y, r, minLevel, maxLevel, out.data(), (int)out.size());
        return std::vector<size_t>(out.begin(), out.begin() + (n > 0 ? n : 0));
    }
};

}  // namespace ORB_SLAM2

#endif
