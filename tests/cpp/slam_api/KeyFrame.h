// Test infrastructure: model of ORB_SLAM2::KeyFrame holding only the members the ported ORBmatcher
// searches read (include/KeyFrame.h: N, mvKeysUn, mvuRight, mDescriptors, mFeatVec, mvScaleFactors,
// mvLevelSigma2, fx, fy, cx, cy, GetMapPointMatches, GetMapPoint, GetCameraCenter, GetRotation,
// GetTranslation).  The pose is Tcw = [R | t]; the camera centre is Ow = -R^T t (KeyFrame::SetPose).
#ifndef ORBGPU_TEST_SLAM_API_KEYFRAME_H
#define ORBGPU_TEST_SLAM_API_KEYFRAME_H
#include <stddef.h>

#include <vector>

#include <opencv2/core/core.hpp>

#include "MapPoint.h"
#include "Thirdparty/DBoW2/DBoW2/FeatureVector.h"

namespace ORB_SLAM2 {

class KeyFrame {
public:
    float fx = 0, fy = 0, cx = 0, cy = 0;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeysUn;
    std::vector<float> mvuRight;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    std::vector<float> mvScaleFactors, mvLevelSigma2;
    std::vector<MapPoint*> mvpMapPoints;
    cv::Mat Rcw, tcw, Ow;   // 3x3, 3x1, 3x1 CV_32F

    void SetPose(const float R[9], const float t[3]) {
        Rcw = cv::Mat(3, 3, CV_32F);
        tcw = cv::Mat(3, 1, CV_32F);
        Ow = cv::Mat(3, 1, CV_32F);
        for (int i = 0; i < 9; i++) Rcw.at<float>(i / 3, i % 3) = R[i];
        for (int i = 0; i < 3; i++) tcw.at<float>(i) = t[i];
        for (int i = 0; i < 3; i++) {   // Ow = -Rcw^T tcw
            double s = 0;
            for (int k = 0; k < 3; k++) s += (double)R[3 * k + i] * (double)t[k];
            Ow.at<float>(i) = (float)-s;
        }
    }
    cv::Mat GetCameraCenter() { return Ow.clone(); }
    cv::Mat GetRotation() { return Rcw.clone(); }
    cv::Mat GetTranslation() { return tcw.clone(); }
    std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
    MapPoint* GetMapPoint(const size_t& idx) { return mvpMapPoints[idx]; }
};

}  // namespace ORB_SLAM2

#endif
