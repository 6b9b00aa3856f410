// Model of ORB_SLAM2::Frame holding only the members the ported ORBmatcher searches read
// (include/Frame.h: N, mvKeys, mvKeysUn, mDescriptors, mFeatVec, mvKeysBird, mDescriptorsBird,
// GetFeaturesInArea, GetFeaturesInAreaBirdview).  This is the CALLER's code (the reference keeps it on
// the CPU): the 64 x 48 grid is built the way Frame::AssignFeaturesToGrid does (Frame.cc:378-413,
// PosInGrid :549-559, PosInGridBirdview :879-889) and queried as Frame::GetFeaturesInArea
// (:494-547) / GetFeaturesInAreaBirdview (:891-945) do.  Used by the adapter test and by the matcher
// bench tool (tools/matcher_latency.cc); AssignFeaturesToGrid() must be called once the keypoints are
// set, as the reference's constructor does.
#ifndef ORBGPU_TEST_SLAM_API_FRAME_H
#define ORBGPU_TEST_SLAM_API_FRAME_H
#include <math.h>
#include <stddef.h>

#include <algorithm>
#include <vector>

#include <opencv2/core/core.hpp>

#include "Thirdparty/DBoW2/DBoW2/FeatureVector.h"

#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

namespace ORB_SLAM2 {

class Frame {
public:
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    cv::Mat mDescriptors;
    DBoW2::FeatureVector mFeatVec;
    // image bounds of the 64 x 48 grid (Frame.cc:156-157: mnMinX .. mnMaxX, mnMinY .. mnMaxY)
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    // birdview stream (Frame.h:167-168); its grid covers [0, birdW) x [0, birdH) (Frame.cc:282-283)
    std::vector<cv::KeyPoint> mvKeysBird;
    cv::Mat mDescriptorsBird;
    float birdW = 0, birdH = 0;

    // the grids (Frame.h:211, 217) and their inverse cell sizes (static members in the reference,
    // Frame.cc:96-97, 156-157, 282-283)
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    float mfGridElementWidthInvBirdview = 0, mfGridElementHeightInvBirdview = 0;
    std::vector<std::size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
    std::vector<std::size_t> mGridBirdview[FRAME_GRID_COLS][FRAME_GRID_ROWS];

    // what the Frame constructor does once its keypoints exist (Frame.cc:156-157, 282-283, 378-413)
    void AssignFeaturesToGrid() {
        mfGridElementWidthInv = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
        mfGridElementHeightInv = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
        fill(mGrid, mvKeysUn, mnMinX, mnMinY, mfGridElementWidthInv, mfGridElementHeightInv);
        mfGridElementWidthInvBirdview = birdW > 0 ? static_cast<float>(FRAME_GRID_COLS) / birdW : 0.f;
        mfGridElementHeightInvBirdview = birdH > 0 ? static_cast<float>(FRAME_GRID_ROWS) / birdH : 0.f;
        fill(mGridBirdview, mvKeysBird, 0.f, 0.f, mfGridElementWidthInvBirdview, mfGridElementHeightInvBirdview);
    }

    std::vector<size_t> GetFeaturesInArea(const float& x, const float& y, const float& r, const int minLevel = -1,
                                          const int maxLevel = -1) const {
        return area(mGrid, mvKeysUn, x - mnMinX, y - mnMinY, x, y, r, mfGridElementWidthInv, mfGridElementHeightInv,
                    minLevel, maxLevel);
    }
    std::vector<size_t> GetFeaturesInAreaBirdview(const float& x, const float& y, const float& r, const int minLevel = -1,
                                                  const int maxLevel = -1) const {
        return area(mGridBirdview, mvKeysBird, x, y, x, y, r, mfGridElementWidthInvBirdview,
                    mfGridElementHeightInvBirdview, minLevel, maxLevel);
    }

private:
    typedef std::vector<std::size_t> Grid[FRAME_GRID_COLS][FRAME_GRID_ROWS];

    static void fill(Grid& g, const std::vector<cv::KeyPoint>& k, float x0, float y0, float gw, float gh) {
        for (int i = 0; i < FRAME_GRID_COLS; i++)
            for (int j = 0; j < FRAME_GRID_ROWS; j++) g[i][j].clear();
        for (size_t i = 0; i < k.size(); i++) {   // PosInGrid: round() of the float product, in double
            const int px = (int)round((k[i].pt.x - x0) * gw), py = (int)round((k[i].pt.y - y0) * gh);
            if (px < 0 || px >= FRAME_GRID_COLS || py < 0 || py >= FRAME_GRID_ROWS) continue;
            g[px][py].push_back(i);
        }
    }

    // (dx, dy) = the query relative to the grid origin; (x, y) the query itself (Frame.cc:499-545)
    static std::vector<size_t> area(const Grid& g, const std::vector<cv::KeyPoint>& k, float dx, float dy, float x,
                                    float y, float r, float gw, float gh, int minLevel, int maxLevel) {
        std::vector<size_t> v;
        v.reserve(k.size());
        const int nMinCellX = std::max(0, (int)floor((dx - r) * gw));
        if (nMinCellX >= FRAME_GRID_COLS) return v;
        const int nMaxCellX = std::min((int)FRAME_GRID_COLS - 1, (int)ceil((dx + r) * gw));
        if (nMaxCellX < 0) return v;
        const int nMinCellY = std::max(0, (int)floor((dy - r) * gh));
        if (nMinCellY >= FRAME_GRID_ROWS) return v;
        const int nMaxCellY = std::min((int)FRAME_GRID_ROWS - 1, (int)ceil((dy + r) * gh));
        if (nMaxCellY < 0) return v;
        const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
                for (size_t j : g[ix][iy]) {
                    const cv::KeyPoint& kp = k[j];
                    if (bCheckLevels) {
                        if (kp.octave < minLevel) continue;
                        if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                    }
                    const float distx = kp.pt.x - x, disty = kp.pt.y - y;
                    if (fabs(distx) < r && fabs(disty) < r) v.push_back(j);
                }
        return v;
    }
};

}  // namespace ORB_SLAM2

#endif
