// Test infrastructure: model of ORB_SLAM2::MapPoint holding only what the ported ORBmatcher searches
// read (include/MapPoint.h: bool isBad()).
#ifndef ORBGPU_TEST_SLAM_API_MAPPOINT_H
#define ORBGPU_TEST_SLAM_API_MAPPOINT_H

namespace ORB_SLAM2 {
class MapPoint {
public:
    explicit MapPoint(bool bad = false) : mbBad(bad) {}
    bool isBad() { return mbBad; }
    bool mbBad;
};
}  // namespace ORB_SLAM2

#endif
