// Test infrastructure: model of DBoW2::FeatureVector (Thirdparty/DBoW2/DBoW2/FeatureVector.h of the
// reference: a std::map from vocabulary node id to the indices of the features under that node).
#ifndef ORBGPU_TEST_SLAM_API_FEATUREVECTOR_H
#define ORBGPU_TEST_SLAM_API_FEATUREVECTOR_H
#include <map>
#include <vector>

namespace DBoW2 {
typedef unsigned int NodeId;
class FeatureVector : public std::map<NodeId, std::vector<unsigned int> > {};
}  // namespace DBoW2

#endif
