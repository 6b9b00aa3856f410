/*
 * Frame::ComputeStereoMatches (src/Frame.cc:662-836) over liborbgpu: the stereo consumer of the
 * extractor's outputs.  The reference method reads mvKeys / mDescriptors / mvKeysRight /
 * mDescriptorsRight, the two extractors' mvImagePyramid, mb and mbf, and writes mvuRight / mvDepth;
 * this mirror takes exactly those members.  The window search reads the pyramids where the GPU
 * extraction left them (no mvImagePyramid download).  Both extractors must sit on one device and
 * have extracted the left / right image last.  GPU failures throw ORB_SLAM2::OrbGpuError.
 */
#ifndef ORBGPU_HOST_STEREO_H
#define ORBGPU_HOST_STEREO_H

#include <vector>

#include "ORBextractor.h"

namespace ORB_SLAM2 {

// Returns the number of left keypoints that received a depth.
int ComputeStereoMatches(const ORBextractor& left, const ORBextractor& right, const std::vector<KeyPoint>& mvKeys,
                         const DescriptorMat& mDescriptors, const std::vector<KeyPoint>& mvKeysRight,
                         const DescriptorMat& mDescriptorsRight, float mb, float mbf, std::vector<float>& mvuRight,
                         std::vector<float>& mvDepth);

}  // namespace ORB_SLAM2

#endif
