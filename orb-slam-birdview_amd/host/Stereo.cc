// Frame::ComputeStereoMatches over liborbgpu (see Stereo.h).
#include "Stereo.h"

namespace ORB_SLAM2 {

int ComputeStereoMatches(const ORBextractor& left, const ORBextractor& right, const std::vector<KeyPoint>& mvKeys,
                         const DescriptorMat& mDescriptors, const std::vector<KeyPoint>& mvKeysRight,
                         const DescriptorMat& mDescriptorsRight, float mb, float mbf, std::vector<float>& mvuRight,
                         std::vector<float>& mvDepth) {
    const int N = (int)mvKeys.size(), Nr = (int)mvKeysRight.size();
    mvuRight.assign(N, -1.0f);   // Frame.cc:664-665
    mvDepth.assign(N, -1.0f);
    if (N == 0) return 0;
    static const uint8_t dummy[32] = {0};
    int n = 0;
    const int st = orb_compute_stereo_matches(left.context(), right.context(), N, mvKeys.data(), mDescriptors.buf.data(),
                                              Nr, Nr ? mvKeysRight.data() : nullptr,
                                              Nr ? mDescriptorsRight.buf.data() : dummy, mb, mbf, mvuRight.data(),
                                              mvDepth.data(), &n);
    if (st != ORB_OK) throw OrbGpuError(st, "ComputeStereoMatches");
    return n;
}

}  // namespace ORB_SLAM2
