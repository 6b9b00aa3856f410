/*
 * ORB_SLAM2::ORBextractor — C++ mirror of the reference class (include/ORBextractor.h:45-111) over
 * liborbgpu's C-ABI (include/orbgpu.h).  Same constructor, operator(), getters and public
 * mvImagePyramid; the work runs in gfx950 HIP kernels, there is no CPU path.
 *
 * Without OpenCV (this image) the image/keypoint/descriptor containers are the plain types below
 * (cv::KeyPoint-compatible 28-byte KeyPoint, n x 32 DescriptorMat).  With -DORBGPU_WITH_OPENCV the
 * reference's exact overload operator()(cv::InputArray, cv::InputArray, std::vector<cv::KeyPoint>&,
 * cv::OutputArray) is added and mvImagePyramid[l] is a cv::Mat.
 *
 * Error behaviour: as the reference, an empty image returns leaving the outputs untouched
 * (ORBextractor.cc:1046-1047) and a non-8UC1 image is an assert (:1050); a GPU failure (no device,
 * HIP error, internal overflow) throws ORB_SLAM2::OrbGpuError — it never falls back to the CPU.
 */
#ifndef ORBGPU_HOST_ORBEXTRACTOR_H
#define ORBGPU_HOST_ORBEXTRACTOR_H

#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"

#ifdef ORBGPU_WITH_OPENCV
#include <opencv2/core/core.hpp>
#endif

namespace ORB_SLAM2 {

class OrbGpuError : public std::runtime_error {
public:
    OrbGpuError(int status, const std::string& what);
    int status;
};

// cv::KeyPoint layout {Point2f pt; float size, angle, response; int octave, class_id;}
typedef orb_keypoint KeyPoint;

struct Point2f {
    float x, y;
};

// Gray 8-bit image view (cv::Mat CV_8UC1 stand-in): rows `step` bytes apart.
struct ImageView {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;
    ImageView() = default;
    ImageView(const uint8_t* d, int c, int r, size_t s = 0) : data(d), cols(c), rows(r), step(s ? s : (size_t)c) {}
    bool empty() const { return data == nullptr || cols <= 0 || rows <= 0; }
    uint8_t at(int y, int x) const { return data[(size_t)y * step + x]; }
};

// n x 32 CV_8U descriptor matrix stand-in (row i = descriptor of keypoint i).
struct DescriptorMat {
    int rows = 0;
    static const int cols = 32;
    std::vector<uint8_t> buf;
    bool empty() const { return rows == 0; }
    void create(int n) {
        rows = n;
        buf.resize((size_t)n * 32);
    }
    void release() {
        rows = 0;
        std::vector<uint8_t>().swap(buf);
    }
    uint8_t* ptr(int r) { return buf.data() + (size_t)r * 32; }
    const uint8_t* ptr(int r) const { return buf.data() + (size_t)r * 32; }
};

class ORBextractor;

// std::vector<cv::Mat> mvImagePyramid (ORBextractor.h:85): levels of the last extracted frame,
// copied device->host on first access after each extraction (Frame::ComputeStereoMatches reads
// them, Frame.cc:669,759).  Level l has GetScaleFactors()[l]-scaled size.
class ImagePyramid {
public:
    size_t size() const;
    bool empty() const { return size() == 0; }
#ifdef ORBGPU_WITH_OPENCV
    const cv::Mat& operator[](size_t level) const;
#else
    const ImageView& operator[](size_t level) const;
#endif

private:
    friend class ORBextractor;
    ORBextractor* owner_ = nullptr;
    mutable std::vector<ImageView> views_;
#ifdef ORBGPU_WITH_OPENCV
    mutable std::vector<cv::Mat> mats_;
#endif
    mutable std::vector<uint8_t> valid_;
    void invalidate(size_t nlevels);
    const ImageView& fetch(size_t level) const;
};

class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    // ORBextractor.cc:410-470.  The device is ORBGPU_DEVICE (default 0) unless given; the OpenCV arithmetic
    // variant (ORB_VARIANT_* bits of include/orbgpu.h, matching the OpenCV the reference build links) is
    // ORBGPU_VARIANT (default 0 = OpenCV 3.2) unless given, so Tracking.cc:121-127 constructs it unchanged.
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device);
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device,
                 int variant);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    // Compute the ORB features and descriptors on an image (ORBextractor.cc:1043-1105).
    // Mask is ignored, as in the reference (ORBextractor.h:58).
    void operator()(const ImageView& image, const ImageView& mask, std::vector<KeyPoint>& keypoints,
                    DescriptorMat& descriptors);
#ifdef ORBGPU_WITH_OPENCV
    void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                    cv::OutputArray descriptors);
#endif

    int inline GetLevels() { return nlevels; }
    float inline GetScaleFactor() { return (float)scaleFactor; }
    std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
    std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
    std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
    std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

    ImagePyramid mvImagePyramid;

    // not in the reference: the device context (for batched multi-frame use through the C-ABI)
    orb_ctx* context() const { return ctx_; }

protected:
    int nfeatures;
    double scaleFactor;   // ORBextractor.h:98 (double member: mvScaleFactor[i] = mvScaleFactor[i-1]*scaleFactor)
    int nlevels;
    int iniThFAST;
    int minThFAST;

    std::vector<int> mnFeaturesPerLevel;
    std::vector<int> umax;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

private:
    friend class ImagePyramid;
    void init(int device, int variant);
    int extract_raw(const uint8_t* data, int cols, int rows, size_t step);   // returns #keypoints in kbuf_/dbuf_
    orb_ctx* ctx_ = nullptr;
    std::vector<KeyPoint> kbuf_;
    std::vector<uint8_t> dbuf_;
};

}  // namespace ORB_SLAM2

#endif
