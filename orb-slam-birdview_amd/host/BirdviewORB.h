/*
 * ORB_SLAM2::BirdviewORB / ORB_SLAM2::cornerSubPix — C++ mirror of the OpenCV calls the birdview stream
 * of Frame::Frame makes (reference src/Frame.cc:318-342) over liborbgpu's orb_bird_* C-ABI:
 *
 *     cv::rectangle(mBirdviewMask, footprint, Scalar(0), -1);         -> BirdviewFootprintMask
 *     cv::Ptr<cv::ORB> extractorBird = cv::ORB::create(2000);         -> BirdviewORB::create(2000)
 *     extractorBird->detect(mBirdviewImg, mvKeysBird, mBirdviewMask); -> detect
 *     cv::cornerSubPix(mBirdviewImg, vKeysBird, Size(5,5), Size(-1,-1), criteria);   -> cornerSubPix
 *     extractorBird->compute(mBirdviewImg, mvKeysBird, mDescriptorsBird);            -> compute
 *
 * plus the fused BirdviewORB::extractBirdview, which does all of it on one device upload.  Only the
 * configuration the reference uses is built: firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31,
 * cornerSubPix window (5,5) without a zero zone; other values throw OrbGpuError(ORB_ERR_ARG).
 * No CPU path: a GPU failure throws OrbGpuError.
 */
#ifndef ORBGPU_HOST_BIRDVIEWORB_H
#define ORBGPU_HOST_BIRDVIEWORB_H

#include <memory>
#include <vector>

#include "ORBextractor.h"

namespace ORB_SLAM2 {

struct Size {
    int width, height;
};

struct TermCriteria {
    enum { COUNT = 1, MAX_ITER = COUNT, EPS = 2 };
    int type, maxCount;
    double epsilon;
    TermCriteria(int t, int m, double e) : type(t), maxCount(m), epsilon(e) {}
};

class BirdviewORB {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };
    // cv::ORB::create (OpenCV 3.2 defaults); Frame.cc:329 calls create(2000)
    static std::shared_ptr<BirdviewORB> create(int nfeatures = 500, float scaleFactor = 1.2f, int nlevels = 8,
                                               int edgeThreshold = 31, int firstLevel = 0, int WTA_K = 2,
                                               int scoreType = HARRIS_SCORE, int patchSize = 31, int fastThreshold = 20);
    BirdviewORB(int nfeatures, float scaleFactor, int nlevels, int edgeThreshold, int fastThreshold, int device);
    ~BirdviewORB();
    BirdviewORB(const BirdviewORB&) = delete;
    BirdviewORB& operator=(const BirdviewORB&) = delete;

    // Feature2D::detect(image, keypoints, mask): empty image -> keypoints cleared
    void detect(const ImageView& image, std::vector<KeyPoint>& keypoints, const ImageView& mask = ImageView());
    // Feature2D::compute(image, keypoints, descriptors): keypoints border-culled / level-sorted in place
    void compute(const ImageView& image, std::vector<KeyPoint>& keypoints, DescriptorMat& descriptors);
    // Frame.cc:320-342 in one call: footprint-masked detect, cornerSubPix(5x5, 40, 0.001), compute
    void extractBirdview(const ImageView& image, const ImageView& birdviewMask, std::vector<KeyPoint>& keypoints,
                         DescriptorMat& descriptors);

    int descriptorSize() const { return 32; }
    orb_bird* handle() const { return h_; }

private:
    orb_bird* h_ = nullptr;
    int nfeatures_;
};

// cv::cornerSubPix(image, corners, winSize, zeroZone, criteria) on the GPU (Frame.cc:336-337)
void cornerSubPix(const ImageView& image, std::vector<Point2f>& corners, Size winSize, Size zeroZone,
                  TermCriteria criteria);

// Frame.cc:320-327: zero the vehicle footprint (+15 px) of a birdview mask (host, in place)
void BirdviewFootprintMask(uint8_t* mask, int cols, int rows, size_t step);

}  // namespace ORB_SLAM2

#endif
