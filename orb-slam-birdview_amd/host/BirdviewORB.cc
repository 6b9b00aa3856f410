// ORB_SLAM2::BirdviewORB over liborbgpu's orb_bird_* entry points (see BirdviewORB.h).
#include "BirdviewORB.h"

#include <stdlib.h>

#include <algorithm>

namespace ORB_SLAM2 {

static void check(int st, const char* what) {
    if (st != ORB_OK) throw OrbGpuError(st, what);
}

static int env_device() {
    const char* e = getenv("ORBGPU_DEVICE");
    return e ? atoi(e) : 0;
}

int env_variant();   // ORBextractor.cc: ORBGPU_VARIANT


std::shared_ptr<BirdviewORB> BirdviewORB::create(int nfeatures, float scaleFactor, int nlevels, int edgeThreshold,
                                                 int firstLevel, int WTA_K, int scoreType, int patchSize,
                                                 int fastThreshold) {
    if (firstLevel != 0 || WTA_K != 2 || scoreType != HARRIS_SCORE || patchSize != 31)
        throw OrbGpuError(ORB_ERR_ARG, "BirdviewORB::create: only firstLevel 0, WTA_K 2, HARRIS_SCORE, patchSize 31");
    return std::make_shared<BirdviewORB>(nfeatures, scaleFactor, nlevels, edgeThreshold, fastThreshold, env_device());
}

BirdviewORB::BirdviewORB(int nfeatures, float scaleFactor, int nlevels, int edgeThreshold, int fastThreshold,
                         int device)
    : nfeatures_(nfeatures) {
    // cv::ORB's pyramid resize and descriptor blur follow the same OpenCV build as ORBextractor's: the
    // resize / blur bits of ORBGPU_VARIANT
    orb_bird_params p{nfeatures, scaleFactor, nlevels, edgeThreshold, fastThreshold, device,
                      env_variant() & (ORB_VARIANT_RESIZE_GENERIC | ORB_VARIANT_BLUR_HALFUP)};
    int st = ORB_OK;
    h_ = orb_bird_create(&p, &st);
    if (!h_) throw OrbGpuError(st, "orb_bird_create");
}

BirdviewORB::~BirdviewORB() { orb_bird_destroy(h_); }

void BirdviewORB::detect(const ImageView& image, std::vector<KeyPoint>& keypoints, const ImageView& mask) {
    if (image.empty()) {
        keypoints.clear();
        return;
    }
    int cap = 2 * std::max(nfeatures_, 1) + 256, n = 0;
    for (;;) {
        keypoints.resize(cap);
        const int st = orb_bird_detect(h_, image.data, image.cols, image.rows, image.step,
                                       mask.empty() ? nullptr : mask.data, mask.empty() ? 0 : mask.step,
                                       keypoints.data(), cap, &n);
        if (st == ORB_ERR_CAPACITY) {
            cap = n;
            continue;
        }
        check(st, "orb_bird_detect");
        break;
    }
    keypoints.resize(n);
}

void BirdviewORB::compute(const ImageView& image, std::vector<KeyPoint>& keypoints, DescriptorMat& descriptors) {
    if (image.empty()) {
        descriptors.release();
        return;
    }
    int n = (int)keypoints.size();
    descriptors.create(std::max(n, 1));
    check(orb_bird_compute(h_, image.data, image.cols, image.rows, image.step, keypoints.data(), &n,
                           descriptors.buf.data()),
          "orb_bird_compute");
    keypoints.resize(n);
    if (n == 0) descriptors.release();
    else descriptors.create(n);
}

void BirdviewORB::extractBirdview(const ImageView& image, const ImageView& birdviewMask,
                                  std::vector<KeyPoint>& keypoints, DescriptorMat& descriptors) {
    keypoints.clear();
    descriptors.release();
    if (image.empty()) return;
    int cap = 2 * std::max(nfeatures_, 1) + 256, n = 0;
    for (;;) {
        keypoints.resize(cap);
        descriptors.create(cap);
        const int st = orb_bird_extract(h_, image.data, image.cols, image.rows, image.step,
                                        birdviewMask.empty() ? nullptr : birdviewMask.data,
                                        birdviewMask.empty() ? 0 : birdviewMask.step, keypoints.data(), cap, &n,
                                        descriptors.buf.data());
        if (st == ORB_ERR_CAPACITY) {
            cap = n;
            continue;
        }
        check(st, "orb_bird_extract");
        break;
    }
    keypoints.resize(n);
    if (n == 0) descriptors.release();
    else descriptors.create(n);
}

void cornerSubPix(const ImageView& image, std::vector<Point2f>& corners, Size winSize, Size zeroZone,
                  TermCriteria criteria) {
    if (zeroZone.width >= 0 && zeroZone.height >= 0)
        throw OrbGpuError(ORB_ERR_ARG, "cornerSubPix: a zero zone is not built (Frame.cc:337 passes (-1,-1))");
    if (corners.empty()) return;
    // per-thread context on the default device (the reference calls cornerSubPix from the Tracking thread)
    thread_local std::unique_ptr<BirdviewORB> ctx;
    if (!ctx) ctx.reset(new BirdviewORB(500, 1.2f, 8, 31, 20, env_device()));
    const int iters = (criteria.type & TermCriteria::MAX_ITER) ? criteria.maxCount : 100;
    const double eps = (criteria.type & TermCriteria::EPS) ? criteria.epsilon : 0.0;
    check(orb_corner_subpix(ctx->handle(), image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<float*>(corners.data()), (int)corners.size(), winSize.width,
                            winSize.height, iters, eps),
          "orb_corner_subpix");
}

void BirdviewFootprintMask(uint8_t* mask, int cols, int rows, size_t step) {
    check(orb_bird_footprint_mask(mask, cols, rows, step), "orb_bird_footprint_mask");
}

}  // namespace ORB_SLAM2
