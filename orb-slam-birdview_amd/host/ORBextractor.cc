// ORB_SLAM2::ORBextractor over liborbgpu (see ORBextractor.h).  Host code only: every pixel is
// processed by the gfx950 kernels behind orb_extract.
#include "ORBextractor.h"

#include <assert.h>
#include <stdlib.h>
#include <string.h>

namespace ORB_SLAM2 {

OrbGpuError::OrbGpuError(int st, const std::string& what)
    : std::runtime_error(what + ": " + orb_last_error() + " (status " + std::to_string(st) + ")"), status(st) {}

static void check(int st, const char* what) {
    if (st != ORB_OK) throw OrbGpuError(st, what);
}

static int env_device() {
    const char* e = getenv("ORBGPU_DEVICE");
    return e ? atoi(e) : 0;
}

int env_variant() {
    const char* e = getenv("ORBGPU_VARIANT");
    return e ? (int)strtol(e, nullptr, 0) : ORB_VARIANT_DEFAULT;
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    init(env_device(), env_variant());
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST,
                           int device)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    init(device, env_variant());
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST,
                           int device, int variant)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST) {
    init(device, variant);
}

void ORBextractor::init(int device, int variant) {
    orb_params p;
    memset(&p, 0, sizeof p);
    p.nfeatures = nfeatures;
    p.scaleFactor = (float)scaleFactor;
    p.nlevels = nlevels;
    p.iniThFAST = iniThFAST;
    p.minThFAST = minThFAST;
    p.device = device;
    p.max_batch = 1;
    p.variant = variant;
    int st = ORB_OK;
    ctx_ = orb_create(&p, &st);
    if (!ctx_) throw OrbGpuError(st, "orb_create");
    // the tables of ORBextractor.cc:410-470, computed by the library (one definition for host and kernels)
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    umax.resize(16);
    check(orb_scale_tables(ctx_, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                           mvInvLevelSigma2.data(), mnFeaturesPerLevel.data(), umax.data()),
          "orb_scale_tables");
    mvImagePyramid.owner_ = this;
}

ORBextractor::~ORBextractor() {
    if (ctx_) orb_destroy(ctx_);
}

int ORBextractor::extract_raw(const uint8_t* data, int cols, int rows, size_t step) {
    const int cap = orb_batch_kp_cap(ctx_, cols, rows);   // exact upper bound for this image size
    if (cap < 0) throw OrbGpuError(cap, "orb_batch_kp_cap");
    if ((int)kbuf_.size() < cap) {
        kbuf_.resize(cap);
        dbuf_.resize((size_t)cap * 32);
    }
    int n = 0;
    check(orb_extract(ctx_, data, cols, rows, step, kbuf_.data(), (int)kbuf_.size(), &n, dbuf_.data()),
          "orb_extract");
    mvImagePyramid.invalidate((size_t)nlevels);
    return n;
}

void ORBextractor::operator()(const ImageView& image, const ImageView& /*mask*/, std::vector<KeyPoint>& keypoints,
                              DescriptorMat& descriptors) {
    if (image.empty()) return;   // ORBextractor.cc:1046-1047
    const int n = extract_raw(image.data, image.cols, image.rows, image.step);
    // :1061-1070: descriptors n x 32, released when there is no keypoint
    if (n == 0)
        descriptors.release();
    else
        descriptors.create(n);
    keypoints.assign(kbuf_.begin(), kbuf_.begin() + n);
    if (n) memcpy(descriptors.buf.data(), dbuf_.data(), (size_t)n * 32);
}

#ifdef ORBGPU_WITH_OPENCV
static_assert(sizeof(cv::KeyPoint) == sizeof(KeyPoint), "cv::KeyPoint layout");

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray /*_mask*/, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors) {
    if (_image.empty()) return;   // ORBextractor.cc:1046-1047
    cv::Mat image = _image.getMat();
    assert(image.type() == CV_8UC1);   // :1050
    const int n = extract_raw(image.data, image.cols, image.rows, image.step);
    if (n == 0) {
        _descriptors.release();
    } else {
        _descriptors.create(n, 32, CV_8U);
        cv::Mat d = _descriptors.getMat();
        memcpy(d.data, dbuf_.data(), (size_t)n * 32);
    }
    _keypoints.resize(n);
    // cv::KeyPoint has user constructors (not trivially copyable by type): copy the layout-checked bytes
    if (n) memcpy(static_cast<void*>(_keypoints.data()), kbuf_.data(), (size_t)n * sizeof(KeyPoint));
}
#endif

/* ---------------- mvImagePyramid ---------------- */
size_t ImagePyramid::size() const { return valid_.size(); }

void ImagePyramid::invalidate(size_t nlevels) {
    views_.assign(nlevels, ImageView());
    valid_.assign(nlevels, 0);
#ifdef ORBGPU_WITH_OPENCV
    mats_.assign(nlevels, cv::Mat());
#endif
}

const ImageView& ImagePyramid::fetch(size_t level) const {
    if (level >= valid_.size()) throw std::out_of_range("mvImagePyramid level");
    if (!valid_[level]) {
        const uint8_t* p = nullptr;
        int w = 0, h = 0;
        size_t stride = 0;
        check(orb_get_level(owner_->ctx_, (int)level, &p, &w, &h, &stride), "orb_get_level");
        views_[level] = ImageView(p, w, h, stride);
        valid_[level] = 1;
    }
    return views_[level];
}

#ifdef ORBGPU_WITH_OPENCV
const cv::Mat& ImagePyramid::operator[](size_t level) const {
    const ImageView& v = fetch(level);
    if (mats_[level].empty()) mats_[level] = cv::Mat(v.rows, v.cols, CV_8U, const_cast<uint8_t*>(v.data), v.step);
    return mats_[level];
}
#else
const ImageView& ImagePyramid::operator[](size_t level) const { return fetch(level); }
#endif

}  // namespace ORB_SLAM2
