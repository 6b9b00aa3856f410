// Test infrastructure: a minimal model of the OpenCV 3.2 core types that the host mirror's
// -DORBGPU_WITH_OPENCV overloads touch (host/ORBextractor.h/.cc).  OpenCV is absent in this image;
// this header lets those overloads be compiled and driven (tests/cpp/test_cv_overload.cc).  It is
// NOT OpenCV: only the member names, argument order and semantics of the calls the mirror makes are
// modelled, after OpenCV 3.2's public API (core/mat.hpp: Mat(rows, cols, type, data, step),
// Mat::create/release/empty/type, _InputArray::getMat/empty, _OutputArray::create/getMat/release;
// core/types.hpp: KeyPoint {Point2f pt; float size, angle, response; int octave, class_id}).
#ifndef ORBGPU_TEST_CV_API_CORE_HPP
#define ORBGPU_TEST_CV_API_CORE_HPP

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 CV_8U

namespace cv {

typedef unsigned char uchar;

struct Point2f {
    float x = 0.f, y = 0.f;
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};

class Mat {
public:
    Mat() = default;
    // external data, not owned (Mat(rows, cols, type, data, step))
    Mat(int r, int c, int t, void* d, size_t s = 0)
        : rows(r), cols(c), data(static_cast<uchar*>(d)), step(s ? s : (size_t)c), type_(t) {}
    void create(int r, int c, int t) {
        if (rows == r && cols == c && type_ == t && data) return;
        store_ = std::make_shared<std::vector<uchar>>((size_t)r * c);
        rows = r;
        cols = c;
        type_ = t;
        step = (size_t)c;
        data = store_->data();
    }
    void release() {
        store_.reset();
        rows = cols = 0;
        step = 0;
        data = nullptr;
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return type_; }
    uchar* ptr(int r) { return data + (size_t)r * step; }
    const uchar* ptr(int r) const { return data + (size_t)r * step; }

    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;

private:
    int type_ = CV_8U;
    std::shared_ptr<std::vector<uchar>> store_;
};

class _InputArray {
public:
    _InputArray(const Mat& m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat* m_;
};

class _OutputArray {
public:
    _OutputArray(Mat& m) : m_(&m) {}
    void create(int r, int c, int t) const { m_->create(r, c, t); }
    Mat getMat() const { return *m_; }
    void release() const { m_->release(); }

private:
    Mat* m_;
};

typedef const _InputArray& InputArray;
typedef const _OutputArray& OutputArray;

}  // namespace cv

#endif
