// Test infrastructure: a minimal model of the OpenCV 3.2 core types that the host mirror's
// -DORBGPU_WITH_OPENCV overloads (host/ORBextractor.h/.cc) and the ORBmatcher adapter
// (adapter/ORBmatcher_gpu.cc) touch.  OpenCV is absent in this image; this header lets that code be
// compiled and driven (tests/cpp/test_cv_overload.cc, tests/cpp/test_matcher_adapter.cc).  It is NOT
// OpenCV: only the member names, argument order and semantics of the calls made are modelled, after
// OpenCV 3.2's public API (core/mat.hpp: Mat(rows, cols, type[, data, step]), Mat::create/release/
// empty/type/ptr/at/row, MatExpr A*B + C evaluated as one gemm; core/types.hpp: Point2f, KeyPoint
// {Point2f pt; float size, angle, response; int octave, class_id}).
//
// gemm (matmul.cpp GEMMSingleMul for CV_32F): products summed in double, alpha*sum + beta*C in double,
// one rounding to float -- the model follows that form; a real OpenCV build computes its own.
#ifndef ORBGPU_TEST_CV_API_CORE_HPP
#define ORBGPU_TEST_CV_API_CORE_HPP

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <vector>

#define CV_8U 0
#define CV_8UC1 CV_8U
#define CV_32F 5

namespace cv {

typedef unsigned char uchar;

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f, angle = -1.f, response = 0.f;
    int octave = 0, class_id = -1;
};

class MatExpr;

class Mat {
public:
    Mat() = default;
    // allocating (zero-filled)
    Mat(int r, int c, int t) { create(r, c, t); }
    // external data, not owned (Mat(rows, cols, type, data, step))
    Mat(int r, int c, int t, void* d, size_t s = 0)
        : rows(r), cols(c), data(static_cast<uchar*>(d)), step(s ? s : (size_t)c * esize(t)), type_(t) {}
    Mat(const MatExpr& e);
    Mat& operator=(const MatExpr& e);
    void create(int r, int c, int t) {
        if (rows == r && cols == c && type_ == t && data) return;
        store_ = std::make_shared<std::vector<uchar>>((size_t)r * c * esize(t));
        rows = r;
        cols = c;
        type_ = t;
        step = (size_t)c * esize(t);
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
    bool isContinuous() const { return rows <= 1 || step == (size_t)cols * esize(type_); }
    uchar* ptr(int r = 0) { return data + (size_t)r * step; }
    const uchar* ptr(int r = 0) const { return data + (size_t)r * step; }
    template <class T>
    T& at(int r, int c) { return reinterpret_cast<T*>(ptr(r))[c]; }
    template <class T>
    const T& at(int r, int c) const { return reinterpret_cast<const T*>(ptr(r))[c]; }
    // single index on a row or column vector (Mat::at<T>(i0))
    template <class T>
    T& at(int i) { return cols == 1 ? at<T>(i, 0) : at<T>(0, i); }
    template <class T>
    const T& at(int i) const { return cols == 1 ? at<T>(i, 0) : at<T>(0, i); }
    // row header sharing the data (Mat::row)
    Mat row(int r) const {
        Mat m(*this);
        m.rows = 1;
        m.data = data + (size_t)r * step;
        return m;
    }
    Mat clone() const {
        Mat m(rows, cols, type_);
        for (int r = 0; r < rows; r++)
            for (size_t b = 0; b < (size_t)cols * esize(type_); b++) m.ptr(r)[b] = ptr(r)[b];
        return m;
    }

    int rows = 0, cols = 0;
    uchar* data = nullptr;
    size_t step = 0;

private:
    static size_t esize(int t) { return t == CV_32F ? 4 : 1; }
    int type_ = CV_8U;
    std::shared_ptr<std::vector<uchar>> store_;
};

// A*B (+ C): evaluated when converted to a Mat, as OpenCV's MatOp_GEMM does
class MatExpr {
public:
    Mat a, b, c;
    bool hasC = false;
    Mat eval() const {
        if (a.type() != CV_32F || b.type() != CV_32F || a.cols != b.rows) throw std::runtime_error("cv model: gemm shape");
        Mat d(a.rows, b.cols, CV_32F);
        for (int i = 0; i < a.rows; i++)
            for (int j = 0; j < b.cols; j++) {
                double s = 0;
                for (int k = 0; k < a.cols; k++) s += (double)a.at<float>(i, k) * (double)b.at<float>(k, j);
                if (hasC) s += (double)c.at<float>(i, j);
                d.at<float>(i, j) = (float)s;
            }
        return d;
    }
};

inline Mat::Mat(const MatExpr& e) { *this = e.eval(); }
inline Mat& Mat::operator=(const MatExpr& e) { return *this = e.eval(); }
inline MatExpr operator*(const Mat& a, const Mat& b) {
    MatExpr e;
    e.a = a;
    e.b = b;
    return e;
}
inline MatExpr operator+(const MatExpr& e, const Mat& c) {
    MatExpr r = e;
    r.c = c;
    r.hasC = true;
    return r;
}

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
