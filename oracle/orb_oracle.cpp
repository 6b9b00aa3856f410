/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  See orb_oracle.h for scope and parity status.
 *
 * Built with -O3 -march=native -ffp-contract=off (oracle/Makefile): the restatement never
 * contracts a*b+c into an FMA, matching the pinned float semantics the HIP path uses.
 * Every function cites the reference file:line it restates.
 */
#include "orb_oracle.h"
#include "glibc_sincosf.inc"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <list>
#include <map>
#include <cstdio>
#include <thread>
#include <utility>
#include <vector>
#include <climits>
#include <cfloat>

namespace {

const int PATCH_SIZE = 31;        // ORBextractor.cc:72
const int HALF_PATCH_SIZE = 15;   // ORBextractor.cc:73
const int EDGE_THRESHOLD = 19;    // ORBextractor.cc:74

#include "pattern31_data.inc"
const int kPattern[1024] = { ORACLE_PATTERN31_VALUES };

/* ---------------- OpenCV 3.2 rounding helpers ---------------- */
inline int cvRound(float v) { return (int)std::nearbyint(v); }     // _mm_cvtss_si32, half-even
inline int cvRound(double v) { return (int)std::nearbyint(v); }    // _mm_cvtsd_si32, half-even
inline int cvFloor(float v) { return (int)std::floor(v); }
inline int cvCeil(float v) { return (int)std::ceil(v); }
inline short sat_short(int v) { return (short)std::min(std::max(v, (int)SHRT_MIN), (int)SHRT_MAX); }
inline uint8_t sat_u8(int v) { return (uint8_t)std::min(std::max(v, 0), 255); }

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> d;
    void create(int W, int H) { w = W; h = H; d.assign((size_t)W * H, 0); }
    uint8_t* row(int y) { return d.data() + (size_t)y * w; }
    const uint8_t* row(int y) const { return d.data() + (size_t)y * w; }
};

struct KP {
    float x, y, size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(KP) == 28, "cv::KeyPoint layout");

/* ---------------- cv::resize INTER_LINEAR, 8UC1 (OpenCV 3.2 imgwarp.cpp; Appendix A.1) ------ */
void resize_linear_8u(const Img& src, Img& dst, int dw, int dh, int flags) {
    const int sw = src.w, sh = src.h;
    dst.create(dw, dh);
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = sat_short(cvRound(c0 * 2048));
        ialpha[2 * dx + 1] = sat_short(cvRound(c1 * 2048));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        yofs[dy] = sy;
        float c0 = 1.f - fy, c1 = fy;
        ibeta[2 * dy] = sat_short(cvRound(c0 * 2048));
        ibeta[2 * dy + 1] = sat_short(cvRound(c1 * 2048));
    }
    std::vector<int> H0(dw), H1(dw);
    auto hresize = [&](const uint8_t* S, int* D) {
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) D[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
            else D[dx] = S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < dh; dy++) {
        int sy0 = std::min(std::max(yofs[dy], 0), sh - 1);
        int sy1 = std::min(std::max(yofs[dy] + 1, 0), sh - 1);
        hresize(src.row(sy0), H0.data());
        hresize(src.row(sy1), H1.data());
        int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = dst.row(dy);
        for (int x = 0; x < dw; x++) {
            if (flags & ORACLE_RESIZE_GENERIC)
                D[x] = sat_u8((b0 * H0[x] + b1 * H1[x] + (1 << 21)) >> 22);
            else
                D[x] = (uint8_t)((((b0 * (H0[x] >> 4)) >> 16) + ((b1 * (H1[x] >> 4)) >> 16) + 2) >> 2);
        }
    }
}

/* ---------------- GaussianBlur(7x7, sigma 2, REFLECT_101), 8U (Appendix A.2) ---------------- */
void gaussian_kernel_q8(int k[7]) {
    // getGaussianKernel(7, 2, CV_32F) then convertTo(CV_32S, 256) (cvRound half-even)
    float cf[7];
    double sum = 0;
    const double sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX);
    for (int i = 0; i < 7; i++) {
        double x = i - 3.0;
        double t = std::exp(scale2X * x * x);
        cf[i] = (float)t;
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) cf[i] = (float)(cf[i] * sum);
    for (int i = 0; i < 7; i++) k[i] = cvRound(cf[i] * 256.f);
}

inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

void gauss7_blur(const Img& src, Img& dst, int flags) {
    int k[7];
    gaussian_kernel_q8(k);
    const int W = src.w, H = src.h;
    // R: the exact integer row pass (RowFilter<uchar,int>), REFLECT_101 at the clone's edges.  The
    // interior loop has no border logic so the compiler vectorises it (the oracle is also the timed
    // CPU baseline); the arithmetic is unchanged.
    std::vector<int> R((size_t)W * H);
    for (int y = 0; y < H; y++) {
        const uint8_t* s = src.row(y);
        int* r = &R[(size_t)y * W];
        auto edge = [&](int x) {
            int acc = 0;
            for (int j = 0; j < 7; j++) acc += k[j] * s[reflect101(x + j - 3, W)];
            r[x] = acc;
        };
        const int x0 = std::min(3, W), x1 = std::max(x0, W - 3);
        for (int x = 0; x < x0; x++) edge(x);
        for (int x = x0; x < x1; x++)
            r[x] = k[0] * s[x - 3] + k[1] * s[x - 2] + k[2] * s[x - 1] + k[3] * s[x] + k[4] * s[x + 1] + k[5] * s[x + 2] +
                   k[6] * s[x + 3];
        for (int x = x1; x < W; x++) edge(x);
    }
    dst.create(W, H);
    const int xsimd = (flags & ORACLE_BLUR_ALL_HALFUP) ? 0 : (W & ~3);   // SymmColumnVec_32s8u covers multiples of 4
    for (int y = 0; y < H; y++) {
        const int* rr[7];
        for (int i = 0; i < 7; i++) rr[i] = &R[(size_t)reflect101(y + i - 3, H) * W];
        uint8_t* o = dst.row(y);
        for (int x = 0; x < W; x++) {
            const int S = k[0] * rr[0][x] + k[1] * rr[1][x] + k[2] * rr[2][x] + k[3] * rr[3][x] + k[4] * rr[4][x] +
                          k[5] * rr[5][x] + k[6] * rr[6][x];
            const int q = S >> 16, rem = S & 0xFFFF;
            // SSE2 body (x < W & ~3): _mm_cvtps_epi32, half to even; scalar tail: FixedPtCastEx, half up
            const int even = rem > 32768 ? q + 1 : (rem < 32768 ? q : q + (q & 1));
            const int v = x < xsimd ? even : (S + 32768) >> 16;
            o[x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
}

/* ---------------- cv::FAST 9/16 with NMS (OpenCV 3.2 fast.cpp FAST_t; Appendix A.3) --------- */
int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[N];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

struct Corner { int x, y, score; };

// FAST on an image ROI (base points at ROI(0,0)); emits (x, y, score) in detection order.
void fast9_roi(const uint8_t* base, int step, int rows, int cols, int threshold, std::vector<Corner>& out) {
    out.clear();
    const int K = 8, N = 25;
    static const int offs[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                                    {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = offs[k][0] + offs[k][1] * step;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    threshold = std::min(std::max(threshold, 0), 255);
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
    if (cols <= 0 || rows <= 0) return;
    // row buffers on the stack for cell-sized ROIs, as OpenCV's AutoBuffer does (no heap traffic per
    // cell: ORACLE_TIE_LITERAL's heap then sees only the allocations the reference makes)
    uint8_t sbuf[3 * 128];
    int scp[3 * 129];
    std::vector<uint8_t> bufv;
    std::vector<int> cpv;
    uint8_t* b0 = sbuf;
    int* c0 = scp;
    if (cols > 128) {
        bufv.assign((size_t)cols * 3, 0);
        cpv.assign((size_t)(cols + 1) * 3, 0);
        b0 = bufv.data();
        c0 = cpv.data();
    } else {
        std::memset(sbuf, 0, (size_t)cols * 3);
        std::memset(scp, 0, sizeof(int) * (size_t)(cols + 1) * 3);
    }
    uint8_t* buf[3] = {b0, b0 + cols, b0 + 2 * cols};
    int* cpbuf[3] = {c0 + 1, c0 + (cols + 1) + 1, c0 + 2 * (cols + 1) + 1};
    for (int i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = base + (size_t)i * step + 3;
        uint8_t* curr = buf[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        std::memset(curr, 0, cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (int j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* t = tab - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (int k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = buf[(i - 4 + 3) % 3];
        const uint8_t* pprev = buf[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (int k = 0; k < ncorners; k++) {
            int j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] && score > pprev[j] &&
                score > pprev[j + 1] && score > curr[j - 1] && score > curr[j] && score > curr[j + 1])
                out.push_back({j, i - 1, score});
        }
    }
}

/* ---------------- fastAtan2 (OpenCV 3.2 mathfuncs; Appendix A.4) ---------------- */
const float atan2_p1 = 0.9997878412794807f * (float)(180 / M_PI);
const float atan2_p3 = -0.3258083974640975f * (float)(180 / M_PI);
const float atan2_p5 = 0.1555786518463281f * (float)(180 / M_PI);
const float atan2_p7 = -0.04432655554792128f * (float)(180 / M_PI);

float fastAtan2(float y, float x) {
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((atan2_p7 * c2 + atan2_p5) * c2 + atan2_p3) * c2 + atan2_p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* IC_Angle  ORBextractor.cc:77-104 */
float IC_Angle(const Img& image, float px, float py, const std::vector<int>& u_max) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = image.row(cvRound(py)) + cvRound(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    int step = image.w;
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = u_max[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fastAtan2((float)m_01, (float)m_10);
}

/* BRIEF rotation trig (ORBextractor.cc:113, std::cos/std::sin of a float = glibc cosf/sinf, merged by
 * GCC -O3 into one sincosf): glibc 2.35's algorithm restated in glibc_sincosf.inc, FMA ifunc variant,
 * pinned bit for bit against libm over every float in [0, 2*pi] (tools/trig_pin.cpp).
 * ORACLE_TRIG_CR gives round 1's correctly rounded pin instead (sensitivity only). */
inline float orb_cos(float a, int flags) {
    return (flags & ORACLE_TRIG_CR) ? (float)std::cos((double)a) : glibc_sincosf::cosf_(a);
}
inline float orb_sin(float a, int flags) {
    return (flags & ORACLE_TRIG_CR) ? (float)std::sin((double)a) : glibc_sincosf::sinf_(a);
}
/* OpenCV's own (uncontracted) build of the same call (cv::ORB, birdview stream): glibc trig too */
inline float cv_cosf(float a) { return glibc_sincosf::cosf_(a); }
inline float cv_sinf(float a) { return glibc_sincosf::sinf_(a); }

const float factorPI = (float)(M_PI / 180.f);   // ORBextractor.cc:107

/* computeOrbDescriptor  ORBextractor.cc:108-147.  The reference is built -O3 -march=native
 * (CMakeLists.txt:10-11), so on an FMA host GCC contracts the two sample-offset expressions of :119-120;
 * tools/ref_flags_probe.cpp compiled with those flags fixes the forms: y = fma(x, b, y*a),
 * x = fma(x, a, -(y*b)).  ORACLE_NO_FMA evaluates them uncontracted (sensitivity only). */
void computeOrbDescriptor(const KP& kpt, const Img& img, const int* pattern, uint8_t* desc, int flags) {
    float angle = (float)kpt.angle * factorPI;
    float a = orb_cos(angle, flags), b = orb_sin(angle, flags);
    const uint8_t* center = img.row(cvRound(kpt.y)) + cvRound(kpt.x);
    const int step = img.w;
    const bool fused = !(flags & ORACLE_NO_FMA);
    auto GET = [&](const int* p, int idx) -> int {
        float px = (float)p[2 * idx], py = (float)p[2 * idx + 1];
        const float oy = fused ? std::fmaf(px, b, py * a) : px * b + py * a;
        const float ox = fused ? std::fmaf(px, a, -(py * b)) : px * a - py * b;
        return center[cvRound(oy) * step + cvRound(ox)];
    };
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int k = 0; k < 8; k++) {
            int t0 = GET(pattern, 2 * k), t1 = GET(pattern, 2 * k + 1);
            val |= (t0 < t1) << k;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ---------------- ExtractorNode / DistributeOctTree  ORBextractor.cc:481-763 ---------------- */
struct Node {
    std::vector<KP> vKeys;
    int ULx = 0, ULy = 0, URx = 0, URy = 0, BLx = 0, BLy = 0, BRx = 0, BRy = 0;
    std::list<Node>::iterator lit;
    bool bNoMore = false;
    long seq = -1;   // creation sequence: the pinned stand-in for the node's heap address (:684)

    void DivideNode(Node& n1, Node& n2, Node& n3, Node& n4) const {   // :481-537
        const int halfX = (int)std::ceil(static_cast<float>(URx - ULx) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(BRy - ULy) / 2);
        n1.ULx = ULx; n1.ULy = ULy;
        n1.URx = ULx + halfX; n1.URy = ULy;
        n1.BLx = ULx; n1.BLy = ULy + halfY;
        n1.BRx = ULx + halfX; n1.BRy = ULy + halfY;
        n1.vKeys.reserve(vKeys.size());
        n2.ULx = n1.URx; n2.ULy = n1.URy;
        n2.URx = URx; n2.URy = URy;
        n2.BLx = n1.BRx; n2.BLy = n1.BRy;
        n2.BRx = URx; n2.BRy = ULy + halfY;
        n2.vKeys.reserve(vKeys.size());
        n3.ULx = n1.BLx; n3.ULy = n1.BLy;
        n3.URx = n1.BRx; n3.URy = n1.BRy;
        n3.BLx = BLx; n3.BLy = BLy;
        n3.BRx = n1.BRx; n3.BRy = BLy;
        n3.vKeys.reserve(vKeys.size());
        n4.ULx = n3.URx; n4.ULy = n3.URy;
        n4.URx = n2.BRx; n4.URy = n2.BRy;
        n4.BLx = n3.BRx; n4.BLy = n3.BRy;
        n4.BRx = BRx; n4.BRy = BRy;
        n4.vKeys.reserve(vKeys.size());
        for (size_t i = 0; i < vKeys.size(); i++) {
            const KP& kp = vKeys[i];
            if (kp.x < n1.URx) {
                if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
                else n3.vKeys.push_back(kp);
            } else if (kp.y < n1.BRy) n2.vKeys.push_back(kp);
            else n4.vKeys.push_back(kp);
        }
        if (n1.vKeys.size() == 1) n1.bNoMore = true;
        if (n2.vKeys.size() == 1) n2.bNoMore = true;
        if (n3.vKeys.size() == 1) n3.bNoMore = true;
        if (n4.vKeys.size() == 1) n4.bNoMore = true;
    }
};

std::vector<KP> DistributeOctTree(const std::vector<KP>& vToDistributeKeys, int minX, int maxX, int minY,
                                  int maxY, int N, bool reverseTie) {
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));   // :543
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<Node> lNodes;
    long seqCounter = 0;
    std::vector<Node*> vpIniNodes(nIni);
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.ULx = (int)(hX * static_cast<float>(i)); ni.ULy = 0;
        ni.URx = (int)(hX * static_cast<float>(i + 1)); ni.URy = 0;
        ni.BLx = ni.ULx; ni.BLy = maxY - minY;
        ni.BRx = ni.URx; ni.BRy = maxY - minY;
        ni.vKeys.reserve(vToDistributeKeys.size());
        ni.seq = seqCounter++;
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (size_t i = 0; i < vToDistributeKeys.size(); i++) {
        const KP& kp = vToDistributeKeys[i];
        vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
    }
    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) { lit->bNoMore = true; lit++; }
        else if (lit->vKeys.empty()) lit = lNodes.erase(lit);
        else lit++;
    }
    bool bFinish = false;
    std::vector<std::pair<int, Node*>> vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    auto push_child = [&](Node& c, std::vector<std::pair<int, Node*>>& vec, int* nToExpand) {
        if (c.vKeys.size() > 0) {
            c.seq = seqCounter++;
            lNodes.push_front(c);
            if (c.vKeys.size() > 1) {
                if (nToExpand) (*nToExpand)++;
                vec.push_back(std::make_pair((int)c.vKeys.size(), &lNodes.front()));
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {                                                            // :594-739
        int prevSize = (int)lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) { lit++; continue; }
            Node n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            push_child(n1, vSizeAndPointerToNode, &nToExpand);
            push_child(n2, vSizeAndPointerToNode, &nToExpand);
            push_child(n3, vSizeAndPointerToNode, &nToExpand);
            push_child(n4, vSizeAndPointerToNode, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                std::vector<std::pair<int, Node*>> vPrev = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                // :684 sort(pair<int,ExtractorNode*>) — pointer tie pinned to creation sequence
                std::sort(vPrev.begin(), vPrev.end(),
                          [reverseTie](const std::pair<int, Node*>& a, const std::pair<int, Node*>& b) {
                              if (a.first != b.first) return a.first < b.first;
                              return reverseTie ? a.second->seq > b.second->seq : a.second->seq < b.second->seq;
                          });
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    Node n1, n2, n3, n4;
                    vPrev[j].second->DivideNode(n1, n2, n3, n4);
                    push_child(n1, vSizeAndPointerToNode, nullptr);
                    push_child(n2, vSizeAndPointerToNode, nullptr);
                    push_child(n3, vSizeAndPointerToNode, nullptr);
                    push_child(n4, vSizeAndPointerToNode, nullptr);
                    lNodes.erase(vPrev[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<KP> vResultKeys;                                                   // :741-762
    for (auto it = lNodes.begin(); it != lNodes.end(); it++) {
        std::vector<KP>& vNodeKeys = it->vKeys;
        KP* pKP = &vNodeKeys[0];
        float maxResponse = pKP->response;
        for (size_t k = 1; k < vNodeKeys.size(); k++)
            if (vNodeKeys[k].response > maxResponse) { pKP = &vNodeKeys[k]; maxResponse = vNodeKeys[k].response; }
        vResultKeys.push_back(*pKP);
    }
    return vResultKeys;
}

/* ---------------- DistributeOctTree as the reference RUNS it (ORACLE_TIE_LITERAL) ----------------
 * ORBextractor.cc:481-763 with the reference's own data structures, so that the heap sees the same
 * allocation sequence: nodes laid out like ExtractorNode (ORBextractor.h:32-43: vector<cv::KeyPoint>,
 * four cv::Point2i, a list iterator, a bool) in a std::list, children created as locals with
 * reserve(parent size) and copied in with push_front, parents erased, and the final phase sorting
 * std::pair<int, node*> — equal sizes ordered by heap ADDRESS (:684), i.e. by whatever glibc malloc
 * handed out in this process.  Used only to measure the tie-order sensitivity (tools/tie_study.py). */
struct LPoint { int x, y; };
struct LNode {
    LNode() : bNoMore(false) {}
    std::vector<KP> vKeys;
    LPoint UL, UR, BL, BR;
    std::list<LNode>::iterator lit;
    bool bNoMore;

    void DivideNode(LNode& n1, LNode& n2, LNode& n3, LNode& n4) {   // :481-537
        const int halfX = (int)std::ceil(static_cast<float>(UR.x - UL.x) / 2);
        const int halfY = (int)std::ceil(static_cast<float>(BR.y - UL.y) / 2);
        n1.UL = UL;
        n1.UR = {UL.x + halfX, UL.y};
        n1.BL = {UL.x, UL.y + halfY};
        n1.BR = {UL.x + halfX, UL.y + halfY};
        n1.vKeys.reserve(vKeys.size());
        n2.UL = n1.UR;
        n2.UR = UR;
        n2.BL = n1.BR;
        n2.BR = {UR.x, UL.y + halfY};
        n2.vKeys.reserve(vKeys.size());
        n3.UL = n1.BL;
        n3.UR = n1.BR;
        n3.BL = BL;
        n3.BR = {n1.BR.x, BL.y};
        n3.vKeys.reserve(vKeys.size());
        n4.UL = n3.UR;
        n4.UR = n2.BR;
        n4.BL = n3.BR;
        n4.BR = BR;
        n4.vKeys.reserve(vKeys.size());
        for (const KP& kp : vKeys) {
            if (kp.x < n1.UR.x) (kp.y < n1.BR.y ? n1 : n3).vKeys.push_back(kp);
            else (kp.y < n1.BR.y ? n2 : n4).vKeys.push_back(kp);
        }
        for (LNode* n : {&n1, &n2, &n3, &n4})
            if (n->vKeys.size() == 1) n->bNoMore = true;
    }
};

std::vector<KP> DistributeOctTreeLiteral(const std::vector<KP>& vToDistributeKeys, int minX, int maxX, int minY,
                                         int maxY, int N, int nfeatures) {
    const int nIni = (int)std::round(static_cast<float>(maxX - minX) / (maxY - minY));   // :543
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<LNode> lNodes;
    std::vector<LNode*> vpIniNodes;
    vpIniNodes.resize(nIni);
    for (int i = 0; i < nIni; i++) {                                                     // :552-563
        LNode ni;
        ni.UL = {(int)(hX * static_cast<float>(i)), 0};
        ni.UR = {(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = {ni.UL.x, maxY - minY};
        ni.BR = {ni.UR.x, maxY - minY};
        ni.vKeys.reserve(vToDistributeKeys.size());
        lNodes.push_back(ni);
        vpIniNodes[i] = &lNodes.back();
    }
    for (const KP& kp : vToDistributeKeys) vpIniNodes[(size_t)(kp.x / hX)]->vKeys.push_back(kp);   // :566-570
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {                             // :574-585
        if (lit->vKeys.size() == 1) { lit->bNoMore = true; ++lit; }
        else if (lit->vKeys.empty()) lit = lNodes.erase(lit);
        else ++lit;
    }
    bool bFinish = false;
    std::vector<std::pair<int, LNode*>> vSizeAndPointerToNode;
    vSizeAndPointerToNode.reserve(lNodes.size() * 4);
    // children n1..n4 of `parent` into the list front (:621-660 / :691-726)
    auto add_children = [&](LNode& n1, LNode& n2, LNode& n3, LNode& n4, int* nToExpand) {
        for (LNode* c : {&n1, &n2, &n3, &n4}) {
            if (c->vKeys.size() > 0) {
                lNodes.push_front(*c);
                if (c->vKeys.size() > 1) {
                    if (nToExpand) (*nToExpand)++;
                    vSizeAndPointerToNode.push_back(std::make_pair((int)c->vKeys.size(), &lNodes.front()));
                    lNodes.front().lit = lNodes.begin();
                }
            }
        }
    };
    while (!bFinish) {                                                                   // :594-739
        int prevSize = (int)lNodes.size();
        auto lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPointerToNode.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) { ++lit; continue; }
            LNode n1, n2, n3, n4;
            lit->DivideNode(n1, n2, n3, n4);
            add_children(n1, n2, n3, n4, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                std::vector<std::pair<int, LNode*>> vPrevSizeAndPointerToNode = vSizeAndPointerToNode;
                vSizeAndPointerToNode.clear();
                std::sort(vPrevSizeAndPointerToNode.begin(), vPrevSizeAndPointerToNode.end());   // :684
                for (int j = (int)vPrevSizeAndPointerToNode.size() - 1; j >= 0; j--) {
                    LNode n1, n2, n3, n4;
                    vPrevSizeAndPointerToNode[j].second->DivideNode(n1, n2, n3, n4);
                    add_children(n1, n2, n3, n4, nullptr);
                    lNodes.erase(vPrevSizeAndPointerToNode[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<KP> vResultKeys;                                                         // :741-762
    vResultKeys.reserve(nfeatures);
    for (auto& node : lNodes) {
        const KP* pKP = &node.vKeys[0];
        float maxResponse = pKP->response;
        for (size_t k = 1; k < node.vKeys.size(); k++)
            if (node.vKeys[k].response > maxResponse) { pKP = &node.vKeys[k]; maxResponse = node.vKeys[k].response; }
        vResultKeys.push_back(*pKP);
    }
    return vResultKeys;
}

/* ---------------- the extractor object (ORBextractor.cc:410-470, 765-853, 1043-1132) ------- */
struct Extractor {
    int nfeatures, nlevels, iniThFAST, minThFAST, flags;
    double scaleFactor;   // ORBextractor.h:98 stores it as double
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;
    std::vector<int> mnFeaturesPerLevel, umax;
    std::vector<Img> pyr, blurred;
    std::vector<std::vector<KP>> cand, lvlKps;
    std::vector<KP> outKps;
    std::vector<uint8_t> outDesc;
    // per-stage wall time (ms), accumulated over run() calls: pyramid, FAST (+NMS), octree, IC angle,
    // blur, BRIEF (the CPU baseline reports where its time goes)
    double stage_ms[6] = {0, 0, 0, 0, 0, 0};
    typedef std::chrono::steady_clock Clock;
    static double ms_since(Clock::time_point& t) {
        const Clock::time_point n = Clock::now();
        const double d = std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
        return d;
    }

    Extractor(int nf, float sf, int nl, int ini, int mn, int fl)
        : nfeatures(nf), nlevels(nl), iniThFAST(ini), minThFAST(mn), flags(fl), scaleFactor(sf) {
        mvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvScaleFactor[0] = 1.0f;
        mvLevelSigma2[0] = 1.0f;
        for (int i = 1; i < nlevels; i++) {
            mvScaleFactor[i] = (float)(mvScaleFactor[i - 1] * scaleFactor);
            mvLevelSigma2[i] = mvScaleFactor[i] * mvScaleFactor[i];
        }
        mvInvScaleFactor.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        for (int i = 0; i < nlevels; i++) {
            mvInvScaleFactor[i] = 1.0f / mvScaleFactor[i];
            mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
        }
        mnFeaturesPerLevel.resize(nlevels);
        float factor = (float)(1.0f / scaleFactor);
        float nDesiredFeaturesPerScale =
            nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
        int sumFeatures = 0;
        for (int level = 0; level < nlevels - 1; level++) {
            mnFeaturesPerLevel[level] = cvRound(nDesiredFeaturesPerScale);
            sumFeatures += mnFeaturesPerLevel[level];
            nDesiredFeaturesPerScale *= factor;
        }
        mnFeaturesPerLevel[nlevels - 1] = std::max(nfeatures - sumFeatures, 0);
        umax.resize(HALF_PATCH_SIZE + 1);
        int v, v0, vmax = cvFloor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
        int vmin = cvCeil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
        const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
        for (v = 0; v <= vmax; ++v) umax[v] = cvRound(std::sqrt(hp2 - v * v));
        for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }

    bool ComputePyramid(const Img& image) {                                        // :1107-1132
        pyr.assign(nlevels, Img());
        for (int level = 0; level < nlevels; ++level) {
            float scale = mvInvScaleFactor[level];
            int w = cvRound((float)image.w * scale), h = cvRound((float)image.h * scale);
            if (w < 2 || h < 2) return false;
            if (level != 0) resize_linear_8u(pyr[level - 1], pyr[level], w, h, flags);
            else pyr[0] = image;
        }
        return true;
    }

    bool ComputeKeyPointsOctTree() {                                                // :765-853
        cand.assign(nlevels, {});
        lvlKps.assign(nlevels, {});
        const bool literal = (flags & ORACLE_TIE_LITERAL) != 0;
        const float W = 30;
        std::vector<Corner> corners;
        corners.reserve(4096);
        for (int level = 0; level < nlevels; ++level) {
            Clock::time_point t = Clock::now();
            const Img& im = pyr[level];
            const int minBorderX = EDGE_THRESHOLD - 3;
            const int minBorderY = minBorderX;
            const int maxBorderX = im.w - EDGE_THRESHOLD + 3;
            const int maxBorderY = im.h - EDGE_THRESHOLD + 3;
            // literal mode: the reference's local vector and its reserve (:778-779), so the heap sees
            // the reference's allocations; the pinned mode keeps the candidates for the debug view
            std::vector<KP> local;
            if (literal) local.reserve((size_t)nfeatures * 10);
            std::vector<KP>& vToDistributeKeys = literal ? local : cand[level];
            const float width = (float)(maxBorderX - minBorderX);
            const float height = (float)(maxBorderY - minBorderY);
            const int nCols = (int)(width / W);
            const int nRows = (int)(height / W);
            if (nCols <= 0 || nRows <= 0) return false;   // reference: division by zero (UB)
            const int wCell = (int)std::ceil(width / nCols);
            const int hCell = (int)std::ceil(height / nRows);
            for (int i = 0; i < nRows; i++) {
                const float iniY = (float)(minBorderY + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBorderY - 3) continue;
                if (maxY > maxBorderY) maxY = (float)maxBorderY;
                for (int j = 0; j < nCols; j++) {
                    const float iniX = (float)(minBorderX + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBorderX - 6) continue;
                    if (maxX > maxBorderX) maxX = (float)maxBorderX;
                    const int y0 = (int)iniY, y1 = (int)maxY, x0 = (int)iniX, x1 = (int)maxX;
                    const uint8_t* roi = im.row(y0) + x0;
                    fast9_roi(roi, im.w, y1 - y0, x1 - x0, iniThFAST, corners);
                    if (corners.empty()) fast9_roi(roi, im.w, y1 - y0, x1 - x0, minThFAST, corners);
                    std::vector<KP> vKeysCell;   // :808, grown by push_back as cv::FAST grows it
                    for (const Corner& c : corners) vKeysCell.push_back(KP{(float)c.x, (float)c.y, 7.f, -1.f, (float)c.score, 0, -1});
                    for (KP& kp : vKeysCell) {
                        kp.x += j * wCell;
                        kp.y += i * hCell;
                        vToDistributeKeys.push_back(kp);
                    }
                }
            }
            if ((float)(maxBorderX - minBorderX) / (maxBorderY - minBorderY) < 0.5f) return false;  // nIni==0
            std::vector<KP>& keypoints = lvlKps[level];
            stage_ms[1] += ms_since(t);
            if (literal) {
                keypoints.reserve(nfeatures);   // :832
                keypoints = DistributeOctTreeLiteral(vToDistributeKeys, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                                     mnFeaturesPerLevel[level], nfeatures);
            } else {
                keypoints = DistributeOctTree(vToDistributeKeys, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                              mnFeaturesPerLevel[level], (flags & ORACLE_TIE_REVERSE_SEQ) != 0);
            }
            stage_ms[2] += ms_since(t);
            const int scaledPatchSize = (int)(PATCH_SIZE * mvScaleFactor[level]);
            for (KP& kp : keypoints) {
                kp.x += minBorderX;
                kp.y += minBorderY;
                kp.octave = level;
                kp.size = (float)scaledPatchSize;
            }
        }
        Clock::time_point t = Clock::now();
        for (int level = 0; level < nlevels; ++level)                             // :851-852
            for (KP& kp : lvlKps[level]) kp.angle = IC_Angle(pyr[level], kp.x, kp.y, umax);
        stage_ms[3] += ms_since(t);
        return true;
    }

    int run(const Img& image) {                                                     // :1043-1105
        if (image.w == 0 || image.h == 0) return -1;
        Clock::time_point t = Clock::now();
        if (!ComputePyramid(image)) return -2;
        stage_ms[0] += ms_since(t);
        if (!ComputeKeyPointsOctTree()) return -2;
        t = Clock::now();
        int nkeypoints = 0;
        for (int level = 0; level < nlevels; ++level) nkeypoints += (int)lvlKps[level].size();
        outKps.clear();
        outDesc.assign((size_t)nkeypoints * 32, 0);
        blurred.assign(nlevels, Img());
        int offset = 0;
        for (int level = 0; level < nlevels; ++level) {
            std::vector<KP> keypoints = lvlKps[level];
            const int nkl = (int)keypoints.size();
            if (nkl == 0) continue;
            gauss7_blur(pyr[level], blurred[level], flags);
            stage_ms[4] += ms_since(t);
            for (int i = 0; i < nkl; i++)
                computeOrbDescriptor(keypoints[i], blurred[level], kPattern, &outDesc[(size_t)(offset + i) * 32], flags);
            stage_ms[5] += ms_since(t);
            offset += nkl;
            if (level != 0) {
                float scale = mvScaleFactor[level];
                for (KP& kp : keypoints) { kp.x *= scale; kp.y *= scale; }
            }
            outKps.insert(outKps.end(), keypoints.begin(), keypoints.end());
        }
        return nkeypoints;
    }
};

/* ---------------- matcher helpers (ORBmatcher.cc) ---------------- */
const int TH_LOW = 50, HISTO_LENGTH = 30;   // ORBmatcher.cc:37-39 (TH_HIGH=100 unused on this path)

int DescriptorDistance(const uint8_t* a, const uint8_t* b) {   // ORBmatcher.cc:1647-1663
    int32_t pa[8], pb[8];
    std::memcpy(pa, a, 32);
    std::memcpy(pb, b, 32);
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        unsigned int v = (unsigned)pa[i] ^ (unsigned)pb[i];
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

void ComputeThreeMaxima(const std::vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3) {  // :1601-1642
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

int rot_bin(float a1, float a2) {   // e.g. ORBmatcher.cc:236-243
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// Iterate nodes present in both FeatureVectors in ascending id order (the std::map merge with
// lower_bound jumps of ORBmatcher.cc:175-264 visits exactly these pairs in this order).
template <class F>
void for_common_nodes(const OracleFeatVec& a, const OracleFeatVec& b, F f) {
    int i = 0, j = 0;
    while (i < a.nnodes && j < b.nnodes) {
        if (a.node_ids[i] == b.node_ids[j]) { f(i, j); i++; j++; }
        else if (a.node_ids[i] < b.node_ids[j]) i++;
        else j++;
    }
}

void cull_rotation(std::vector<int>* rotHist, std::vector<int>& matches, int& nmatches) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    ComputeThreeMaxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
    for (int i = 0; i < HISTO_LENGTH; i++) {
        if (i == ind1 || i == ind2 || i == ind3) continue;
        for (size_t j = 0; j < rotHist[i].size(); j++) {
            if (matches[rotHist[i][j]] >= 0) { matches[rotHist[i][j]] = -1; nmatches--; }
        }
    }
}

const float* CheckF(const float* F, int r, int c) { return &F[r * 3 + c]; }

bool CheckDistEpipolarLine(const KP& kp1, const KP& kp2, const float* F12, const float* sigma2) {  // :140-157
    // the contraction GCC applies to these lines under the reference's -O3 -march=native on an FMA host,
    // as tools/ref_flags_probe.cpp compiles them (the oracle itself is built -ffp-contract=off)
    const float a = std::fmaf(kp1.x, *CheckF(F12, 0, 0), kp1.y * *CheckF(F12, 1, 0)) + *CheckF(F12, 2, 0);
    const float b = std::fmaf(kp1.x, *CheckF(F12, 0, 1), kp1.y * *CheckF(F12, 1, 1)) + *CheckF(F12, 2, 1);
    const float c = std::fmaf(kp1.y, *CheckF(F12, 1, 2), kp1.x * *CheckF(F12, 0, 2)) + *CheckF(F12, 2, 2);
    const float num = std::fmaf(b, kp2.y, a * kp2.x) + c;
    const float den = std::fmaf(a, a, b * b);
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2[kp2.octave];
}

}  // namespace

/* ============================== extern "C" API ============================== */
extern "C" {

void* oracle_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int flags) {
    if (nlevels < 1 || nfeatures < 0) return nullptr;
    return new Extractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, flags);
}
void oracle_destroy(void* h) { delete (Extractor*)h; }

int oracle_run(void* h, const uint8_t* img, int w, int hgt, int stride) {
    Extractor* e = (Extractor*)h;
    if (!img || w <= 0 || hgt <= 0) return -1;
    Img im;
    im.create(w, hgt);
    for (int y = 0; y < hgt; y++) std::memcpy(im.row(y), img + (size_t)y * stride, w);
    return e->run(im);
}

int oracle_level_size(void* h, int level, int* w, int* hgt) {
    Extractor* e = (Extractor*)h;
    if (level < 0 || level >= (int)e->pyr.size()) return -1;
    *w = e->pyr[level].w;
    *hgt = e->pyr[level].h;
    return 0;
}
int oracle_get_level(void* h, int level, uint8_t* out) {
    Extractor* e = (Extractor*)h;
    if (level < 0 || level >= (int)e->pyr.size()) return -1;
    std::memcpy(out, e->pyr[level].d.data(), e->pyr[level].d.size());
    return 0;
}
int oracle_get_blurred(void* h, int level, uint8_t* out) {
    Extractor* e = (Extractor*)h;
    if (level < 0 || level >= (int)e->pyr.size()) return -1;
    Img b;
    gauss7_blur(e->pyr[level], b, e->flags);
    std::memcpy(out, b.d.data(), b.d.size());
    return 0;
}
int oracle_get_candidates(void* h, int level, int* out, int cap) {
    Extractor* e = (Extractor*)h;
    if (level < 0 || level >= (int)e->cand.size()) return -1;
    const auto& c = e->cand[level];
    if ((int)c.size() > cap) return -(int)c.size() - 1;
    for (size_t i = 0; i < c.size(); i++) {
        out[3 * i] = (int)c[i].x;
        out[3 * i + 1] = (int)c[i].y;
        out[3 * i + 2] = (int)c[i].response;
    }
    return (int)c.size();
}
int oracle_get_level_keypoints(void* h, int level, OracleKeyPoint* out, int cap) {
    Extractor* e = (Extractor*)h;
    if (level < 0 || level >= (int)e->lvlKps.size()) return -1;
    const auto& k = e->lvlKps[level];
    if ((int)k.size() > cap) return -(int)k.size() - 1;
    std::memcpy(out, k.data(), k.size() * sizeof(KP));
    return (int)k.size();
}
int oracle_get_output(void* h, OracleKeyPoint* kps, uint8_t* desc, int cap) {
    Extractor* e = (Extractor*)h;
    int n = (int)e->outKps.size();
    if (n > cap) return -n - 1;
    std::memcpy(kps, e->outKps.data(), n * sizeof(KP));
    std::memcpy(desc, e->outDesc.data(), (size_t)n * 32);
    return n;
}
void oracle_tables(void* h, float* scale, float* invScale, float* sigma2, float* invSigma2, int* nPerLevel,
                   int* umax16) {
    Extractor* e = (Extractor*)h;
    for (int i = 0; i < e->nlevels; i++) {
        scale[i] = e->mvScaleFactor[i];
        invScale[i] = e->mvInvScaleFactor[i];
        sigma2[i] = e->mvLevelSigma2[i];
        invSigma2[i] = e->mvInvLevelSigma2[i];
        nPerLevel[i] = e->mnFeaturesPerLevel[i];
    }
    for (int i = 0; i < 16; i++) umax16[i] = e->umax[i];
}

float oracle_fast_atan2(float y, float x) { return fastAtan2(y, x); }
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return DescriptorDistance(a, b); }
void oracle_three_maxima(const int* sizes, int L, int* i1, int* i2, int* i3) {
    std::vector<std::vector<int>> h(L);
    for (int i = 0; i < L; i++) h[i].resize(sizes[i]);
    *i1 = *i2 = *i3 = -1;
    ComputeThreeMaxima(h.data(), L, *i1, *i2, *i3);
}
int oracle_rot_bin(float a1, float a2) { return rot_bin(a1, a2); }
int oracle_fast_roi(const uint8_t* roi, int w, int h, int stride, int th, int* out, int cap) {
    std::vector<Corner> v;
    fast9_roi(roi, stride, h, w, th, v);
    if ((int)v.size() > cap) return -(int)v.size() - 1;
    for (size_t i = 0; i < v.size(); i++) {
        out[3 * i] = v[i].x;
        out[3 * i + 1] = v[i].y;
        out[3 * i + 2] = v[i].score;
    }
    return (int)v.size();
}
void oracle_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, int flags) {
    Img s, d;
    s.create(sw, sh);
    std::memcpy(s.d.data(), src, (size_t)sw * sh);
    resize_linear_8u(s, d, dw, dh, flags);
    std::memcpy(dst, d.d.data(), (size_t)dw * dh);
}
void oracle_blur(const uint8_t* src, int w, int h, uint8_t* dst, int flags) {
    Img s, d;
    s.create(w, h);
    std::memcpy(s.d.data(), src, (size_t)w * h);
    gauss7_blur(s, d, flags);
    std::memcpy(dst, d.d.data(), (size_t)w * h);
}
void oracle_pattern(int* out) { std::memcpy(out, kPattern, sizeof(kPattern)); }
void oracle_sincosf(const float* x, int n, float* s, float* c) {
    for (int i = 0; i < n; i++) {
        s[i] = glibc_sincosf::sinf_(x[i]);
        c[i] = glibc_sincosf::cosf_(x[i]);
    }
}

double oracle_time_extract(const uint8_t* frames, int nframes, int w, int h, int nfeatures, float scaleFactor,
                           int nlevels, int iniTh, int minTh, int nthreads, int iters, long long* total_kps) {
    if (nthreads < 1) nthreads = 1;
    std::vector<Img> imgs(nframes);
    for (int f = 0; f < nframes; f++) {
        imgs[f].create(w, h);
        std::memcpy(imgs[f].d.data(), frames + (size_t)f * w * h, (size_t)w * h);
    }
    std::atomic<long long> kps{0};
    std::atomic<int> next{0};
    const int total = nframes * iters;
    auto t0 = std::chrono::steady_clock::now();
    auto worker = [&]() {
        Extractor e(nfeatures, scaleFactor, nlevels, iniTh, minTh, 0);   // one instance per thread
        for (;;) {
            int k = next.fetch_add(1);
            if (k >= total) break;
            int n = e.run(imgs[k % nframes]);
            if (k < nframes) kps += n;
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) th.emplace_back(worker);
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    if (total_kps) *total_kps = kps.load();
    return std::chrono::duration<double>(t1 - t0).count();
}

/* ---- CPU baseline protocol: single thread, warm-up then individually timed frames
 * (per-frame ms and per-stage ms out), and frame-parallel over nthreads (one extractor per thread,
 * `warmup` frames each before the clock starts, then `total` frames from a shared counter). ---- */
int oracle_bench_single(const uint8_t* frames, int nframes, int w, int h, int nfeatures, int warmup, int timed,
                        double* frame_ms, double* stage_ms6, long long* total_kps) {
    std::vector<Img> imgs(nframes);
    for (int f = 0; f < nframes; f++) {
        imgs[f].create(w, h);
        std::memcpy(imgs[f].d.data(), frames + (size_t)f * w * h, (size_t)w * h);
    }
    Extractor e(nfeatures, 1.2f, 8, 20, 7, 0);
    for (int i = 0; i < warmup; i++) e.run(imgs[i % nframes]);
    for (double& v : e.stage_ms) v = 0;
    long long kps = 0;
    for (int i = 0; i < timed; i++) {
        auto t0 = std::chrono::steady_clock::now();
        const int n = e.run(imgs[(warmup + i) % nframes]);
        frame_ms[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        kps += n > 0 ? n : 0;
    }
    for (int k = 0; k < 6; k++) stage_ms6[k] = e.stage_ms[k];
    if (total_kps) *total_kps = kps;
    return 0;
}

double oracle_bench_parallel(const uint8_t* frames, int nframes, int w, int h, int nfeatures, int nthreads, int warmup,
                             int total, long long* total_kps) {
    if (nthreads < 1) nthreads = 1;
    std::vector<Img> imgs(nframes);
    for (int f = 0; f < nframes; f++) {
        imgs[f].create(w, h);
        std::memcpy(imgs[f].d.data(), frames + (size_t)f * w * h, (size_t)w * h);
    }
    std::atomic<long long> kps{0};
    std::atomic<int> next{0}, ready{0};
    std::atomic<bool> go{false};
    auto worker = [&](int tid) {
        Extractor e(nfeatures, 1.2f, 8, 20, 7, 0);   // one instance per thread (ORBextractor.h:85)
        for (int i = 0; i < warmup; i++) e.run(imgs[(tid + i) % nframes]);
        ready++;
        while (!go.load()) std::this_thread::yield();
        for (;;) {
            const int k = next.fetch_add(1);
            if (k >= total) break;
            const int n = e.run(imgs[k % nframes]);
            kps += n > 0 ? n : 0;
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) th.emplace_back(worker, t);
    while (ready.load() < nthreads) std::this_thread::yield();
    auto t0 = std::chrono::steady_clock::now();
    go = true;
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    if (total_kps) *total_kps = kps.load();
    return std::chrono::duration<double>(t1 - t0).count();
}

/* Hamming CPU baseline: for each (query frame, train frame) pair, either ORBmatcher::SearchByBoW(KF, F)
 * with one FeatureVector node holding every feature (the C4 brute-force semantics, SURVEY §8(d):
 * nnratio 0.7, checkOri on, all MapPoints valid; ORBmatcher.cc:159-288) or the plain all-pairs top-2
 * DescriptorDistance loop the GPU kernel computes (mode 1).  Pairs are spread over nthreads; `iters`
 * passes.  Returns wall seconds; *evals = sum of nq * nt over one pass. */
double oracle_bench_hamming(const uint8_t* desc, const float* angles, const int* counts, int stride, int npairs,
                            const int* qf, const int* tf, int mode, int nthreads, int iters, long long* evals) {
    if (nthreads < 1) nthreads = 1;
    long long ev = 0;
    for (int p = 0; p < npairs; p++) ev += (long long)counts[qf[p]] * counts[tf[p]];
    if (evals) *evals = ev;
    std::atomic<int> next{0};
    std::atomic<long long> sink{0};
    const int total = npairs * iters;
    auto worker = [&]() {
        std::vector<int> idxq, idxt, match, best(1), second(1);
        long long local = 0;
        for (;;) {
            const int k = next.fetch_add(1);
            if (k >= total) break;
            const int p = k % npairs;
            const int nq = counts[qf[p]], nt = counts[tf[p]];
            const uint8_t* dq = desc + (size_t)qf[p] * stride * 32;
            const uint8_t* dt = desc + (size_t)tf[p] * stride * 32;
            if (mode == 0) {
                idxq.resize(nq);
                idxt.resize(nt);
                for (int i = 0; i < nq; i++) idxq[i] = i;
                for (int i = 0; i < nt; i++) idxt[i] = i;
                std::vector<uint8_t> mp(nq, 1);
                const uint32_t node = 0;
                const int offq[2] = {0, nq}, offt[2] = {0, nt};
                OracleFeatVec fq{1, &node, offq, idxq.data()}, ft{1, &node, offt, idxt.data()};
                match.resize(std::max(nt, 1));
                local += oracle_search_by_bow_kf_f(0.7f, 1, nq, dq, angles + (size_t)qf[p] * stride, mp.data(), fq, nt, dt,
                                                   angles + (size_t)tf[p] * stride, ft, match.data());
            } else {
                for (int i = 0; i < nq; i++) {
                    int b1 = 256, b2 = 256, bi = -1;
                    for (int j = 0; j < nt; j++) {
                        const int d = DescriptorDistance(dq + (size_t)i * 32, dt + (size_t)j * 32);
                        if (d < b1) { b2 = b1; b1 = d; bi = j; }
                        else if (d < b2) b2 = d;
                    }
                    local += bi + b2;
                }
            }
        }
        sink += local;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) th.emplace_back(worker);
    for (auto& t : th) t.join();
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count() + (sink.load() == -1 ? 1 : 0);
}

/* SearchByBoW(KF, F)  ORBmatcher.cc:159-288 */
int oracle_search_by_bow_kf_f(float nnratio, int checkOri, int n_kf, const uint8_t* desc_kf, const float* angle_kf,
                              const uint8_t* mp_kf, OracleFeatVec fv_kf, int n_f, const uint8_t* desc_f,
                              const float* angle_f, OracleFeatVec fv_f, int* match_f) {
    (void)n_kf;
    std::vector<int> matches(n_f, -1);
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    for_common_nodes(fv_kf, fv_f, [&](int a, int b) {
        for (int iKF = fv_kf.offsets[a]; iKF < fv_kf.offsets[a + 1]; iKF++) {
            const int realIdxKF = fv_kf.indices[iKF];
            if (!mp_kf[realIdxKF]) continue;
            const uint8_t* dKF = desc_kf + (size_t)realIdxKF * 32;
            int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
            for (int iF = fv_f.offsets[b]; iF < fv_f.offsets[b + 1]; iF++) {
                const int realIdxF = fv_f.indices[iF];
                if (matches[realIdxF] >= 0) continue;
                const int dist = DescriptorDistance(dKF, desc_f + (size_t)realIdxF * 32);
                if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF; }
                else if (dist < bestDist2) bestDist2 = dist;
            }
            if (bestDist1 <= TH_LOW) {
                if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                    matches[bestIdxF] = realIdxKF;
                    if (checkOri) rotHist[rot_bin(angle_kf[realIdxKF], angle_f[bestIdxF])].push_back(bestIdxF);
                    nmatches++;
                }
            }
        }
    });
    if (checkOri) cull_rotation(rotHist, matches, nmatches);
    std::memcpy(match_f, matches.data(), n_f * sizeof(int));
    return nmatches;
}

/* SearchByBoW(KF1, KF2)  ORBmatcher.cc:522-655 */
int oracle_search_by_bow_kf_kf(float nnratio, int checkOri, int n1, const uint8_t* desc1, const float* angle1,
                               const uint8_t* mp1, OracleFeatVec fv1, int n2, const uint8_t* desc2,
                               const float* angle2, const uint8_t* mp2, OracleFeatVec fv2, int* match12) {
    std::vector<int> matches(n1, -1);
    std::vector<char> vbMatched2(n2, 0);
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    for_common_nodes(fv1, fv2, [&](int a, int b) {
        for (int i1 = fv1.offsets[a]; i1 < fv1.offsets[a + 1]; i1++) {
            const int idx1 = fv1.indices[i1];
            if (!mp1[idx1]) continue;
            const uint8_t* d1 = desc1 + (size_t)idx1 * 32;
            int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
            for (int i2 = fv2.offsets[b]; i2 < fv2.offsets[b + 1]; i2++) {
                const int idx2 = fv2.indices[i2];
                if (vbMatched2[idx2] || !mp2[idx2]) continue;
                int dist = DescriptorDistance(d1, desc2 + (size_t)idx2 * 32);
                if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = idx2; }
                else if (dist < bestDist2) bestDist2 = dist;
            }
            if (bestDist1 < TH_LOW) {
                if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                    matches[idx1] = bestIdx2;
                    vbMatched2[bestIdx2] = 1;
                    if (checkOri) rotHist[rot_bin(angle1[idx1], angle2[bestIdx2])].push_back(idx1);
                    nmatches++;
                }
            }
        }
    });
    if (checkOri) cull_rotation(rotHist, matches, nmatches);
    std::memcpy(match12, matches.data(), n1 * sizeof(int));
    return nmatches;
}

/* SearchForTriangulation  ORBmatcher.cc:657-823 */
int oracle_search_for_triangulation(int checkOri, int onlyStereo, int n1, const uint8_t* desc1,
                                    const OracleKeyPoint* kps1_, const uint8_t* has_mp1, const float* uright1,
                                    OracleFeatVec fv1, int n2, const uint8_t* desc2, const OracleKeyPoint* kps2_,
                                    const uint8_t* has_mp2, const float* uright2, OracleFeatVec fv2, const float* F12,
                                    float ex, float ey, const float* scaleFactors2, const float* levelSigma2_2,
                                    int* pairs_out, int cap) {
    const KP* kps1 = (const KP*)kps1_;
    const KP* kps2 = (const KP*)kps2_;
    std::vector<char> vbMatched2(n2, 0);   // never set in the reference (:738): kept for fidelity
    std::vector<int> vMatches12(n1, -1);
    int nmatches = 0;
    std::vector<int> rotHist[HISTO_LENGTH];
    for_common_nodes(fv1, fv2, [&](int a, int b) {
        for (int i1 = fv1.offsets[a]; i1 < fv1.offsets[a + 1]; i1++) {
            const int idx1 = fv1.indices[i1];
            if (has_mp1[idx1]) continue;
            const bool bStereo1 = uright1[idx1] >= 0;
            if (onlyStereo && !bStereo1) continue;
            const KP& kp1 = kps1[idx1];
            const uint8_t* d1 = desc1 + (size_t)idx1 * 32;
            int bestDist = TH_LOW, bestIdx2 = -1;
            for (int i2 = fv2.offsets[b]; i2 < fv2.offsets[b + 1]; i2++) {
                const int idx2 = fv2.indices[i2];
                if (vbMatched2[idx2] || has_mp2[idx2]) continue;
                const bool bStereo2 = uright2[idx2] >= 0;
                if (onlyStereo && !bStereo2) continue;
                const int dist = DescriptorDistance(d1, desc2 + (size_t)idx2 * 32);
                if (dist > TH_LOW || dist > bestDist) continue;
                const KP& kp2 = kps2[idx2];
                if (!bStereo1 && !bStereo2) {
                    const float distex = ex - kp2.x;
                    const float distey = ey - kp2.y;
                    if (std::fmaf(distex, distex, distey * distey) < 100 * scaleFactors2[kp2.octave]) continue;   // contracted, as above
                }
                if (CheckDistEpipolarLine(kp1, kp2, F12, levelSigma2_2)) { bestIdx2 = idx2; bestDist = dist; }
            }
            if (bestIdx2 >= 0) {
                const KP& kp2 = kps2[bestIdx2];
                vMatches12[idx1] = bestIdx2;
                nmatches++;
                if (checkOri) rotHist[rot_bin(kp1.angle, kp2.angle)].push_back(idx1);
            }
        }
    });
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ComputeThreeMaxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (size_t j = 0; j < rotHist[i].size(); j++) { vMatches12[rotHist[i][j]] = -1; nmatches--; }
        }
    }
    int np = 0;
    for (int i = 0; i < n1; i++) {
        if (vMatches12[i] < 0) continue;
        if (np < cap) { pairs_out[2 * np] = i; pairs_out[2 * np + 1] = vMatches12[i]; }
        np++;
    }
    return np;
}

/* SearchForInitialization (:405-520) / BirdviewMatch(const Frame&,...) (:1790-1899) */
int oracle_window_match(float nnratio, int checkOri, int level0_only, int n1, const uint8_t* desc1,
                        const OracleKeyPoint* kps1_, int n2, const uint8_t* desc2, const OracleKeyPoint* kps2_,
                        const int* cand_off, const int* cand_idx, int* match12) {
    const KP* kps1 = (const KP*)kps1_;
    const KP* kps2 = (const KP*)kps2_;
    int nmatches = 0;
    std::vector<int> vnMatches12(n1, -1);
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<int> vMatchedDistance(n2, INT_MAX);
    std::vector<int> vnMatches21(n2, -1);
    for (int i1 = 0; i1 < n1; i1++) {
        const KP kp1 = kps1[i1];
        if (level0_only && kp1.octave > 0) continue;
        if (cand_off[i1 + 1] == cand_off[i1]) continue;
        const uint8_t* d1 = desc1 + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int c = cand_off[i1]; c < cand_off[i1 + 1]; c++) {
            const int i2 = cand_idx[c];
            int dist = DescriptorDistance(d1, desc2 + (size_t)i2 * 32);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) { vnMatches12[vnMatches21[bestIdx2]] = -1; nmatches--; }
                vnMatches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) rotHist[rot_bin(kps1[i1].angle, kps2[bestIdx2].angle)].push_back(i1);
            }
        }
    }
    if (checkOri) cull_rotation(rotHist, vnMatches12, nmatches);
    std::memcpy(match12, vnMatches12.data(), n1 * sizeof(int));
    return nmatches;
}

/* Frame::GetFeaturesInArea  Frame.cc:494-547 over the grid of Frame.cc:378-392, 549-560 */
int oracle_features_in_area(int n, const OracleKeyPoint* kpsUn_, float mnMinX, float mnMaxX, float mnMinY,
                            float mnMaxY, float x, float y, float r, int minLevel, int maxLevel, int* out, int cap) {
    const KP* kpsUn = (const KP*)kpsUn_;
    const int COLS = 64, ROWS = 48;   // Frame.h:39-40
    const float gw = static_cast<float>(COLS) / static_cast<float>(mnMaxX - mnMinX);
    const float gh = static_cast<float>(ROWS) / static_cast<float>(mnMaxY - mnMinY);
    std::vector<std::vector<int>> grid((size_t)COLS * ROWS);
    for (int i = 0; i < n; i++) {
        int px = (int)std::round((kpsUn[i].x - mnMinX) * gw);
        int py = (int)std::round((kpsUn[i].y - mnMinY) * gh);
        if (px < 0 || px >= COLS || py < 0 || py >= ROWS) continue;
        grid[(size_t)px * ROWS + py].push_back(i);
    }
    std::vector<int> v;
    const int nMinCellX = std::max(0, (int)std::floor((x - mnMinX - r) * gw));
    const int nMaxCellX = std::min(COLS - 1, (int)std::ceil((x - mnMinX + r) * gw));
    const int nMinCellY = std::max(0, (int)std::floor((y - mnMinY - r) * gh));
    const int nMaxCellY = std::min(ROWS - 1, (int)std::ceil((y - mnMinY + r) * gh));
    if (nMinCellX < COLS && nMaxCellX >= 0 && nMinCellY < ROWS && nMaxCellY >= 0) {
        const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
                for (int idx : grid[(size_t)ix * ROWS + iy]) {
                    const KP& kpUn = kpsUn[idx];
                    if (bCheckLevels) {
                        if (kpUn.octave < minLevel) continue;
                        if (maxLevel >= 0 && kpUn.octave > maxLevel) continue;
                    }
                    const float distx = kpUn.x - x, disty = kpUn.y - y;
                    if (std::fabs(distx) < r && std::fabs(disty) < r) v.push_back(idx);
                }
    }
    if ((int)v.size() > cap) return -(int)v.size() - 1;
    std::memcpy(out, v.data(), v.size() * sizeof(int));
    return (int)v.size();
}

/* Frame::ComputeStereoMatches  Frame.cc:662-836.  left/right: oracle extractors that ran on the
 * rectified left/right images (their pyramids are mpORBextractorLeft/Right->mvImagePyramid);
 * kpsL/descL = mvKeys/mDescriptors, kpsR/descR = mvKeysRight/mDescriptorsRight; scale tables of
 * the left extractor (Frame copies them, Frame.cc:104-109).  Writes mvuRight / mvDepth (N each). */
int oracle_stereo_matches(void* left, void* right, int N, const OracleKeyPoint* kpsL_, const uint8_t* descL, int Nr,
                          const OracleKeyPoint* kpsR_, const uint8_t* descR, float mb, float mbf, float* mvuRight,
                          float* mvDepth) {
    const Extractor* eL = (const Extractor*)left;
    const Extractor* eR = (const Extractor*)right;
    const KP* mvKeys = (const KP*)kpsL_;
    const KP* mvKeysRight = (const KP*)kpsR_;
    const std::vector<float>& mvScaleFactors = eL->mvScaleFactor;
    const std::vector<float>& mvInvScaleFactors = eL->mvInvScaleFactor;
    for (int i = 0; i < N; i++) {   // :664-665
        mvuRight[i] = -1.0f;
        mvDepth[i] = -1.0f;
    }
    const int TH_HIGH = 100;
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;   // :667
    const int nRows = eL->pyr[0].h;                  // :669
    std::vector<std::vector<size_t>> vRowIndices(nRows, std::vector<size_t>());
    for (int iR = 0; iR < Nr; iR++) {   // :678-689
        const KP& kp = mvKeysRight[iR];
        const float& kpY = kp.y;
        const float r = 2.0f * mvScaleFactors[mvKeysRight[iR].octave];
        const int maxr = (int)std::ceil(kpY + r);
        const int minr = (int)std::floor(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) vRowIndices[yi].push_back(iR);   // (reference indexes unchecked)
    }
    const float minZ = mb;   // :692-694
    const float minD = 0;
    const float maxD = mbf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    vDistIdx.reserve(N);
    for (int iL = 0; iL < N; iL++) {
        const KP& kpL = mvKeys[iL];
        const int& levelL = kpL.octave;
        const float& vL = kpL.y;
        const float& uL = kpL.x;
        const std::vector<size_t>& vCandidates = vRowIndices[(size_t)vL];   // :707 float index, truncated
        if (vCandidates.empty()) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        size_t bestIdxR = 0;
        const uint8_t* dL = descL + (size_t)iL * 32;
        for (size_t iC = 0; iC < vCandidates.size(); iC++) {   // :724-745
            const size_t iR = vCandidates[iC];
            const KP& kpR = mvKeysRight[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float& uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = DescriptorDistance(dL, descR + iR * 32);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {   // :748-834
            const float uR0 = mvKeysRight[bestIdxR].x;
            const float scaleFactor = mvInvScaleFactors[kpL.octave];
            const float scaleduL = std::round(kpL.x * scaleFactor);
            const float scaledvL = std::round(kpL.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5;
            const Img& PL = eL->pyr[kpL.octave];
            const Img& PR = eR->pyr[kpL.octave];
            const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
            const float cL = (float)PL.row(yl0 + w)[xl0 + w];
            int bestDist2 = INT_MAX;
            int bestincR = 0;
            const int L = 5;
            float vDists[2 * L + 1];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= PR.w) continue;
            for (int incR = -L; incR <= +L; incR++) {
                const int xr0 = (int)scaleduR0 + incR - w;
                const float cR = (float)PR.row(yl0 + w)[xr0 + w];
                // cv::norm(IL, IR, NORM_L1) on centred float patches: exact integer sum (|values| <= 510)
                double acc = 0;
                for (int yy = 0; yy < 2 * w + 1; yy++)
                    for (int xx = 0; xx < 2 * w + 1; xx++) {
                        const float a = (float)PL.row(yl0 + yy)[xl0 + xx] - cL;
                        const float b = (float)PR.row(yl0 + yy)[xr0 + xx] - cR;
                        acc += std::fabs((double)(a - b));
                    }
                const float dist = (float)acc;
                if (dist < bestDist2) {
                    bestDist2 = (int)dist;
                    bestincR = incR;
                }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1];
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = mvScaleFactors[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01;
                    bestuR = uL - 0.01;
                }
                mvDepth[iL] = mbf / disparity;
                mvuRight[iL] = bestuR;
                vDistIdx.push_back(std::pair<int, int>(bestDist2, iL));
            }
        }
    }
    if (vDistIdx.empty()) return 0;   // (the reference reads vDistIdx[0] of an empty vector: UB)
    std::sort(vDistIdx.begin(), vDistIdx.end());   // :822-835
    const float median = vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    int nvalid = (int)vDistIdx.size();
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist) break;
        mvuRight[vDistIdx[i].second] = -1;
        mvDepth[vDistIdx[i].second] = -1;
        nvalid--;
    }
    return nvalid;
}

/* ---------------- DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary.h:32) ----------------
 * loadFromBinaryFile  Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1466-1510 (including its
 * while(!f.eof()) quirk: the last record is read twice, adding a duplicate last child that can never
 * win a strict '<' descent), transform(feature, ...)  :1240-1277, transform(features, BowVector&,
 * FeatureVector&, levelsup)  :1139-1210, BowVector::addWeight/addIfNotExist/normalize
 * (BowVector.cpp:34-86), FeatureVector::addFeature (FeatureVector.cpp:31-45). */
struct OVNode {
    int parent = 0;
    std::vector<int> children;
    uint8_t desc[32] = {0};
    double weight = 0;
    int word_id = -1;
    bool isLeaf() const { return children.empty(); }
};
struct OVocab {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<OVNode> nodes;
    int nwords = 0;
};

void* oracle_vocab_load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return nullptr;
    OVocab* v = new OVocab();
    unsigned int nb_nodes = 0, size_node = 0;
    if (fread(&nb_nodes, 4, 1, f) != 1 || fread(&size_node, 4, 1, f) != 1 || fread(&v->k, 4, 1, f) != 1 ||
        fread(&v->L, 4, 1, f) != 1 || fread(&v->scoring, 4, 1, f) != 1 || fread(&v->weighting, 4, 1, f) != 1 ||
        size_node != 41) {
        fclose(f);
        delete v;
        return nullptr;
    }
    v->nodes.resize(nb_nodes + 1);
    std::vector<char> buf(size_node, 0);
    int nid = 1;
    for (;;) {   // while (!f.eof()): a failed read leaves buf as it was and still creates a node
        const size_t got = fread(buf.data(), 1, size_node, f);
        if (nid >= (int)v->nodes.size()) break;
        OVNode& n = v->nodes[nid];
        std::memcpy(&n.parent, buf.data(), 4);
        v->nodes[n.parent].children.push_back(nid);
        std::memcpy(n.desc, buf.data() + 4, 32);
        float w;
        std::memcpy(&w, buf.data() + 36, 4);
        n.weight = w;
        if (buf[40]) n.word_id = v->nwords++;
        nid += 1;
        if (got < size_node) break;   // eof reached on this read: the loop ends after this node
    }
    fclose(f);
    return v;
}

void oracle_vocab_destroy(void* h) { delete (OVocab*)h; }

int oracle_vocab_info(void* h, int* k, int* L, int* scoring, int* weighting, int* nnodes, int* nwords) {
    const OVocab* v = (const OVocab*)h;
    *k = v->k;
    *L = v->L;
    *scoring = v->scoring;
    *weighting = v->weighting;
    *nnodes = (int)v->nodes.size();
    *nwords = v->nwords;
    return 0;
}

/* transform(feature, word_id, weight, nid, levelsup) for each of n descriptors. */
void oracle_vocab_transform_each(void* h, const uint8_t* desc, int n, int levelsup, int* word_id, double* weight,
                                 uint32_t* nid_out) {
    const OVocab* v = (const OVocab*)h;
    for (int i = 0; i < n; i++) {
        const uint8_t* feature = desc + (size_t)i * 32;
        const int nid_level = v->L - levelsup;
        uint32_t nid = 0;   // (uninitialised in the reference when a leaf comes before nid_level)
        if (nid_level <= 0) nid = 0;
        int final_id = 0;
        int current_level = 0;
        do {
            ++current_level;
            const std::vector<int>& nodes = v->nodes[final_id].children;
            final_id = nodes[0];
            double best_d = DescriptorDistance(feature, v->nodes[final_id].desc);
            for (size_t c = 1; c < nodes.size(); c++) {
                const int id = nodes[c];
                const double d = DescriptorDistance(feature, v->nodes[id].desc);
                if (d < best_d) {
                    best_d = d;
                    final_id = id;
                }
            }
            if (current_level == nid_level) nid = (uint32_t)final_id;
        } while (!v->nodes[final_id].isLeaf());
        word_id[i] = v->nodes[final_id].word_id;
        weight[i] = v->nodes[final_id].weight;
        nid_out[i] = nid;
    }
}

/* transform(features, BowVector&, FeatureVector&, levelsup).  BowVector out: nbow (word, value)
 * pairs ascending by word; FeatureVector out: nfv nodes ascending, fv_off (nfv+1) / fv_idx CSR.
 * Returns 0, or -1 if a capacity is too small (caps: n each). */
int oracle_vocab_transform(void* h, const uint8_t* desc, int n, int levelsup, int* bow_words, double* bow_values,
                           int* nbow, uint32_t* fv_nodes, int* fv_off, int* fv_idx, int* nfv) {
    const OVocab* v = (const OVocab*)h;
    std::map<int, double> bow;
    std::map<uint32_t, std::vector<int>> fv;
    if (v->nwords > 0) {   // if(empty()) return;  TemplatedVocabulary.h:1146-1149
        // scoring -> (must normalise, norm): L1, L2, ChiSquare, KL, Bhattacharyya: true; DotProduct: false
        const bool must = v->scoring != 5;
        const bool l1 = v->scoring != 1;
        std::vector<int> wid(n);
        std::vector<double> w(n);
        std::vector<uint32_t> nid(n);
        oracle_vocab_transform_each(h, desc, n, levelsup, wid.data(), w.data(), nid.data());
        const bool tf = v->weighting == 0 || v->weighting == 1;   // TF_IDF, TF
        for (int i = 0; i < n; i++) {
            if (w[i] > 0) {
                if (tf) bow[wid[i]] += w[i];                       // addWeight
                else if (!bow.count(wid[i])) bow[wid[i]] = w[i];   // addIfNotExist
                fv[nid[i]].push_back(i);
            }
        }
        if (tf && !bow.empty() && !must) {
            const double nd = (double)bow.size();
            for (auto& e : bow) e.second /= nd;
        }
        if (must) {   // BowVector::normalize
            double norm = 0.0;
            if (l1)
                for (auto& e : bow) norm += std::fabs(e.second);
            else {
                for (auto& e : bow) norm += e.second * e.second;
                norm = std::sqrt(norm);
            }
            if (norm > 0.0)
                for (auto& e : bow) e.second /= norm;
        }
    }
    int b = 0;
    for (auto& e : bow) {
        bow_words[b] = e.first;
        bow_values[b] = e.second;
        b++;
    }
    *nbow = b;
    int j = 0, o = 0;
    fv_off[0] = 0;
    for (auto& e : fv) {
        fv_nodes[j] = e.first;
        for (int i : e.second) fv_idx[o++] = i;
        fv_off[++j] = o;
    }
    *nfv = j;
    return 0;
}

/* MapPoint::ComputeDistinctiveDescriptors  MapPoint.cc:242-307 (the distance / median part). */
int oracle_distinctive_descriptor(const uint8_t* desc, int N) {
    if (N <= 0) return -1;
    std::vector<float> Distances((size_t)N * N);
    for (int i = 0; i < N; i++) {
        Distances[(size_t)i * N + i] = 0;
        for (int j = i + 1; j < N; j++) {
            const int distij = DescriptorDistance(desc + (size_t)i * 32, desc + (size_t)j * 32);
            Distances[(size_t)i * N + j] = distij;
            Distances[(size_t)j * N + i] = distij;
        }
    }
    int BestMedian = INT_MAX;
    int BestIdx = 0;
    for (int i = 0; i < N; i++) {
        std::vector<int> vDists(Distances.begin() + (size_t)i * N, Distances.begin() + (size_t)(i + 1) * N);
        std::sort(vDists.begin(), vDists.end());
        const int median = vDists[(size_t)(0.5 * (N - 1))];
        if (median < BestMedian) {
            BestMedian = median;
            BestIdx = i;
        }
    }
    return BestIdx;
}

}  // extern "C"

#include "cvorb_oracle.inc"
