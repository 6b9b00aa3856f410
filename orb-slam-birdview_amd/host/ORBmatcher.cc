// ORB_SLAM2::ORBmatcher over liborbgpu (see ORBmatcher.h).  Marshals the Frame/KeyFrame members
// into the C-ABI's flat arrays; all descriptor distances are computed by the gfx950 kernels.
#include "ORBmatcher.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace ORBGPU_MATCHER_NAMESPACE {

const int ORBmatcher::TH_HIGH = 100;   // ORBmatcher.cc:37-39
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

namespace {

void check(int st, const char* what) {
    if (st != ORB_OK) throw OrbGpuError(st, what);
}

// Matchers are stack objects in the reference (one per call site, any thread): they share one
// context per (host thread, device), created on first use.
struct ThreadCtx {
    int device = -1;
    orb_ctx* ctx = nullptr;
    ~ThreadCtx() {
        if (ctx) orb_destroy(ctx);
    }
};

orb_ctx* matcher_ctx() {
    static thread_local ThreadCtx tc;
    const char* e = getenv("ORBGPU_DEVICE");
    const int dev = e ? atoi(e) : 0;
    if (tc.ctx && tc.device == dev) return tc.ctx;
    if (tc.ctx) orb_destroy(tc.ctx);
    tc.ctx = nullptr;
    orb_params p;
    memset(&p, 0, sizeof p);
    p.nfeatures = 1000;
    p.scaleFactor = 1.2f;
    p.nlevels = 8;
    p.iniThFAST = 20;
    p.minThFAST = 7;
    p.device = dev;
    int st = ORB_OK;
    tc.ctx = orb_create(&p, &st);
    if (!tc.ctx) throw OrbGpuError(st, "orb_create (matcher)");
    tc.device = dev;
    return tc.ctx;
}

// DBoW2::FeatureVector -> CSR over ascending node ids (std::map order = the reference's iteration order)
struct Csr {
    std::vector<uint32_t> ids;
    std::vector<int> off, idx;
    orb_featvec fv;
    explicit Csr(const FeatureVector* f) {
        off.push_back(0);
        if (f)
            for (FeatureVector::const_iterator it = f->begin(); it != f->end(); ++it) {
                ids.push_back(it->first);
                for (size_t j = 0; j < it->second.size(); j++) idx.push_back((int)it->second[j]);
                off.push_back((int)idx.size());
            }
        if (idx.empty()) idx.push_back(0);
        fv.nnodes = (int)ids.size();
        fv.node_ids = ids.empty() ? nullptr : ids.data();
        fv.offsets = off.data();
        fv.indices = idx.data();
    }
};

std::vector<float> angles(const FeatureSet& s) {
    std::vector<float> a(std::max(s.N(), 1), 0.f);
    for (int i = 0; i < s.N(); i++) a[i] = s.keys[i].angle;
    return a;
}

const uint8_t* desc_ptr(const FeatureSet& s) {
    static const uint8_t dummy[32] = {0};
    return (s.descriptors && s.N()) ? s.descriptors : dummy;
}

const KeyPoint* keys_ptr(const FeatureSet& s) {
    static const KeyPoint dummy = {0, 0, 0, 0, 0, 0, 0};
    return (s.keys && s.N()) ? s.keys : &dummy;
}

void require(bool ok, const char* what) {
    if (!ok) throw OrbGpuError(ORB_ERR_ARG, what);
}

std::vector<uint8_t> flags_or(const uint8_t* v, int n, uint8_t dflt) {
    return v ? std::vector<uint8_t>(v, v + n) : std::vector<uint8_t>(n, dflt);
}

std::vector<float> floats_or(const float* v, int n, float dflt) {
    return v ? std::vector<float>(v, v + n) : std::vector<float>(n, dflt);
}

}  // namespace

/* ---------------- Frame grid (Frame.cc:378-412, 494-560, 877-940) ---------------- */
FrameGrid::FrameGrid(const KeyPoint* keysUn, int n, float minX, float maxX, float minY, float maxY) {
    minX_ = minX;
    minY_ = minY;
    invW_ = static_cast<float>(ORBGPU_FRAME_GRID_COLS) / static_cast<float>(maxX - minX);   // Frame.cc:156-157
    invH_ = static_cast<float>(ORBGPU_FRAME_GRID_ROWS) / static_cast<float>(maxY - minY);
    assign(keysUn, n);
}

FrameGrid FrameGrid::Birdview(const KeyPoint* keysBird, int n, float widthInv, float heightInv) {
    FrameGrid g;
    g.invW_ = widthInv;
    g.invH_ = heightInv;
    g.assign(keysBird, n);
    return g;
}

void FrameGrid::assign(const KeyPoint* keys, int n) {
    keys_ = keys;
    cells_.assign((size_t)ORBGPU_FRAME_GRID_COLS * ORBGPU_FRAME_GRID_ROWS, std::vector<size_t>());
    for (int i = 0; i < n; i++) {
        // PosInGrid (Frame.cc:549-560): round((x - mnMinX) * inv)
        const int posX = (int)round((keys[i].x - minX_) * invW_);
        const int posY = (int)round((keys[i].y - minY_) * invH_);
        if (posX < 0 || posX >= ORBGPU_FRAME_GRID_COLS || posY < 0 || posY >= ORBGPU_FRAME_GRID_ROWS) continue;
        cells_[(size_t)posX * ORBGPU_FRAME_GRID_ROWS + posY].push_back(i);
    }
}

std::vector<size_t> FrameGrid::GetFeaturesInArea(float x, float y, float r, int minLevel, int maxLevel) const {
    std::vector<size_t> vIndices;
    if (cells_.empty()) return vIndices;
    const int nMinCellX = std::max(0, (int)floor((x - minX_ - r) * invW_));
    if (nMinCellX >= ORBGPU_FRAME_GRID_COLS) return vIndices;
    const int nMaxCellX = std::min((int)ORBGPU_FRAME_GRID_COLS - 1, (int)ceil((x - minX_ + r) * invW_));
    if (nMaxCellX < 0) return vIndices;
    const int nMinCellY = std::max(0, (int)floor((y - minY_ - r) * invH_));
    if (nMinCellY >= ORBGPU_FRAME_GRID_ROWS) return vIndices;
    const int nMaxCellY = std::min((int)ORBGPU_FRAME_GRID_ROWS - 1, (int)ceil((y - minY_ + r) * invH_));
    if (nMaxCellY < 0) return vIndices;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const std::vector<size_t>& vCell = cells_[(size_t)ix * ORBGPU_FRAME_GRID_ROWS + iy];
            for (size_t j = 0; j < vCell.size(); j++) {
                const KeyPoint& kp = keys_[vCell[j]];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (fabs(distx) < r && fabs(disty) < r) vIndices.push_back(vCell[j]);
            }
        }
    return vIndices;
}

/* ---------------- ORBmatcher ---------------- */
ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orb_descriptor_distance(a, b); }

int ORBmatcher::SearchByBoW(const KeyFrameData& KF, const FrameData& F, std::vector<int>& vpMapPointMatches) {
    const int nKF = KF.N(), nF = F.N();
    vpMapPointMatches.assign(nF, -1);   // :163 vector<MapPoint*>(F.N, NULL)
    Csr a(KF.featVec), b(F.featVec);
    require(nKF == 0 || (KF.keys && KF.descriptors), "SearchByBoW: KF keys/descriptors");
    require(nF == 0 || (F.keys && F.descriptors), "SearchByBoW: F keys/descriptors");
    std::vector<float> angKF = angles(KF), angF = angles(F);
    std::vector<uint8_t> mp = flags_or(KF.hasMapPoint, std::max(nKF, 1), 1);
    std::vector<int> out(std::max(nF, 1), -1);
    int nmatches = 0;
    check(orb_search_by_bow_kf_f(matcher_ctx(), mfNNratio, mbCheckOrientation, nKF, desc_ptr(KF), angKF.data(),
                                 mp.data(), a.fv, nF, desc_ptr(F), angF.data(), b.fv, out.data(), &nmatches),
          "SearchByBoW(KF,F)");
    std::copy(out.begin(), out.begin() + nF, vpMapPointMatches.begin());
    return nmatches;
}

int ORBmatcher::SearchByBoW(const KeyFrameData& KF1, const KeyFrameData& KF2, std::vector<int>& vpMatches12) {
    const int n1 = KF1.N(), n2 = KF2.N();
    vpMatches12.assign(n1, -1);   // :535
    Csr a(KF1.featVec), b(KF2.featVec);
    require(n1 == 0 || (KF1.keys && KF1.descriptors), "SearchByBoW: KF1 keys/descriptors");
    require(n2 == 0 || (KF2.keys && KF2.descriptors), "SearchByBoW: KF2 keys/descriptors");
    std::vector<float> ang1 = angles(KF1), ang2 = angles(KF2);
    std::vector<uint8_t> mp1 = flags_or(KF1.hasMapPoint, std::max(n1, 1), 1),
                         mp2 = flags_or(KF2.hasMapPoint, std::max(n2, 1), 1);
    std::vector<int> out(std::max(n1, 1), -1);
    int nmatches = 0;
    check(orb_search_by_bow_kf_kf(matcher_ctx(), mfNNratio, mbCheckOrientation, n1, desc_ptr(KF1), ang1.data(),
                                  mp1.data(), a.fv, n2, desc_ptr(KF2), ang2.data(), mp2.data(), b.fv, out.data(),
                                  &nmatches),
          "SearchByBoW(KF,KF)");
    std::copy(out.begin(), out.begin() + n1, vpMatches12.begin());
    return nmatches;
}

int ORBmatcher::SearchForTriangulation(const KeyFrameData& KF1, const KeyFrameData& KF2, const float F12[9], float ex,
                                       float ey, std::vector<std::pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo) {
    const int n1 = KF1.N(), n2 = KF2.N();
    Csr a(KF1.featVec), b(KF2.featVec);
    require(n1 == 0 || (KF1.keys && KF1.descriptors), "SearchForTriangulation: KF1 keys/descriptors");
    require(n2 == 0 || (KF2.keys && KF2.descriptors), "SearchForTriangulation: KF2 keys/descriptors");
    require(KF2.scaleFactors && KF2.levelSigma2 && KF2.nlevels > 0, "SearchForTriangulation: KF2 scale tables");
    std::vector<uint8_t> mp1 = flags_or(KF1.hasMapPoint, std::max(n1, 1), 0),
                         mp2 = flags_or(KF2.hasMapPoint, std::max(n2, 1), 0);
    std::vector<float> ur1 = floats_or(KF1.uRight, std::max(n1, 1), -1.f), ur2 = floats_or(KF2.uRight, std::max(n2, 1), -1.f);
    std::vector<int> pairs(2 * (size_t)std::max(n1, 1));
    int np = 0;
    check(orb_search_for_triangulation(matcher_ctx(), mbCheckOrientation, bOnlyStereo, n1, desc_ptr(KF1), keys_ptr(KF1),
                                       mp1.data(), ur1.data(), a.fv, n2, desc_ptr(KF2), keys_ptr(KF2), mp2.data(),
                                       ur2.data(), b.fv, F12, ex, ey, KF2.scaleFactors, KF2.levelSigma2,
                                       KF2.nlevels, pairs.data(),
                                       std::max(n1, 1), &np),
          "SearchForTriangulation");
    vMatchedPairs.clear();   // :813-820
    vMatchedPairs.reserve(np);
    for (int i = 0; i < np; i++) vMatchedPairs.push_back(std::make_pair((size_t)pairs[2 * i], (size_t)pairs[2 * i + 1]));
    return np;
}

int ORBmatcher::SearchForTriangulation(const KeyFrameData& KF1, const std::vector<TriangulationNeighbour>& neighbours,
                                       std::vector<std::vector<std::pair<size_t, size_t> > >& vvMatchedPairs,
                                       const bool bOnlyStereo) {
    const int n1 = KF1.N(), np = (int)neighbours.size();
    require(n1 == 0 || (KF1.keys && KF1.descriptors), "SearchForTriangulation: KF1 keys/descriptors");
    Csr a(KF1.featVec);
    std::vector<uint8_t> mp1 = flags_or(KF1.hasMapPoint, std::max(n1, 1), 0);
    std::vector<float> ur1 = floats_or(KF1.uRight, std::max(n1, 1), -1.f);
    struct Side {   // one neighbour's views, alive until the call returns
        std::vector<uint8_t> mp;
        std::vector<float> ur;
        std::vector<int> pairs;
        int n = 0;
    };
    std::vector<Side> side(np);
    std::vector<Csr> csr;
    csr.reserve(np);
    std::vector<orb_tri_pair> P(np);
    for (int p = 0; p < np; p++) {
        require(neighbours[p].KF2 != nullptr, "SearchForTriangulation: neighbour KeyFrame");
        const KeyFrameData& KF2 = *neighbours[p].KF2;
        const int n2 = KF2.N();
        require(n2 == 0 || (KF2.keys && KF2.descriptors), "SearchForTriangulation: KF2 keys/descriptors");
        require(KF2.scaleFactors && KF2.levelSigma2 && KF2.nlevels > 0, "SearchForTriangulation: KF2 scale tables");
        Side& sd = side[p];
        sd.mp = flags_or(KF2.hasMapPoint, std::max(n2, 1), 0);
        sd.ur = floats_or(KF2.uRight, std::max(n2, 1), -1.f);
        sd.pairs.resize(2 * (size_t)std::max(n1, 1));
        csr.emplace_back(KF2.featVec);
        P[p] = orb_tri_pair{n2, desc_ptr(KF2), keys_ptr(KF2), sd.mp.data(), sd.ur.data(), csr.back().fv,
                            neighbours[p].F12, neighbours[p].ex, neighbours[p].ey, KF2.scaleFactors, KF2.levelSigma2,
                            KF2.nlevels, sd.pairs.data(), std::max(n1, 1), &sd.n};
    }
    check(orb_search_for_triangulation_batch(matcher_ctx(), mbCheckOrientation, bOnlyStereo, n1, desc_ptr(KF1),
                                             keys_ptr(KF1), mp1.data(), ur1.data(), a.fv, np, P.data()),
          "SearchForTriangulation(batch)");
    vvMatchedPairs.assign(np, std::vector<std::pair<size_t, size_t> >());
    int total = 0;
    for (int p = 0; p < np; p++) {
        for (int i = 0; i < side[p].n; i++)
            vvMatchedPairs[p].push_back(std::make_pair((size_t)side[p].pairs[2 * i], (size_t)side[p].pairs[2 * i + 1]));
        total += side[p].n;
    }
    return total;
}

int ORBmatcher::window_match(bool level0_only, const FeatureSet& F1, const FeatureSet& F2,
                             const std::vector<Point2f>* centres, int windowSize, std::vector<int>& vnMatches12) {
    const int n1 = F1.N(), n2 = F2.N();
    vnMatches12.assign(n1, -1);
    require(F2.grid != nullptr, "window match: F2 grid");
    require(n1 == 0 || (F1.keys && F1.descriptors), "window match: F1 keys/descriptors");
    require(n2 == 0 || (F2.keys && F2.descriptors), "window match: F2 keys/descriptors");
    // candidate lists: F2.GetFeaturesInArea(centre, windowSize, level1, level1) per query (:425, :1686, :1806)
    std::vector<int> off(n1 + 1, 0), idx;
    for (int i1 = 0; i1 < n1; i1++) {
        const KeyPoint& kp1 = F1.keys[i1];
        if (!(level0_only && kp1.octave > 0)) {
            const float x = centres ? (*centres)[i1].x : kp1.x, y = centres ? (*centres)[i1].y : kp1.y;
            const std::vector<size_t> v = F2.grid->GetFeaturesInArea(x, y, (float)windowSize, kp1.octave, kp1.octave);
            for (size_t j = 0; j < v.size(); j++) idx.push_back((int)v[j]);
        }
        off[i1 + 1] = (int)idx.size();
    }
    if (idx.empty()) idx.push_back(0);
    std::vector<int> out(std::max(n1, 1), -1);
    int nmatches = 0;
    check(orb_window_match(matcher_ctx(), mfNNratio, mbCheckOrientation, level0_only, n1, desc_ptr(F1), keys_ptr(F1),
                           n2, desc_ptr(F2), keys_ptr(F2), off.data(), idx.data(), out.data(), &nmatches),
          "window match");
    std::copy(out.begin(), out.begin() + n1, vnMatches12.begin());
    return nmatches;
}

int ORBmatcher::SearchForInitialization(const FrameData& F1, const FrameData& F2, std::vector<Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
    const int n = window_match(true, F1, F2, &vbPrevMatched, windowSize, vnMatches12);
    for (size_t i1 = 0; i1 < vnMatches12.size(); i1++)   // :514-517 update prev matched
        if (vnMatches12[i1] >= 0) {
            const KeyPoint& k = F2.keys[vnMatches12[i1]];
            vbPrevMatched[i1].x = k.x;
            vbPrevMatched[i1].y = k.y;
        }
    return n;
}

int ORBmatcher::BirdviewMatch(const FrameData& F1, const FrameData& F2, std::vector<int>& vnMatches12,
                              std::vector<Point2f>& vPrevMatched, int windowSize) {
    const int n = window_match(true, F1, F2, &vPrevMatched, windowSize, vnMatches12);
    for (size_t i1 = 0; i1 < vnMatches12.size(); i1++)   // :1778-1781
        if (vnMatches12[i1] >= 0) {
            const KeyPoint& k = F2.keys[vnMatches12[i1]];
            vPrevMatched[i1].x = k.x;
            vPrevMatched[i1].y = k.y;
        }
    return n;
}

int ORBmatcher::BirdviewMatch(const FrameData& F1, const FrameData& F2, std::vector<int>& vnMatches12,
                              int windowSize) {
    return window_match(false, F1, F2, nullptr, windowSize, vnMatches12);
}

std::vector<int> ComputeDistinctiveDescriptors(const std::vector<std::vector<const uint8_t*> >& observations) {
    const int nmp = (int)observations.size();
    std::vector<int> off(nmp + 1, 0), best(std::max(nmp, 1), -1);
    for (int m = 0; m < nmp; m++) off[m + 1] = off[m] + (int)observations[m].size();
    std::vector<uint8_t> flat((size_t)std::max(off[nmp], 1) * 32);
    for (int m = 0; m < nmp; m++)
        for (size_t j = 0; j < observations[m].size(); j++)
            memcpy(&flat[((size_t)off[m] + j) * 32], observations[m][j], 32);
    check(orb_distinctive_descriptors(matcher_ctx(), nmp, off.data(), flat.data(), best.data()),
          "ComputeDistinctiveDescriptors");
    best.resize(nmp);
    return best;
}

}  // namespace ORBGPU_MATCHER_NAMESPACE
