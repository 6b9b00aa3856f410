/*
 * ORBmatcher_gpu.cc — the reference's descriptor-matcher methods with their exact signatures
 * (include/ORBmatcher.h:65-73, 87-89 of donglinb/ORB-SLAM-BIRDVIEW), computed by liborbgpu.
 *
 * This file is compiled INSIDE the reference's libORB_SLAM2, next to src/ORBmatcher.cc, from which
 * the maintainer removes the six bodies defined here:
 *
 *   int ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)              ORBmatcher.cc:159-288
 *   int ORBmatcher::SearchForInitialization(Frame&, Frame&, vector<cv::Point2f>&,
 *                                           vector<int>&, int)                      :405-520
 *   int ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)           :522-655
 *   int ORBmatcher::SearchForTriangulation(KeyFrame*, KeyFrame*, cv::Mat,
 *                                          vector<pair<size_t,size_t>>&, const bool) :657-823
 *   int ORBmatcher::BirdviewMatch(Frame&, Frame&, vector<int>&, vector<cv::Point2f>&, int)  :1667-1786
 *   int ORBmatcher::BirdviewMatch(const Frame&, const Frame&, vector<int>&, int)          :1788-1899
 *
 * plus three additions for the callers' loops over keyframes, one call each (their declarations go into
 * include/ORBmatcher.h; INTEGRATION.md §3 shows the callers):
 *   int SearchByBoW(const vector<KeyFrame*>&, Frame&, vector<vector<MapPoint*>>&, vector<int>&)   Tracking.cc:1931-1938
 *   int SearchByBoW(KeyFrame*, const vector<KeyFrame*>&, vector<vector<MapPoint*>>&, vector<int>&) LoopClosing.cc:252-265
 *   int SearchForTriangulation(KeyFrame*, const vector<KeyFrame*>&, const vector<cv::Mat>&,
 *                              vector<vector<pair<size_t,size_t>>>&, const bool)                  LocalMapping.cc:247-278
 *
 * Everything else in ORBmatcher (the projection-gated searches, Fuse, SearchBySim3, DescriptorDistance,
 * CheckDistEpipolarLine, ComputeThreeMaxima) stays the reference's own CPU code.  Callers
 * (Tracking.cc:739,1032,1938; LocalMapping.cc:278; LoopClosing.cc:265) are unchanged.
 *
 * Each method reads the same Frame / KeyFrame / MapPoint members as the reference body, hands them to
 * the C-ABI (include/orbgpu.h) as flat views, and maps the returned indices back to the reference's
 * outputs (MapPoint* for the BoW searches).  The GPU computes the distances and candidate filtering;
 * the order-dependent acceptance (taken sets, vMatchedDistance stealing, ratio test, rotation
 * histogram + ComputeThreeMaxima) is replayed by liborbgpu in the reference's iteration order, so the
 * outputs are the reference's.  The window searches' candidate lists are Frame::GetFeaturesInArea /
 * GetFeaturesInAreaBirdview evaluated on the GPU over the grid the Frame constructor built (mGrid /
 * mGridBirdview, read here); the epipole is the reference's own expression (:664-670).  A GPU failure throws std::runtime_error (the reference has no error path;
 * there is no CPU fallback).
 *
 * Thread safety: the reference calls these from the Tracking, LocalMapping and LoopClosing threads at
 * once; each host thread gets its own liborbgpu context (device ORBGPU_DEVICE, default 0).
 */
#include "ORBmatcher.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/orbgpu.h"

namespace ORB_SLAM2 {

namespace orbgpu_adapter {

static_assert(sizeof(cv::KeyPoint) == sizeof(orb_keypoint), "cv::KeyPoint must keep its 28-byte layout");

void check(int st, const char* what) {
    if (st != ORB_OK) throw std::runtime_error(std::string("liborbgpu ") + what + ": " + orb_last_error());
}

struct ThreadCtx {
    int device = -1;
    orb_ctx* ctx = nullptr;
    ~ThreadCtx() {
        if (ctx) orb_destroy(ctx);
    }
};

// one context per (host thread, device): the matchers are stack objects called from several threads
orb_ctx* ctx() {
    static thread_local ThreadCtx tc;
    static thread_local int dev = -1;   // ORBGPU_DEVICE, read once per thread (getenv scans the environment)
    if (dev < 0) {
        const char* e = getenv("ORBGPU_DEVICE");
        dev = e ? atoi(e) : 0;
    }
    if (tc.ctx && tc.device == dev) return tc.ctx;
    if (tc.ctx) orb_destroy(tc.ctx);
    tc.ctx = nullptr;
    orb_params p;
    memset(&p, 0, sizeof p);
    p.nfeatures = 1000;   // extraction parameters are unused by the matcher entry points
    p.scaleFactor = 1.2f;
    p.nlevels = 8;
    p.iniThFAST = 20;
    p.minThFAST = 7;
    p.device = dev;
    int st = ORB_OK;
    tc.ctx = orb_create(&p, &st);
    if (!tc.ctx) check(st, "orb_create");
    tc.device = dev;
    return tc.ctx;
}

// An n x 32 CV_8U descriptor matrix as one contiguous block (mDescriptors is continuous in the reference:
// ORBextractor allocates it with create(); a strided view is copied row by row).
const uint8_t* desc_rows(const cv::Mat& M, int n, std::vector<uint8_t>& tmp) {
    static const uint8_t dummy[32] = {0};
    if (n <= 0 || M.empty()) return dummy;
    if ((size_t)M.step == 32) return M.ptr(0);
    tmp.resize((size_t)n * 32);
    for (int r = 0; r < n; r++) memcpy(&tmp[(size_t)r * 32], M.ptr(r), 32);
    return tmp.data();
}

const orb_keypoint* keys_of(const std::vector<cv::KeyPoint>& k) {
    static const orb_keypoint dummy = {0, 0, 0, 0, 0, 0, 0};
    return k.empty() ? &dummy : reinterpret_cast<const orb_keypoint*>(k.data());
}

const float* angles_of(const std::vector<cv::KeyPoint>& k, std::vector<float>& a) {
    a.assign(k.size() ? k.size() : 1, 0.f);
    for (size_t i = 0; i < k.size(); i++) a[i] = k[i].angle;
    return a.data();
}

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>) as the C-ABI's CSR; std::map order
// is the reference's iteration order
struct FeatCsr {
    std::vector<uint32_t> ids;
    std::vector<int> off, idx;
    orb_featvec fv;
    FeatCsr() = default;
    explicit FeatCsr(const DBoW2::FeatureVector& f) { assign(f); }
    FeatCsr& assign(const DBoW2::FeatureVector& f) {   // (storage reused across calls)
        ids.clear();
        off.clear();
        idx.clear();
        size_t nnz = 0;
        for (DBoW2::FeatureVector::const_iterator it = f.begin(); it != f.end(); ++it) nnz += it->second.size();
        ids.reserve(f.size());
        off.reserve(f.size() + 1);
        idx.reserve(nnz + 1);
        off.push_back(0);
        for (DBoW2::FeatureVector::const_iterator it = f.begin(); it != f.end(); ++it) {
            ids.push_back(it->first);
            for (size_t j = 0; j < it->second.size(); j++) idx.push_back((int)it->second[j]);
            off.push_back((int)idx.size());
        }
        if (idx.empty()) idx.push_back(0);
        fv.nnodes = (int)ids.size();
        fv.node_ids = ids.empty() ? nullptr : ids.data();
        fv.offsets = off.data();
        fv.indices = idx.data();
        return *this;
    }
};

// A host thread's conversion buffers, reused across calls: a matcher call is tens of microseconds, and the
// dozen small allocations of building its flat views fresh every time were a measurable part of it
struct Scratch {
    FeatCsr f1, f2;
    std::vector<uint8_t> mp1, mp2, t1, t2;
    std::vector<float> ur1, ur2, a1, a2;
    std::vector<int> pairs;
};
Scratch& scratch() {
    static thread_local Scratch s;
    return s;
}

// pMP && !pMP->isBad() per feature (the BoW searches' admission test, :191-197, :558-562, :574-580)
const uint8_t* good_points(const std::vector<MapPoint*>& v, std::vector<uint8_t>& f) {
    f.assign(v.size() ? v.size() : 1, 0);
    for (size_t i = 0; i < v.size(); i++) f[i] = v[i] && !v[i]->isBad();
    return f.data();
}

}  // namespace orbgpu_adapter

using namespace orbgpu_adapter;

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(NULL));
    Scratch& S = scratch();
    const uint8_t* mp = good_points(vpMapPointsKF, S.mp1);
    const float *aKF = angles_of(pKF->mvKeysUn, S.a1), *aF = angles_of(F.mvKeys, S.a2);
    const FeatCsr& fkf = S.f1.assign(pKF->mFeatVec);
    const FeatCsr& ff = S.f2.assign(F.mFeatVec);
    std::vector<int>& match = S.pairs;
    match.assign(F.N > 0 ? F.N : 1, -1);
    int nmatches = 0;
    check(orb_search_by_bow_kf_f(ctx(), mfNNratio, mbCheckOrientation, pKF->N, desc_rows(pKF->mDescriptors, pKF->N, S.t1),
                                 aKF, mp, fkf.fv, F.N, desc_rows(F.mDescriptors, F.N, S.t2), aF, ff.fv, match.data(),
                                 &nmatches),
          "SearchByBoW(KeyFrame*, Frame&)");
    for (int iF = 0; iF < F.N; iF++)
        if (match[iF] >= 0) vpMapPointMatches[iF] = vpMapPointsKF[match[iF]];
    return nmatches;
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
    const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    vpMatches12 = std::vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(NULL));
    Scratch& S = scratch();
    const uint8_t *mp1 = good_points(vpMapPoints1, S.mp1), *mp2 = good_points(vpMapPoints2, S.mp2);
    const float *a1 = angles_of(pKF1->mvKeysUn, S.a1), *a2 = angles_of(pKF2->mvKeysUn, S.a2);
    const FeatCsr& f1 = S.f1.assign(pKF1->mFeatVec);
    const FeatCsr& f2 = S.f2.assign(pKF2->mFeatVec);
    const int n1 = (int)vpMapPoints1.size(), n2 = (int)vpMapPoints2.size();
    std::vector<int>& match = S.pairs;
    match.assign(n1 > 0 ? n1 : 1, -1);
    int nmatches = 0;
    check(orb_search_by_bow_kf_kf(ctx(), mfNNratio, mbCheckOrientation, n1, desc_rows(pKF1->mDescriptors, n1, S.t1), a1,
                                  mp1, f1.fv, n2, desc_rows(pKF2->mDescriptors, n2, S.t2), a2, mp2, f2.fv, match.data(),
                                  &nmatches),
          "SearchByBoW(KeyFrame*, KeyFrame*)");
    for (int i1 = 0; i1 < n1; i1++)
        if (match[i1] >= 0) vpMatches12[i1] = vpMapPoints2[match[i1]];
    return nmatches;
}

// SearchByBoW(pKF, F) for every keyframe of vpKFs in one call (orb_search_by_bow_kf_f_batch): the relocalisation
// candidates of Tracking::Relocalization (Tracking.cc:1931-1938), whose iterations are independent.
// vvpMapPointMatches[i] / the returned vnMatches[i] are SearchByBoW(vpKFs[i], F, ...)'s outputs.
int ORBmatcher::SearchByBoW(const std::vector<KeyFrame*>& vpKFs, Frame& F,
                            std::vector<std::vector<MapPoint*> >& vvpMapPointMatches, std::vector<int>& vnMatches) {
    const int nk = (int)vpKFs.size();
    struct Side {
        std::vector<MapPoint*> mps;
        std::vector<uint8_t> mp, t;
        std::vector<float> a;
        FeatCsr f;
        std::vector<int> match;
        int n = 0;
    };
    std::vector<Side> side(nk);
    std::vector<orb_bow_kf> K(nk);
    Scratch& S = scratch();
    const float* aF = angles_of(F.mvKeys, S.a2);
    const FeatCsr& ff = S.f2.assign(F.mFeatVec);
    for (int i = 0; i < nk; i++) {
        KeyFrame* pKF = vpKFs[i];
        Side& sd = side[i];
        sd.mps = pKF->GetMapPointMatches();
        sd.f.assign(pKF->mFeatVec);
        sd.match.assign(F.N > 0 ? F.N : 1, -1);
        K[i] = orb_bow_kf{pKF->N, desc_rows(pKF->mDescriptors, pKF->N, sd.t), angles_of(pKF->mvKeysUn, sd.a),
                          good_points(sd.mps, sd.mp), sd.f.fv, sd.match.data(), &sd.n};
    }
    check(orb_search_by_bow_kf_f_batch(ctx(), mfNNratio, mbCheckOrientation, F.N, desc_rows(F.mDescriptors, F.N, S.t2),
                                       aF, ff.fv, nk, K.data()),
          "SearchByBoW(vector<KeyFrame*>, Frame&)");
    vvpMapPointMatches.assign(nk, std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(NULL)));
    vnMatches.assign(nk, 0);
    int total = 0;
    for (int i = 0; i < nk; i++) {
        for (int iF = 0; iF < F.N; iF++)
            if (side[i].match[iF] >= 0) vvpMapPointMatches[i][iF] = side[i].mps[side[i].match[iF]];
        vnMatches[i] = side[i].n;
        total += side[i].n;
    }
    return total;
}

// SearchByBoW(pKF1, pKF2) for every pKF2 of vpKF2 in one call (orb_search_by_bow_kf_kf_batch): the loop candidates of
// LoopClosing::ComputeSim3 (LoopClosing.cc:252-265).  vvpMatches12[i] / vnMatches[i] are SearchByBoW(pKF1,
// vpKF2[i], ...)'s outputs.
int ORBmatcher::SearchByBoW(KeyFrame* pKF1, const std::vector<KeyFrame*>& vpKF2,
                            std::vector<std::vector<MapPoint*> >& vvpMatches12, std::vector<int>& vnMatches) {
    const int nk = (int)vpKF2.size();
    const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const int n1 = (int)vpMapPoints1.size();
    Scratch& S = scratch();
    const uint8_t* mp1 = good_points(vpMapPoints1, S.mp1);
    const float* a1 = angles_of(pKF1->mvKeysUn, S.a1);
    const FeatCsr& f1 = S.f1.assign(pKF1->mFeatVec);
    struct Side {
        std::vector<MapPoint*> mps;
        std::vector<uint8_t> mp, t;
        std::vector<float> a;
        FeatCsr f;
        std::vector<int> match;
        int n = 0;
    };
    std::vector<Side> side(nk);
    std::vector<orb_bow_kf> K(nk);
    for (int i = 0; i < nk; i++) {
        KeyFrame* pKF2 = vpKF2[i];
        Side& sd = side[i];
        sd.mps = pKF2->GetMapPointMatches();
        sd.f.assign(pKF2->mFeatVec);
        sd.match.assign(n1 > 0 ? n1 : 1, -1);
        K[i] = orb_bow_kf{(int)sd.mps.size(), desc_rows(pKF2->mDescriptors, (int)sd.mps.size(), sd.t),
                          angles_of(pKF2->mvKeysUn, sd.a), good_points(sd.mps, sd.mp), sd.f.fv, sd.match.data(), &sd.n};
    }
    check(orb_search_by_bow_kf_kf_batch(ctx(), mfNNratio, mbCheckOrientation, n1,
                                        desc_rows(pKF1->mDescriptors, n1, S.t1), a1, mp1, f1.fv, nk, K.data()),
          "SearchByBoW(KeyFrame*, vector<KeyFrame*>)");
    vvpMatches12.assign(nk, std::vector<MapPoint*>(n1, static_cast<MapPoint*>(NULL)));
    vnMatches.assign(nk, 0);
    int total = 0;
    for (int i = 0; i < nk; i++) {
        for (int i1 = 0; i1 < n1; i1++)
            if (side[i].match[i1] >= 0) vvpMatches12[i][i1] = side[i].mps[side[i].match[i1]];
        vnMatches[i] = side[i].n;
        total += side[i].n;
    }
    return total;
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<std::pair<size_t, size_t> >& vMatchedPairs, const bool bOnlyStereo) {
    // epipole of KF1's camera centre in KF2, the reference's own expressions (:664-670)
    cv::Mat Cw = pKF1->GetCameraCenter();
    cv::Mat R2w = pKF2->GetRotation();
    cv::Mat t2w = pKF2->GetTranslation();
    cv::Mat C2 = R2w * Cw + t2w;
    const float invz = 1.0f / C2.at<float>(2);
    const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
    const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;

    const int n1 = pKF1->N, n2 = pKF2->N;
    Scratch& S = scratch();
    std::vector<uint8_t>&mp1 = S.mp1, &mp2 = S.mp2;   // GetMapPoint(idx) != NULL (:699, :722)
    mp1.assign(n1 > 0 ? n1 : 1, 0);
    mp2.assign(n2 > 0 ? n2 : 1, 0);
    {   // GetMapPoint(idx) != NULL (:699, :722), from one snapshot (one lock instead of one per feature)
        const std::vector<MapPoint*> v1 = pKF1->GetMapPointMatches(), v2 = pKF2->GetMapPointMatches();
        for (int i = 0; i < n1; i++) mp1[i] = v1[i] != NULL;
        for (int i = 0; i < n2; i++) mp2[i] = v2[i] != NULL;
    }
    float F[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) F[3 * r + c] = F12.at<float>(r, c);   // CheckDistEpipolarLine (:143-147)
    std::vector<float>&ur1 = S.ur1, &ur2 = S.ur2;
    ur1.assign(pKF1->mvuRight.begin(), pKF1->mvuRight.end());
    ur2.assign(pKF2->mvuRight.begin(), pKF2->mvuRight.end());
    ur1.resize(n1 > 0 ? n1 : 1, -1.f);
    ur2.resize(n2 > 0 ? n2 : 1, -1.f);
    const FeatCsr& f1 = S.f1.assign(pKF1->mFeatVec);
    const FeatCsr& f2 = S.f2.assign(pKF2->mFeatVec);
    std::vector<int>& pairs = S.pairs;
    pairs.resize(2 * (size_t)(n1 > 0 ? n1 : 1));
    int np = 0;
    check(orb_search_for_triangulation(ctx(), mbCheckOrientation, bOnlyStereo, n1, desc_rows(pKF1->mDescriptors, n1, S.t1),
                                       keys_of(pKF1->mvKeysUn), mp1.data(), ur1.data(), f1.fv, n2,
                                       desc_rows(pKF2->mDescriptors, n2, S.t2), keys_of(pKF2->mvKeysUn), mp2.data(),
                                       ur2.data(), f2.fv, F, ex, ey, pKF2->mvScaleFactors.data(),
                                       pKF2->mvLevelSigma2.data(), (int)pKF2->mvScaleFactors.size(), pairs.data(),
                                       n1 > 0 ? n1 : 1, &np),
          "SearchForTriangulation");
    vMatchedPairs.clear();   // :812-820
    vMatchedPairs.reserve(np);
    for (int i = 0; i < np; i++) vMatchedPairs.push_back(std::make_pair((size_t)pairs[2 * i], (size_t)pairs[2 * i + 1]));
    return np;
}

// SearchForTriangulation of KF1 against several KF2s in one call (orb_search_for_triangulation_batch): the
// neighbour loop of LocalMapping::CreateNewMapPoints (LocalMapping.cc:247-278) with the F12s computed first.
// vvMatchedPairs[p] = SearchForTriangulation(pKF1, vpKF2[p], vF12[p], ..., bOnlyStereo) with KF1's map points as
// they are now; a caller that triangulates pair by pair drops the entries of pair p whose idx1 received a map
// point from an earlier pair (include/orbgpu.h).  Returns the total number of pairs.
int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, const std::vector<KeyFrame*>& vpKF2, const std::vector<cv::Mat>& vF12,
                                       std::vector<std::vector<std::pair<size_t, size_t> > >& vvMatchedPairs,
                                       const bool bOnlyStereo) {
    if (vF12.size() != vpKF2.size()) throw std::invalid_argument("SearchForTriangulation: one F12 per KeyFrame");
    const int n1 = pKF1->N, np = (int)vpKF2.size();
    Scratch& S = scratch();
    std::vector<uint8_t>& mp1 = S.mp1;
    mp1.assign(n1 > 0 ? n1 : 1, 0);
    {
        const std::vector<MapPoint*> v1 = pKF1->GetMapPointMatches();   // (one lock, not one per feature)
        for (int i = 0; i < n1; i++) mp1[i] = v1[i] != NULL;
    }
    std::vector<float>& ur1 = S.ur1;
    ur1.assign(pKF1->mvuRight.begin(), pKF1->mvuRight.end());
    ur1.resize(n1 > 0 ? n1 : 1, -1.f);
    const FeatCsr& f1 = S.f1.assign(pKF1->mFeatVec);
    cv::Mat Cw = pKF1->GetCameraCenter();
    struct Side {   // one KF2's arrays, alive until the call returns
        std::vector<uint8_t> mp, t;
        std::vector<float> ur;
        FeatCsr f;
        float F[9];
        std::vector<int> pairs;
        int n = 0;
    };
    std::vector<Side> side(np);
    std::vector<orb_tri_pair> P(np);
    for (int p = 0; p < np; p++) {
        KeyFrame* pKF2 = vpKF2[p];
        Side& sd = side[p];
        cv::Mat C2 = pKF2->GetRotation() * Cw + pKF2->GetTranslation();   // the epipole (:664-670)
        const float invz = 1.0f / C2.at<float>(2);
        const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
        const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
        const int n2 = pKF2->N;
        sd.mp.assign(n2 > 0 ? n2 : 1, 0);
        {
            const std::vector<MapPoint*> v2 = pKF2->GetMapPointMatches();
            for (int i = 0; i < n2; i++) sd.mp[i] = v2[i] != NULL;
        }
        sd.ur.assign(pKF2->mvuRight.begin(), pKF2->mvuRight.end());
        sd.ur.resize(n2 > 0 ? n2 : 1, -1.f);
        sd.f.assign(pKF2->mFeatVec);
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) sd.F[3 * r + c] = vF12[p].at<float>(r, c);
        sd.pairs.resize(2 * (size_t)(n1 > 0 ? n1 : 1));
        P[p] = orb_tri_pair{n2, desc_rows(pKF2->mDescriptors, n2, sd.t), keys_of(pKF2->mvKeysUn), sd.mp.data(),
                            sd.ur.data(), sd.f.fv, sd.F, ex, ey, pKF2->mvScaleFactors.data(), pKF2->mvLevelSigma2.data(),
                            (int)pKF2->mvScaleFactors.size(), sd.pairs.data(), n1 > 0 ? n1 : 1, &sd.n};
    }
    check(orb_search_for_triangulation_batch(ctx(), mbCheckOrientation, bOnlyStereo, n1,
                                             desc_rows(pKF1->mDescriptors, n1, S.t1), keys_of(pKF1->mvKeysUn), mp1.data(),
                                             ur1.data(), f1.fv, np, P.data()),
          "SearchForTriangulation(batch)");
    vvMatchedPairs.assign(np, std::vector<std::pair<size_t, size_t> >());
    int total = 0;
    for (int p = 0; p < np; p++) {
        vvMatchedPairs[p].reserve(side[p].n);
        for (int i = 0; i < side[p].n; i++)
            vvMatchedPairs[p].push_back(std::make_pair((size_t)side[p].pairs[2 * i], (size_t)side[p].pairs[2 * i + 1]));
        total += side[p].n;
    }
    return total;
}

namespace orbgpu_adapter {

// The window searches (:405-520, :1667-1899).  The candidate lists are GetFeaturesInArea(Birdview) over
// F2's grid, computed on the GPU (orb_window_match_grid) from the grid the Frame constructor built
// (mGrid / mGridBirdview, Frame.cc:378-413) and its cell geometry: the same lists, in the same order.
struct GridCsr {
    std::vector<int> off, idx;
    orb_frame_grid g;
    GridCsr(const std::vector<std::size_t> (&grid)[FRAME_GRID_COLS][FRAME_GRID_ROWS], float min_x, float min_y,
            float inv_w, float inv_h) {
        off.resize(FRAME_GRID_COLS * FRAME_GRID_ROWS + 1);
        off[0] = 0;
        for (int ix = 0; ix < FRAME_GRID_COLS; ix++)
            for (int iy = 0; iy < FRAME_GRID_ROWS; iy++) {
                const std::vector<std::size_t>& cell = grid[ix][iy];
                for (size_t j = 0; j < cell.size(); j++) idx.push_back((int)cell[j]);
                off[ix * FRAME_GRID_ROWS + iy + 1] = (int)idx.size();
            }
        if (idx.empty()) idx.push_back(0);
        g.min_x = min_x;
        g.min_y = min_y;
        g.inv_w = inv_w;
        g.inv_h = inv_h;
        g.cell_off = off.data();
        g.cell_idx = idx.data();
    }
};

int window_match(float nnratio, bool checkOri, bool level0_only, const std::vector<cv::KeyPoint>& k1,
                 const cv::Mat& d1, const std::vector<cv::KeyPoint>& k2, const cv::Mat& d2, const GridCsr& grid2,
                 const std::vector<cv::Point2f>* centres, int windowSize, std::vector<int>& vnMatches12) {
    static_assert(sizeof(cv::Point2f) == 8, "cv::Point2f must be two floats");
    const int n1 = (int)k1.size(), n2 = (int)k2.size();
    // the reference reads vbPrevMatched[i1] / vPrevMatched[i1] for every query i1 (:429, :1690): one centre
    // per F1 keypoint, or none (the own-position form)
    if (centres && !centres->empty() && centres->size() != k1.size())
        throw std::invalid_argument("window match: " + std::to_string(centres->size()) + " window centres for " +
                                    std::to_string(n1) + " keypoints");
    std::vector<uint8_t> t1, t2;
    std::vector<int> out(n1 > 0 ? n1 : 1, -1);
    int nmatches = 0;
    const float* cen = centres && !centres->empty() ? reinterpret_cast<const float*>(centres->data()) : nullptr;
    check(orb_window_match_grid(ctx(), nnratio, checkOri, level0_only, n1, desc_rows(d1, n1, t1), keys_of(k1), cen,
                                (float)windowSize, n2, desc_rows(d2, n2, t2), keys_of(k2), grid2.g, out.data(),
                                &nmatches),
          "window match");
    vnMatches12.assign(out.begin(), out.begin() + n1);
    return nmatches;
}

}  // namespace orbgpu_adapter

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
    // :416-437: level-0 queries, GetFeaturesInArea(vbPrevMatched[i1], windowSize, level1, level1)
    const GridCsr g2(F2.mGrid, F2.mnMinX, F2.mnMinY, F2.mfGridElementWidthInv, F2.mfGridElementHeightInv);
    const int nm = window_match(mfNNratio, mbCheckOrientation, true, F1.mvKeysUn, F1.mDescriptors, F2.mvKeysUn,
                                F2.mDescriptors, g2, &vbPrevMatched, windowSize, vnMatches12);
    for (size_t i1 = 0, iend1 = vnMatches12.size(); i1 < iend1; i1++)   // :514-517
        if (vnMatches12[i1] >= 0) vbPrevMatched[i1] = F2.mvKeysUn[vnMatches12[i1]].pt;
    return nm;
}

int ORBmatcher::BirdviewMatch(Frame& F1, Frame& F2, std::vector<int>& vnMatches12, std::vector<cv::Point2f>& vPrevMatched,
                              int windowSize) {
    // :1680-1700: level-0 queries around vPrevMatched[i1] in the birdview grid
    const GridCsr g2(F2.mGridBirdview, 0.f, 0.f, F2.mfGridElementWidthInvBirdview, F2.mfGridElementHeightInvBirdview);
    const int nm = window_match(mfNNratio, mbCheckOrientation, true, F1.mvKeysBird, F1.mDescriptorsBird, F2.mvKeysBird,
                                F2.mDescriptorsBird, g2, &vPrevMatched, windowSize, vnMatches12);
    for (size_t i1 = 0, iend1 = vnMatches12.size(); i1 < iend1; i1++)   // :1778-1781
        if (vnMatches12[i1] >= 0) vPrevMatched[i1] = F2.mvKeysBird[vnMatches12[i1]].pt;
    return nm;
}

int ORBmatcher::BirdviewMatch(const Frame& F1, const Frame& F2, std::vector<int>& vnMatches12, int windowSize) {
    // :1801-1812: every query, window around its own keypoint, candidates at its octave
    const GridCsr g2(F2.mGridBirdview, 0.f, 0.f, F2.mfGridElementWidthInvBirdview, F2.mfGridElementHeightInvBirdview);
    return window_match(mfNNratio, mbCheckOrientation, false, F1.mvKeysBird, F1.mDescriptorsBird, F2.mvKeysBird,
                        F2.mDescriptorsBird, g2, nullptr, windowSize, vnMatches12);
}

}  // namespace ORB_SLAM2
