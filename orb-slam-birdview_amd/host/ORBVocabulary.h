/*
 * ORB_SLAM2::ORBVocabulary — mirror of DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (include/ORBVocabulary.h:32, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) for the two members the
 * tracking front-end uses: loadFromBinaryFile (:1466-1510) and transform(features, BowVector&,
 * FeatureVector&, levelsup) (:1139-1210, called by Frame::ComputeBoW, Frame.cc:562-569).  The tree
 * descent of every feature runs on the GPU; BowVector / FeatureVector are assembled in feature order
 * exactly as DBoW2 does.  GPU failures throw ORB_SLAM2::OrbGpuError.
 */
#ifndef ORBGPU_HOST_ORBVOCABULARY_H
#define ORBGPU_HOST_ORBVOCABULARY_H

#include <map>
#include <string>
#include <vector>

#include "ORBextractor.h"

namespace ORB_SLAM2 {

typedef std::map<unsigned int, double> BowVector;                          // DBoW2::BowVector (BowVector.h)
typedef std::map<unsigned int, std::vector<unsigned int> > BowFeatureVector;   // DBoW2::FeatureVector

class ORBVocabulary {
public:
    explicit ORBVocabulary(int device = -1);   // -1: ORBGPU_DEVICE (default 0)
    ~ORBVocabulary();
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;

    bool loadFromBinaryFile(const std::string& filename);
    void transform(const DescriptorMat& features, BowVector& v, BowFeatureVector& fv, int levelsup) const;

    bool empty() const { return nwords_ == 0; }
    unsigned int size() const { return (unsigned int)nwords_; }
    int getBranchingFactor() const { return k_; }
    int getDepthLevels() const { return L_; }

private:
    orb_ctx* ctx_ = nullptr;
    orb_vocab* voc_ = nullptr;
    int k_ = 0, L_ = 0, nwords_ = 0;
};

}  // namespace ORB_SLAM2

#endif
