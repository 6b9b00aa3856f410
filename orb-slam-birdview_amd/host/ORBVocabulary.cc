// ORB_SLAM2::ORBVocabulary over liborbgpu (see ORBVocabulary.h).
#include "ORBVocabulary.h"

#include <stdlib.h>
#include <string.h>

namespace ORB_SLAM2 {

ORBVocabulary::ORBVocabulary(int device) {
    if (device < 0) {
        const char* e = getenv("ORBGPU_DEVICE");
        device = e ? atoi(e) : 0;
    }
    orb_params p;
    memset(&p, 0, sizeof p);
    p.nfeatures = 1000;
    p.scaleFactor = 1.2f;
    p.nlevels = 8;
    p.iniThFAST = 20;
    p.minThFAST = 7;
    p.device = device;
    int st = ORB_OK;
    ctx_ = orb_create(&p, &st);
    if (!ctx_) throw OrbGpuError(st, "orb_create (vocabulary)");
}

ORBVocabulary::~ORBVocabulary() {
    if (voc_) orb_vocab_destroy(voc_);
    if (ctx_) orb_destroy(ctx_);
}

bool ORBVocabulary::loadFromBinaryFile(const std::string& filename) {
    if (voc_) orb_vocab_destroy(voc_);
    voc_ = nullptr;
    if (orb_vocab_load(ctx_, filename.c_str(), &voc_) != ORB_OK) return false;
    int sc, wt, nn;
    orb_vocab_info(voc_, &k_, &L_, &sc, &wt, &nn, &nwords_);
    return true;
}

void ORBVocabulary::transform(const DescriptorMat& features, BowVector& v, BowFeatureVector& fv, int levelsup) const {
    v.clear();
    fv.clear();
    if (!voc_ || empty()) return;   // :1146-1149
    const int n = features.rows;
    if (n == 0) return;
    std::vector<int> word(n), bw(n), off(n + 1), idx(n);
    std::vector<float> weight(n);
    std::vector<uint32_t> node(n), fn(n);
    std::vector<double> bv(n);
    int st = orb_vocab_transform(ctx_, voc_, features.buf.data(), n, levelsup, word.data(), weight.data(), node.data());
    if (st != ORB_OK) throw OrbGpuError(st, "ORBVocabulary::transform");
    int nb = 0, nf = 0;
    st = orb_vocab_bow(voc_, n, word.data(), weight.data(), node.data(), bw.data(), bv.data(), &nb, fn.data(),
                       off.data(), idx.data(), &nf);
    if (st != ORB_OK) throw OrbGpuError(st, "ORBVocabulary::transform (assembly)");
    for (int i = 0; i < nb; i++) v.insert(v.end(), BowVector::value_type((unsigned)bw[i], bv[i]));
    for (int j = 0; j < nf; j++)
        fv.insert(fv.end(), BowFeatureVector::value_type(fn[j], std::vector<unsigned int>(idx.begin() + off[j],
                                                                                              idx.begin() + off[j + 1])));
}

}  // namespace ORB_SLAM2
