// CPU sanitizer harness of the ORACLE (tests/test_sanitizers.py builds it with
// -fsanitize=address,undefined and with -fsanitize=thread, together with oracle/orb_oracle.cpp).
// Drives every oracle entry point on the frames given: extraction under every flag (pinned, literal octree,
// sensitivity switches), the birdview cv::ORB + cornerSubPix stream, SearchByBoW with one node, stereo,
// distinctive descriptors, and the multi-threaded CPU-baseline paths (bench_parallel / bench_hamming),
// which are the TSan target.  Exit 0 when every run returns sane counts.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../oracle/orb_oracle.h"

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s frames.raw w h nframes\n", argv[0]);
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), n = atoi(argv[4]);
    const bool threads_only = argc > 5 && !strcmp(argv[5], "threads");
    std::vector<uint8_t> frames((size_t)w * h * n);
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(frames.data(), 1, frames.size(), fp) != frames.size()) return 2;
    fclose(fp);
    int bad = 0;
    const int nf = 1000;
    std::vector<OracleKeyPoint> k[2];
    std::vector<uint8_t> d[2];
    void* ex[2] = {nullptr, nullptr};
    if (!threads_only) {
        const int flags[] = {0, ORACLE_TIE_LITERAL, ORACLE_TIE_REVERSE_SEQ, ORACLE_RESIZE_GENERIC, ORACLE_BLUR_ALL_HALFUP,
                             ORACLE_NO_FMA, ORACLE_TRIG_CR};
        for (int fl : flags) {
            void* e = oracle_create(nf, 1.2f, 8, 20, 7, fl);
            for (int f = 0; f < n; f++) {
                const int r = oracle_run(e, frames.data() + (size_t)f * w * h, w, h, w);
                if (r < 0) bad++;
            }
            oracle_destroy(e);
        }
        for (int i = 0; i < 2 && i < n; i++) {   // frames 0, 1 kept for the matchers and stereo
            ex[i] = oracle_create(nf, 1.2f, 8, 20, 7, 0);
            const int r = oracle_run(ex[i], frames.data() + (size_t)i * w * h, w, h, w);
            k[i].resize(r > 0 ? r : 1);
            d[i].resize((size_t)(r > 0 ? r : 1) * 32);
            if (oracle_get_output(ex[i], k[i].data(), d[i].data(), (int)k[i].size()) != r) bad++;
            k[i].resize(r > 0 ? r : 0);
        }
        if (n >= 2 && !k[0].empty() && !k[1].empty()) {
            const int n0 = (int)k[0].size(), n1 = (int)k[1].size();
            std::vector<int> i0(n0), i1(n1), m(n1);
            for (int i = 0; i < n0; i++) i0[i] = i;
            for (int i = 0; i < n1; i++) i1[i] = i;
            std::vector<float> a0(n0), a1(n1);
            for (int i = 0; i < n0; i++) a0[i] = k[0][i].angle;
            for (int i = 0; i < n1; i++) a1[i] = k[1][i].angle;
            std::vector<uint8_t> mp(n0, 1);
            const uint32_t node = 0;
            const int o0[2] = {0, n0}, o1[2] = {0, n1};
            OracleFeatVec f0{1, &node, o0, i0.data()}, f1{1, &node, o1, i1.data()};
            if (oracle_search_by_bow_kf_f(0.7f, 1, n0, d[0].data(), a0.data(), mp.data(), f0, n1, d[1].data(), a1.data(),
                                          f1, m.data()) < 0)
                bad++;
            std::vector<float> u(n0), dep(n0);
            if (oracle_stereo_matches(ex[0], ex[1], n0, k[0].data(), d[0].data(), n1, k[1].data(), d[1].data(), 0.12f,
                                      60.f, u.data(), dep.data()) < 0)
                bad++;
            if (oracle_distinctive_descriptor(d[0].data(), n0 < 12 ? n0 : 12) < 0) bad++;
            void* orb = oracle_cvorb_create(2000, 1.2f, 8, 31, 20);
            std::vector<OracleKeyPoint> bk(8192);
            std::vector<uint8_t> bd(8192 * 32);
            std::vector<uint8_t> mask((size_t)w * h, 255);
            if (oracle_bird_extract(orb, frames.data(), w, h, w, mask.data(), w, bk.data(), 8192, bd.data()) < 0) bad++;
            oracle_cvorb_destroy(orb);
        }
        for (void* e : ex)
            if (e) oracle_destroy(e);
    }
    // multi-threaded CPU-baseline paths (one extractor per thread; a shared work counter)
    long long kps = 0;
    if (oracle_bench_parallel(frames.data(), n, w, h, nf, 4, 1, 2 * n, &kps) <= 0 || kps <= 0) bad++;
    if (n >= 2) {
        std::vector<uint8_t> dd((size_t)2 * 64 * 32);
        std::vector<float> aa(2 * 64);
        for (size_t i = 0; i < dd.size(); i++) dd[i] = (uint8_t)(i * 2654435761u >> 13);
        const int counts[2] = {64, 64}, qf[1] = {0}, tf[1] = {1};
        long long ev = 0;
        for (int mode = 0; mode < 2; mode++)
            if (oracle_bench_hamming(dd.data(), aa.data(), counts, 64, 1, qf, tf, mode, 4, 4, &ev) <= 0 || ev != 64 * 64)
                bad++;
    }
    printf("SANITIZE %s bad=%d\n", threads_only ? "threads" : "all", bad);
    return bad ? 1 : 0;
}
