// DistributeOctTree tie-order study driver (tools/tie_study.py).  Runs the oracle's extractor with
// ORACLE_TIE_LITERAL — the reference's std::list / pair<int, node*> algorithm, ties decided by the heap
// addresses glibc malloc hands out in THIS process — over frames read from a raw file, and writes each
// frame's keypoints.  The heap context is the point of the study:
//   fresh   one frame per process (tie_study.py starts one process per frame)
//   warm    one process, one extractor, the frames in sequence (a tracking thread's steady state)
//   thread  one extractor, each frame on a fresh std::thread (Frame.cc:124-127 spawns them per frame)
// Output file: per frame, int32 n then n OracleKeyPoint (28 B each).  Test infrastructure only.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../oracle/orb_oracle.h"

int main(int argc, char** argv) {
    if (argc < 9) {
        std::fprintf(stderr, "usage: tie_driver frames.raw w h nfeatures fresh|warm|thread first count out.bin [flags]\n");
        return 2;
    }
    const char* path = argv[1];
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), nf = std::atoi(argv[4]);
    const char* mode = argv[5];
    const int first = std::atoi(argv[6]), count = std::atoi(argv[7]);
    const int flags = argc > 9 ? std::atoi(argv[9]) : ORACLE_TIE_LITERAL;
    const size_t fb = (size_t)w * h;
    std::vector<unsigned char> frames(fb * count);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fseek(f, (long)(fb * first), SEEK_SET) != 0 || std::fread(frames.data(), 1, frames.size(), f) != frames.size()) {
        std::fprintf(stderr, "cannot read frames\n");
        return 1;
    }
    std::fclose(f);
    FILE* out = std::fopen(argv[8], "wb");
    if (!out) return 1;
    void* ex = oracle_create(nf, 1.2f, 8, 20, 7, flags);
    std::vector<OracleKeyPoint> kps(16 * (size_t)nf + 1024);
    std::vector<unsigned char> desc(kps.size() * 32);
    auto one = [&](int i) {
        const int n = oracle_run(ex, frames.data() + fb * i, w, h, w);
        const int m = n > 0 ? oracle_get_output(ex, kps.data(), desc.data(), (int)kps.size()) : 0;
        std::fwrite(&m, 4, 1, out);
        if (m > 0) std::fwrite(kps.data(), sizeof(OracleKeyPoint), m, out);
    };
    for (int i = 0; i < count; i++) {
        if (!std::strcmp(mode, "thread")) {
            std::thread t(one, i);
            t.join();
        } else {
            one(i);
        }
    }
    oracle_destroy(ex);
    std::fclose(out);
    return 0;
}
