// Per-frame latency of the drop-in boundary as the reference's caller sees it (Frame::ExtractORB,
// Frame.cc:414-420): ORB_SLAM2::ORBextractor::operator() of the C++ mirror (liborbslam_host) on host
// images, one frame in flight, synchronous.  Frames are raw 8-bit images read from a file (bench.py
// writes its synthetic frames there).  Prints one JSON line.
//
//   host_latency <frames.raw> <w> <h> <nframes> <nfeatures> <reps> [device]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../orb-slam-birdview_amd/host/ORBextractor.h"

int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s frames.raw w h nframes nfeatures reps [device]\n", argv[0]);
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), nf = atoi(argv[4]), nfeat = atoi(argv[5]), reps = atoi(argv[6]);
    const int dev = argc > 7 ? atoi(argv[7]) : 0;
    std::vector<uint8_t> frames((size_t)w * h * nf);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(frames.data(), 1, frames.size(), f) != frames.size()) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(f);
    ORB_SLAM2::ORBextractor ex(nfeat, 1.2f, 8, 20, 7, dev);
    std::vector<ORB_SLAM2::KeyPoint> kps;
    ORB_SLAM2::DescriptorMat desc;
    auto frame = [&](int i) { return ORB_SLAM2::ImageView(frames.data() + (size_t)(i % nf) * w * h, w, h); };
    for (int i = 0; i < 8; i++) ex(frame(i), ORB_SLAM2::ImageView(), kps, desc);   // warm-up (graph capture)
    std::vector<double> ms;
    long long nkp = 0;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        ex(frame(r), ORB_SLAM2::ImageView(), kps, desc);
        const auto t1 = std::chrono::steady_clock::now();
        ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        nkp += (long long)kps.size();
    }
    std::vector<double> s = ms;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (double v : ms) sum += v;
    printf("{\"ms_per_frame_median\": %.4f, \"ms_per_frame_mean\": %.4f, \"ms_per_frame_p90\": %.4f, "
           "\"keypoints_per_frame\": %.1f, \"frames\": %d}\n",
           s[s.size() / 2], sum / ms.size(), s[(size_t)(s.size() * 0.9)], (double)nkp / reps, reps);
    return 0;
}
