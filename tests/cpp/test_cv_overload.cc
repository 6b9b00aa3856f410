// The host mirror's OpenCV-typed boundary (-DORBGPU_WITH_OPENCV), driven as Frame.cc:414-420 calls
// the reference: (*extractor)(im, cv::Mat(), mvKeys, mDescriptors) with std::vector<cv::KeyPoint> and
// a cv::Mat descriptor matrix, and mvImagePyramid[l] read as cv::Mat (Frame.cc:669,759).  Built
// against tests/cpp/cv_api (a model of the OpenCV 3.2 types; OpenCV is absent here).  Every result is
// compared byte for byte with the ImageView / DescriptorMat overload of the same extractor.
//
// usage: test_cv_overload <frames.raw> <w> <h> <nframes> <nfeatures>
// Prints "CHECK <name> PASS|FAIL <detail>" lines and "SUMMARY <npass> <nfail>"; exit 0 iff all pass.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../orb-slam-birdview_amd/host/ORBextractor.h"

using namespace ORB_SLAM2;

static int g_pass = 0, g_fail = 0;

static void report(const std::string& name, bool ok, const std::string& detail = "") {
    printf("CHECK %s %s %s\n", name.c_str(), ok ? "PASS" : "FAIL", detail.c_str());
    (ok ? g_pass : g_fail)++;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s frames.raw w h nframes nfeatures\n", argv[0]);
        return 2;
    }
    const int w = atoi(argv[2]), h = atoi(argv[3]), nfr = atoi(argv[4]), nf = atoi(argv[5]);
    std::vector<uint8_t> frames((size_t)w * h * nfr);
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(frames.data(), 1, frames.size(), fp) != frames.size()) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(fp);
    try {
        ORBextractor ex(nf, 1.2f, 8, 20, 7);
        for (int f = 0; f < nfr; f++) {
            const uint8_t* img = frames.data() + (size_t)f * w * h;
            const std::string tag = "frame" + std::to_string(f);
            // reference path: a padded cv::Mat (step > cols), empty mask, cv::KeyPoint vector
            const size_t step = (size_t)w + 40;
            std::vector<uint8_t> padded(step * h, 0xA5);
            for (int y = 0; y < h; y++) memcpy(padded.data() + y * step, img + (size_t)y * w, w);
            cv::Mat im(h, w, CV_8UC1, padded.data(), step);
            std::vector<cv::KeyPoint> cvk;
            cv::Mat cvd;
            ex(im, cv::Mat(), cvk, cvd);
            // pyramid level 0 as cv::Mat, read before the next extraction replaces it
            const cv::Mat& l0 = ex.mvImagePyramid[0];
            bool l0ok = l0.rows == h && l0.cols == w && l0.type() == CV_8U;
            for (int y = 0; l0ok && y < h; y++) l0ok = memcmp(l0.ptr(y), img + (size_t)y * w, w) == 0;
            report(tag + "_pyramid0_as_mat", l0ok);
            const cv::Mat& l7 = ex.mvImagePyramid[7];
            const float i7 = ex.GetInverseScaleFactors()[7];   // cvRound(cols * scale), ORBextractor.cc:1112
            report(tag + "_pyramid7_as_mat", l7.rows == (int)lrintf((float)h * i7) && l7.cols == (int)lrintf((float)w * i7),
                   std::to_string(l7.cols) + "x" + std::to_string(l7.rows));
            // the plain overload of the same extractor
            std::vector<KeyPoint> k;
            DescriptorMat d;
            ex(ImageView(img, w, h), ImageView(), k, d);
            const bool nk = cvk.size() == k.size() && !k.empty();
            report(tag + "_keypoint_count", nk, std::to_string(cvk.size()) + " vs " + std::to_string(k.size()));
            report(tag + "_keypoints_bytes",
                   nk && memcmp(cvk.data(), k.data(), k.size() * sizeof(KeyPoint)) == 0);
            bool dok = nk && cvd.rows == (int)k.size() && cvd.cols == 32 && cvd.type() == CV_8U;
            for (int i = 0; dok && i < cvd.rows; i++) dok = memcmp(cvd.ptr(i), d.ptr(i), 32) == 0;
            report(tag + "_descriptors_bytes", dok);
        }
        // empty image: outputs untouched (ORBextractor.cc:1046-1047)
        std::vector<cv::KeyPoint> keep(3);
        keep[1].octave = 5;
        cv::Mat keepd;
        keepd.create(3, 32, CV_8U);
        keepd.ptr(2)[31] = 77;
        ex(cv::Mat(), cv::Mat(), keep, keepd);
        report("empty_image_untouched", keep.size() == 3 && keep[1].octave == 5 && keepd.rows == 3 && keepd.ptr(2)[31] == 77);
        // flat image: zero keypoints, descriptors released (ORBextractor.cc:1071-1074)
        std::vector<uint8_t> flat((size_t)w * h, 128);
        ex(cv::Mat(h, w, CV_8UC1, flat.data()), cv::Mat(), keep, keepd);
        report("flat_image_released", keep.empty() && keepd.empty());
    } catch (const OrbGpuError& e) {
        printf("CHECK exception FAIL %s\n", e.what());
        g_fail++;
    }
    printf("SUMMARY %d %d\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
