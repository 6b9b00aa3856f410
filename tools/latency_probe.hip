// Round-trip latency of the pieces a per-call C-ABI entry point is made of (one stream, one device),
// median over 200 repetitions, in microseconds: an empty kernel + sync; a pinned H2D of N bytes + sync;
// H2D + kernel + D2H + sync; the same with the kernel writing its result straight into pinned host memory
// (no D2H command); and a pageable H2D for comparison.  Guides the matcher / extractor host paths.
//   hipcc --offload-arch=gfx950 -O2 -o tools/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <vector>

__global__ void k_empty() {}
__global__ void k_touch(const int* __restrict__ in, int* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] + 1;
}

template <class F>
static double med(F f) {
    std::vector<double> t;
    for (int r = 0; r < 220; r++) {
        const auto a = std::chrono::steady_clock::now();
        f();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        if (r >= 20) t.push_back(us);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t big = 1 << 20;
    int *d_in, *d_out, *h_in, *h_out;
    CK(hipMalloc(&d_in, big * 4));
    CK(hipMalloc(&d_out, big * 4));
    CK(hipHostMalloc(&h_in, big * 4, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, big * 4, hipHostMallocDefault));
    std::vector<int> pageable(big);
    printf("{");
    printf("\"empty_kernel_sync_us\": %.1f", med([&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
               (void)hipStreamSynchronize(s);
           }));
    for (size_t bytes : {4096ul, 65536ul, 262144ul}) {
        const int n = (int)(bytes / 4);
        printf(", \"h2d_pinned_%zu_us\": %.1f", bytes, med([&] {
                   (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"h2d_pageable_%zu_us\": %.1f", bytes, med([&] {
                   (void)hipMemcpyAsync(d_in, pageable.data(), bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"h2d_kernel_d2h_%zu_us\": %.1f", bytes, med([&] {
                   (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s);
                   hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, d_in, d_out, n);
                   (void)hipMemcpyAsync(h_out, d_out, 4096, hipMemcpyDeviceToHost, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"h2d_kernel_to_host_%zu_us\": %.1f", bytes, med([&] {
                   (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s);
                   hipLaunchKernelGGL(k_touch, dim3((1024 + 255) / 256), dim3(256), 0, s, d_in, h_out, 1024);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"kernel_reads_host_%zu_us\": %.1f", bytes, med([&] {
                   hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, h_in, d_out, n);
                   (void)hipStreamSynchronize(s);
               }));
    }
    // a C3 host image (1280 x 720 u8) as ORBextractor::operator() receives it: pageable caller memory
    {
        const size_t W = 1280, H = 720, bytes = W * H;
        std::vector<uint8_t> img(bytes, 7);
        uint8_t *d_img, *h_stage;
        CK(hipMalloc(&d_img, bytes));
        CK(hipHostMalloc(&h_stage, bytes, hipHostMallocDefault));
        printf(", \"img_pageable_1d_us\": %.1f", med([&] {
                   (void)hipMemcpyAsync(d_img, img.data(), bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_pageable_2d_us\": %.1f", med([&] {
                   (void)hipMemcpy2DAsync(d_img, W, img.data(), W, W, H, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_pageable_1d_then_kernel_us\": %.1f", med([&] {
                   (void)hipMemcpyAsync(d_img, img.data(), bytes, hipMemcpyHostToDevice, s);
                   hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_pageable_2d_then_kernel_us\": %.1f", med([&] {
                   (void)hipMemcpy2DAsync(d_img, W, img.data(), W, W, H, hipMemcpyHostToDevice, s);
                   hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_host_memcpy_to_pinned_us\": %.1f", med([&] { std::memcpy(h_stage, img.data(), bytes); }));
        printf(", \"img_memcpy_pinned_dma_us\": %.1f", med([&] {
                   std::memcpy(h_stage, img.data(), bytes);
                   (void)hipMemcpyAsync(d_img, h_stage, bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_pinned_dma_us\": %.1f", med([&] {
                   (void)hipMemcpyAsync(d_img, h_stage, bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
               }));
        printf(", \"img_register_dma_unregister_us\": %.1f", med([&] {
                   (void)hipHostRegister(img.data(), bytes, hipHostRegisterDefault);
                   void* dp = nullptr;
                   (void)hipHostGetDevicePointer(&dp, img.data(), 0);
                   (void)hipMemcpyAsync(d_img, img.data(), bytes, hipMemcpyHostToDevice, s);
                   (void)hipStreamSynchronize(s);
                   (void)hipHostUnregister(img.data());
               }));
        printf(", \"img_memcpy_pinned_dma_then_kernel_us\": %.1f", med([&] {
                   std::memcpy(h_stage, img.data(), bytes);
                   (void)hipMemcpyAsync(d_img, h_stage, bytes, hipMemcpyHostToDevice, s);
                   hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                   (void)hipStreamSynchronize(s);
               }));
        hipStream_t s2[4];
        hipEvent_t ev[4];
        for (int i = 0; i < 4; i++) {
            CK(hipStreamCreateWithFlags(&s2[i], hipStreamNonBlocking));
            CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        }
        for (int parts : {2, 4}) {
            const size_t pb = bytes / parts;
            printf(", \"img_pinned_dma_%dstreams_then_kernel_us\": %.1f", parts, med([&] {
                       for (int i = 0; i < parts; i++) {
                           (void)hipMemcpyAsync(d_img + i * pb, h_stage + i * pb, pb, hipMemcpyHostToDevice, s2[i]);
                           (void)hipEventRecord(ev[i], s2[i]);
                           (void)hipStreamWaitEvent(s, ev[i], 0);
                       }
                       hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                       (void)hipStreamSynchronize(s);
                   }));
            printf(", \"img_memcpy_pinned_dma_%dstreams_then_kernel_us\": %.1f", parts, med([&] {
                       for (int i = 0; i < parts; i++) {
                           std::memcpy(h_stage + i * pb, img.data() + i * pb, pb);
                           (void)hipMemcpyAsync(d_img + i * pb, h_stage + i * pb, pb, hipMemcpyHostToDevice, s2[i]);
                           (void)hipEventRecord(ev[i], s2[i]);
                           (void)hipStreamWaitEvent(s, ev[i], 0);
                       }
                       hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                       (void)hipStreamSynchronize(s);
                   }));
            printf(", \"img_memcpy_pinned_dma_%dchunks_1stream_then_kernel_us\": %.1f", parts, med([&] {
                       for (int i = 0; i < parts; i++) {
                           std::memcpy(h_stage + i * pb, img.data() + i * pb, pb);
                           (void)hipMemcpyAsync(d_img + i * pb, h_stage + i * pb, pb, hipMemcpyHostToDevice, s);
                       }
                       hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
                       (void)hipStreamSynchronize(s);
                   }));
        }
        printf(", \"img_kernel_reads_pinned_us\": %.1f", med([&] {
                   hipLaunchKernelGGL(k_touch, dim3((int)(bytes / 4 + 255) / 256), dim3(256), 0, s, (const int*)h_stage, (int*)d_img, (int)(bytes / 4));
                   (void)hipStreamSynchronize(s);
               }));
        (void)hipFree(d_img);
        (void)hipHostFree(h_stage);
    }
    printf("}\n");
    return 0;
}
