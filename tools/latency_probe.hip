// Round-trip latency of the pieces a per-call C-ABI entry point is made of (one stream, one device),
// median over 200 repetitions, in microseconds: an empty kernel + sync; a pinned H2D of N bytes + sync;
// H2D + kernel + D2H + sync; the same with the kernel writing its result straight into pinned host memory
// (no D2H command); and a pageable H2D for comparison.  Guides the matcher / extractor host paths.
//   hipcc --offload-arch=gfx950 -O2 -o tools/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
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
    printf("}\n");
    return 0;
}
