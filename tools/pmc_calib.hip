// FETCH_SIZE / WRITE_SIZE calibration for the access widths liborbgpu uses (MI355X_MICROARCH.md
// §HBM: "other access widths are uncalibrated: calibrate on a known byte count").  Streams a
// 512 MiB buffer (past the 256 MiB Infinity Cache) once per kernel with 1-, 4- and 16-byte
// per-lane loads, and writes 256 MiB with 4-byte per-lane stores.  Run under
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) --kernel-trace; tools/pmc_report.py divides the
// counter by the known byte count to get the correction factor per width.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k_calib_read_u8(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_calib_read_u32(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_calib_read_u128(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_calib_write_u32(uint32_t* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)i;
}

int main() {
    const size_t bytes = 512ull << 20, wbytes = 256ull << 20;
    uint8_t *a = nullptr, *b = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, wbytes) != hipSuccess ||
        hipMalloc(&out, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, wbytes);
    (void)hipDeviceSynchronize();
    const dim3 grid(4096), block(256);
    hipLaunchKernelGGL(k_calib_read_u8, grid, block, 0, 0, a, bytes, out);
    hipLaunchKernelGGL(k_calib_read_u32, grid, block, 0, 0, (const uint32_t*)a, bytes / 4, out);
    hipLaunchKernelGGL(k_calib_read_u128, grid, block, 0, 0, (const uint4*)a, bytes / 16, out);
    hipLaunchKernelGGL(k_calib_write_u32, grid, block, 0, 0, (uint32_t*)b, wbytes / 4);
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
    }
    printf("{\"read_bytes\": %zu, \"write_bytes\": %zu}\n", bytes, wbytes);
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(out);
    return 0;
}
