// Is the result of a dependent chain of v_mfma_f32_32x32x64_f8f6f4 (fp4, unscaled) complete when the compiler's
// hazard padding lets a VALU read it?  One wave runs a chain of NCH MFMAs (each taking the previous result as C)
// and reads the result (a) right away (hipcc's own wait states), (b) after 32 and (c) after 128 extra wait
// states, many times with different data; counts results that differ from the exact sums.  The A fragments of
// successive MFMAs are loaded from LDS into reused registers, as k_top2_mfma does.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_fp4_chain_probe tools/mfma_fp4_chain_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int PAD>
__global__ void k(const int* A, const int* B, float* D, int reps) {
    __shared__ v4i sA[4][64];
    const int l = threadIdx.x;
    for (int s = 0; s < 4; s++) sA[s][l] = v4i{A[(s * 64 + l) * 4], A[(s * 64 + l) * 4 + 1], A[(s * 64 + l) * 4 + 2], A[(s * 64 + l) * 4 + 3]};
    __syncthreads();
    const v8i b = {B[4 * l], B[4 * l + 1], B[4 * l + 2], B[4 * l + 3], 0, 0, 0, 0};
    v16f seed;
    for (int r = 0; r < 16; r++) seed[r] = 8388608.f + 4096.f + (float)r;
    for (int it = 0; it < reps; it++) {
        v16f acc = seed;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const v4i av = sA[(s + it) & 3][l];
            const v8i a8 = {av[0], av[1], av[2], av[3], 0, 0, 0, 0};
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b, acc, 4, 4, 0, 0, 0, 0);
        }
        if (PAD == 32) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc));
        if (PAD == 128) {
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc));
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(acc));
        }
        for (int r = 0; r < 16; r++) D[((size_t)it * 64 + l) * 16 + r] = acc[r];
    }
}

static int nib(unsigned char* f, int lane, int e) { const unsigned char b = f[16 * lane + e / 2]; return (e & 1) ? b >> 4 : b & 15; }
static int pm4(int n) { return (n & 8) ? -4 : 4; }

int main() {
    const int reps = 64;
    unsigned char fa[4][1024], fb[1024];
    srand(11);
    for (int s = 0; s < 4; s++)
        for (int i = 0; i < 1024; i++) fa[s][i] = (unsigned char)((rand() & 1 ? 0x6 : 0xE) | ((rand() & 1 ? 0x6 : 0xE) << 4));
    for (int i = 0; i < 1024; i++) fb[i] = (unsigned char)((rand() & 1 ? 0x6 : 0xE) | ((rand() & 1 ? 0x6 : 0xE) << 4));
    // expected per (it, lane, reg): seed + sum over the 4 steps of dot(A_step row, B col); element maps of one lane pair
    static float want[64][64][16];
    for (int it = 0; it < reps; it++)
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 16; r++) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
                long long sum = 0;
                for (int s = 0; s < 4; s++) {
                    const int st = (s + it) & 3;
                    for (int h = 0; h < 2; h++)
                        for (int e = 0; e < 32; e++) sum += (long long)pm4(nib(fa[st], row + 32 * h, e)) * pm4(nib(fb, col + 32 * h, e));
                }
                want[it][l][r] = 8388608.f + 4096.f + (float)r + (float)sum;
            }
    int *dA, *dB;
    float* dD;
    hipMalloc(&dA, sizeof fa);
    hipMalloc(&dB, sizeof fb);
    hipMalloc(&dD, (size_t)reps * 64 * 16 * 4);
    hipMemcpy(dA, fa, sizeof fa, hipMemcpyHostToDevice);
    hipMemcpy(dB, fb, sizeof fb, hipMemcpyHostToDevice);
    static float got[64 * 64 * 16];
    int fail = 0;
    for (int pad : {0, 32, 128}) {
        if (pad == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, dA, dB, dD, reps);
        if (pad == 32) hipLaunchKernelGGL(k<32>, dim3(1), dim3(64), 0, 0, dA, dB, dD, reps);
        if (pad == 128) hipLaunchKernelGGL(k<128>, dim3(1), dim3(64), 0, 0, dA, dB, dD, reps);
        if (hipMemcpy(got, dD, sizeof got, hipMemcpyDeviceToHost) != hipSuccess) return printf("launch failed\n"), 2;
        int bad = 0;
        for (int it = 0; it < reps; it++)
            for (int l = 0; l < 64; l++)
                for (int r = 0; r < 16; r++) bad += got[(it * 64 + l) * 16 + r] != want[it][l][r];
        printf("pad %3d: %d of %d results differ\n", pad, bad, reps * 64 * 16);
        fail |= bad != 0;
    }
    printf(fail ? "FAIL\n" : "ok\n");
    return fail;
}
