// Verifies the v_mfma_i32_16x16x64_i8 operand / result lane maps used by k_describe's row pass:
// A[i][k] at lane (i + 16 * (k / 16)), byte k % 16 of its 16-byte fragment; B[k][j] at lane (j + 16 * (k / 16)),
// byte k % 16; D[i][j] at lane (j + 16 * (i / 4)), register i % 4.  Prints "ok" or the first mismatch.
//   hipcc --offload-arch=gfx950 -O2 -o tools/mfma_i8_probe tools/mfma_i8_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const signed char* A, const signed char* B, int* D) {
    const int l = threadIdx.x;
    v4i a, b;
    signed char* pa = reinterpret_cast<signed char*>(&a);
    signed char* pb = reinterpret_cast<signed char*>(&b);
    for (int e = 0; e < 16; e++) {
        pa[e] = A[(l & 15) * 64 + 16 * (l >> 4) + e];   // A[i][k], i = l & 15, k = 16 (l >> 4) + e
        pb[e] = B[(16 * (l >> 4) + e) * 16 + (l & 15)];  // B[k][j], j = l & 15
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];   // D[i][j]
}
int main() {
    signed char hA[16 * 64], hB[64 * 16];
    for (int i = 0; i < 16 * 64; i++) hA[i] = (signed char)((i * 7 + 3) % 23 - 11);
    for (int i = 0; i < 64 * 16; i++) hB[i] = (signed char)((i * 5 + 1) % 19 - 9);
    signed char *dA, *dB;
    int* dD;
    hipMalloc(&dA, sizeof hA);
    hipMalloc(&dB, sizeof hB);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int hD[256];
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            int s = 0;
            for (int kk = 0; kk < 64; kk++) s += hA[i * 64 + kk] * hB[kk * 16 + j];
            if (s != hD[i * 16 + j]) {
                printf("mismatch D[%d][%d] = %d, expected %d\n", i, j, hD[i * 16 + j], s);
                return 1;
            }
        }
    printf("ok\n");
    return 0;
}
