// What a ds_read_b32 / ds_read2_b32 at a 2-byte (not 4-byte) aligned LDS address returns on gfx950, and what it
// costs: k_describe's BRIEF samples read u16 runs of RT at even or odd element offsets (brief_sampled).  Prints
// the returned dwords of lanes 0..3 (aligned data would be 0x05040302 for lane 0; a masked address gives
// 0x03020100) and the cycles per dependent read, aligned vs misaligned, with random per-lane addresses.
//   hipcc --offload-arch=gfx950 -O2 -o tools/lds_unaligned_probe tools/lds_unaligned_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_probe(unsigned* out, unsigned long long* cyc, int mis) {
    __shared__ __attribute__((aligned(16))) unsigned char s[8192];
    for (int i = threadIdx.x; i < 8192; i += 64) s[i] = (unsigned char)i;
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)s;
    const int l = threadIdx.x;  // (threadIdx.y: other waves sharing the LDS)
    unsigned a = base + 4 * l + 2, r0, r1, r2;
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r0) : "v"(a));
    asm volatile("ds_read2_b32 %0, %1 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(*(unsigned long long*)&r1) : "v"(a));
    asm volatile("ds_read_u16 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r2) : "v"(a));
    out[l * 4 + 0] = r0;
    out[l * 4 + 1] = r1;
    out[l * 4 + 2] = r2;
    // timing: 1024 dependent reads at pseudo-random even (mis = 0: 4-aligned) or 2 mod 4 (mis = 1) addresses
    unsigned x = l * 2654435761u + 12345u, acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1024; i++) {
        x = x * 1664525u + 1013904223u + acc;
        const unsigned ad = base + (((x >> 8) & 2047u) << 2) + (mis ? 2u : 0u);
        unsigned v;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ad));
        acc += v & 1u;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    // issue rate: 8 independent reads per wait, 256 rounds (1 wave; 4 waves of a workgroup share the LDS pipe)
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; i++) {
        unsigned v[8];
        x = x * 1664525u + 1013904223u + acc;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const unsigned ad = base + ((((x >> 8) + 97u * k) & 2047u) << 2) + (mis ? 2u : 0u);
            asm volatile("ds_read_b32 %0, %1" : "=v"(v[k]) : "v"(ad));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; k++) acc += v[k] & 1u;
    }
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    out[l * 4 + 3] = acc;
    if (l == 0 && threadIdx.y == 0) {
        cyc[mis * 2] = t1 - t0;
        cyc[mis * 2 + 1] = t3 - t2;
    }
}

int main() {
    unsigned* d;
    unsigned long long* dc;
    hipMalloc(&d, 64 * 4 * 4);
    hipMalloc(&dc, 4 * 8);
    unsigned h[256];
    unsigned long long hc[4];
    for (int w = 1; w <= 4; w *= 4) {
        for (int mis = 0; mis < 2; mis++) hipLaunchKernelGGL(k_probe, dim3(1), dim3(64, w), 0, 0, d, dc, mis);
        hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
        printf("%d wave(s): ticks per 1024 dependent reads aligned %llu, 2-mod-4 %llu; per 2048 batched reads aligned %llu, 2-mod-4 %llu\n",
               w, hc[0], hc[2], hc[1], hc[3]);
    }
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int l = 0; l < 4; l++)
        printf("lane %d (byte %d): b32 %08x  read2 lo %08x  u16 %04x\n", l, 4 * l + 2, h[l * 4], h[l * 4 + 1], h[l * 4 + 2]);
    return 0;
}
