// Microbenchmark (diagnostic): issue rate of the integer VALU instructions the FAST / describe kernels
// use, at 8 waves per SIMD, 8 independent chains per wave.  Prints cycles per wave64 instruction per
// SIMD (2 = full SIMD-32 rate).  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rate tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>


#define OP2(name, asmop)                                                                                  \
    __global__ __launch_bounds__(256) void name(unsigned* out, unsigned seed, int rep) {                           \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, \
                 a6 = a0 * 13, a7 = a0 * 15, b = seed * 17 + threadIdx.x;                                 \
        for (int i = 0; i < rep; i++) {                                                                   \
            asm volatile(asmop " %0, %0, %8\n\t" asmop " %1, %1, %8\n\t" asmop " %2, %2, %8\n\t" asmop    \
                         " %3, %3, %8\n\t" asmop " %4, %4, %8\n\t" asmop " %5, %5, %8\n\t" asmop           \
                         " %6, %6, %8\n\t" asmop " %7, %7, %8"                                             \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b));                                                                       \
        }                                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                       \
    }

#define OP3(name, asmop)                                                                                  \
    __global__ __launch_bounds__(256) void name(unsigned* out, unsigned seed, int rep) {                           \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, \
                 a6 = a0 * 13, a7 = a0 * 15, b = seed * 17 + threadIdx.x, c = seed ^ 0x0c020c00u;         \
        for (int i = 0; i < rep; i++) {                                                                   \
            asm volatile(asmop " %0, %0, %8, %9\n\t" asmop " %1, %1, %8, %9\n\t" asmop " %2, %2, %8, %9\n\t" \
                         asmop " %3, %3, %8, %9\n\t" asmop " %4, %4, %8, %9\n\t" asmop " %5, %5, %8, %9\n\t" \
                         asmop " %6, %6, %8, %9\n\t" asmop " %7, %7, %8, %9"                               \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b), "v"(c));                                                               \
        }                                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                       \
    }

OP2(k2_v_add_u32, "v_add_u32")
OP2(k2_v_sub_u32, "v_sub_u32")
OP2(k2_v_and_b32, "v_and_b32")
OP2(k2_v_or_b32, "v_or_b32")
OP2(k2_v_xor_b32, "v_xor_b32")
OP2(k2_v_lshlrev_b32, "v_lshlrev_b32")
OP2(k2_v_lshrrev_b32, "v_lshrrev_b32")
OP2(k2_v_max_u32, "v_max_u32")
OP2(k2_v_max_i32, "v_max_i32")
OP2(k2_v_min_u32, "v_min_u32")
OP2(k2_v_mul_lo_u32, "v_mul_lo_u32")
OP2(k2_v_mul_u32_u24, "v_mul_u32_u24")
OP2(k2_v_add_f32, "v_add_f32")
OP2(k2_v_sub_f32, "v_sub_f32")
OP2(k2_v_mul_f32, "v_mul_f32")
OP2(k2_v_max_f32, "v_max_f32")
OP2(k2_v_min_f32, "v_min_f32")
OP2(k2_v_pk_max_u16, "v_pk_max_u16")
OP2(k2_v_pk_min_u16, "v_pk_min_u16")
OP2(k2_v_pk_sub_i16, "v_pk_sub_i16")
OP2(k2_v_pk_add_u16, "v_pk_add_u16")
OP2(k2_v_pk_max_i16, "v_pk_max_i16")
OP2(k2_v_pk_max_f16, "v_pk_max_f16")
OP2(k2_v_pk_min_f16, "v_pk_min_f16")
OP2(k2_v_pk_add_f16, "v_pk_add_f16")
OP2(k2_v_pk_mul_f16, "v_pk_mul_f16")
OP2(k2_v_max_f16, "v_max_f16")
OP2(k2_v_add_f16, "v_add_f16")
OP2(k2_v_bcnt_u32_b32, "v_bcnt_u32_b32")
OP3(k3_v_perm_b32, "v_perm_b32")
OP3(k3_v_alignbyte_b32, "v_alignbyte_b32")
OP3(k3_v_alignbit_b32, "v_alignbit_b32")
OP3(k3_v_min3_i32, "v_min3_i32")
OP3(k3_v_max3_i32, "v_max3_i32")
OP3(k3_v_min3_f32, "v_min3_f32")
OP3(k3_v_max3_f32, "v_max3_f32")
OP3(k3_v_med3_f32, "v_med3_f32")
OP3(k3_v_lerp_u8, "v_lerp_u8")
OP3(k3_v_dot4_u32_u8, "v_dot4_u32_u8")
OP3(k3_v_dot2_u32_u16, "v_dot2_u32_u16")
OP3(k3_v_and_or_b32, "v_and_or_b32")
OP3(k3_v_or3_b32, "v_or3_b32")
OP3(k3_v_lshl_or_b32, "v_lshl_or_b32")
OP3(k3_v_add3_u32, "v_add3_u32")
OP3(k3_v_bfe_u32, "v_bfe_u32")
OP3(k3_v_bfi_b32, "v_bfi_b32")
OP3(k3_v_fma_f32, "v_fma_f32")
OP3(k3_v_pk_fma_f16, "v_pk_fma_f16")
OP3(k3_v_mad_u32_u24, "v_mad_u32_u24")
OP3(k3_v_sad_u8, "v_sad_u8")

typedef void (*K)(unsigned*, unsigned, int);

int main() {
    int ncu = 0, clk = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);   // kHz
    const int blocks = ncu * 8;   // 8 x 256 threads per CU = 8 waves per SIMD
    unsigned* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    struct {
        const char* n;
        K k;
    } ks[] = {{"v_add_u32", k2_v_add_u32}, {"v_sub_u32", k2_v_sub_u32}, {"v_and_b32", k2_v_and_b32}, {"v_or_b32", k2_v_or_b32}, {"v_xor_b32", k2_v_xor_b32}, {"v_lshlrev_b32", k2_v_lshlrev_b32}, {"v_lshrrev_b32", k2_v_lshrrev_b32}, {"v_max_u32", k2_v_max_u32}, {"v_max_i32", k2_v_max_i32}, {"v_min_u32", k2_v_min_u32}, {"v_mul_lo_u32", k2_v_mul_lo_u32}, {"v_mul_u32_u24", k2_v_mul_u32_u24}, {"v_add_f32", k2_v_add_f32}, {"v_sub_f32", k2_v_sub_f32}, {"v_mul_f32", k2_v_mul_f32}, {"v_max_f32", k2_v_max_f32}, {"v_min_f32", k2_v_min_f32}, {"v_pk_max_u16", k2_v_pk_max_u16}, {"v_pk_min_u16", k2_v_pk_min_u16}, {"v_pk_sub_i16", k2_v_pk_sub_i16}, {"v_pk_add_u16", k2_v_pk_add_u16}, {"v_pk_max_i16", k2_v_pk_max_i16}, {"v_pk_max_f16", k2_v_pk_max_f16}, {"v_pk_min_f16", k2_v_pk_min_f16}, {"v_pk_add_f16", k2_v_pk_add_f16}, {"v_pk_mul_f16", k2_v_pk_mul_f16}, {"v_max_f16", k2_v_max_f16}, {"v_add_f16", k2_v_add_f16}, {"v_bcnt_u32_b32", k2_v_bcnt_u32_b32}, {"v_perm_b32", k3_v_perm_b32}, {"v_alignbyte_b32", k3_v_alignbyte_b32}, {"v_alignbit_b32", k3_v_alignbit_b32}, {"v_min3_i32", k3_v_min3_i32}, {"v_max3_i32", k3_v_max3_i32}, {"v_min3_f32", k3_v_min3_f32}, {"v_max3_f32", k3_v_max3_f32}, {"v_med3_f32", k3_v_med3_f32}, {"v_lerp_u8", k3_v_lerp_u8}, {"v_dot4_u32_u8", k3_v_dot4_u32_u8}, {"v_dot2_u32_u16", k3_v_dot2_u32_u16}, {"v_and_or_b32", k3_v_and_or_b32}, {"v_or3_b32", k3_v_or3_b32}, {"v_lshl_or_b32", k3_v_lshl_or_b32}, {"v_add3_u32", k3_v_add3_u32}, {"v_bfe_u32", k3_v_bfe_u32}, {"v_bfi_b32", k3_v_bfi_b32}, {"v_fma_f32", k3_v_fma_f32}, {"v_pk_fma_f16", k3_v_pk_fma_f16}, {"v_mad_u32_u24", k3_v_mad_u32_u24}, {"v_sad_u8", k3_v_sad_u8}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& k : ks) {
        float t[2];
        const int reps[2] = {1024, 5120};
        for (int q = 0; q < 2; q++) {
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 1u, reps[q]);
            hipDeviceSynchronize();
            float best = 1e30f;
            for (int r = 0; r < 5; r++) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, (unsigned)r, reps[q]);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            t[q] = best;
        }
        // per SIMD: 8 waves x rep x 8 instructions; the slope between the two rep counts removes the
        // launch and ramp overhead
        const double cycles = (t[1] - t[0]) * 1e-3 * (double)clk * 1e3;
        const double per = cycles / (8.0 * (reps[1] - reps[0]) * 8);
        printf("%-16s %.3f / %.3f ms  %.2f cycles per wave64 instruction per SIMD (clock %d MHz)\n", k.n, t[0], t[1], per,
               clk / 1000);
    }
    hipFree(out);
    return 0;
}
