// Micro-benchmark: issue rate and dependent latency of the VALU ops the SW
// kernels use (gfx950).  Build: hipcc --offload-arch=gfx950 -O3 ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// OP(d, a, b, c) as inline asm; 8 independent chains (ILP) or 1 chain.
#define DEF_KERNEL(NAME, ASM)                                                          \
template <int CHAINS>                                                                  \
__global__ void NAME(uint32_t* out, int iters, uint32_t seed) {                       \
    uint32_t v[8];                                                                     \
    for (int k = 0; k < 8; ++k) v[k] = seed * (threadIdx.x + k + 1);                   \
    uint32_t b = seed ^ 0x1234u, c = seed ^ 0x777u;                                    \
    for (int i = 0; i < iters; ++i) {                                                  \
        _Pragma("unroll")                                                              \
        for (int r = 0; r < 16; ++r) {                                                 \
            _Pragma("unroll")                                                          \
            for (int k = 0; k < CHAINS; ++k) asm volatile(ASM : "+v"(v[k]) : "v"(b), "v"(c)); \
        }                                                                              \
    }                                                                                  \
    uint32_t s = 0;                                                                    \
    for (int k = 0; k < CHAINS; ++k) s ^= v[k];                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
}

DEF_KERNEL(k_pk_max_u16, "v_pk_max_u16 %0, %0, %1")
DEF_KERNEL(k_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1 clamp")
DEF_KERNEL(k_pk_max3_f16, "v_pk_maximum3_f16 %0, %0, %1, %2")
DEF_KERNEL(k_max3_u32, "v_max3_u32 %0, %0, %1, %2")
DEF_KERNEL(k_max_u32, "v_max_u32 %0, %0, %1")
DEF_KERNEL(k_xor_b32, "v_xor_b32 %0, %0, %1")
DEF_KERNEL(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")
DEF_KERNEL(k_dpp_mov, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1")
DEF_KERNEL(k_add_dpp, "v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1")
DEF_KERNEL(k_pk_max_i16, "v_pk_max_i16 %0, %0, %1")
DEF_KERNEL(k_max_i16, "v_max_i16 %0, %0, %1")
DEF_KERNEL(k_add_u32, "v_add_u32 %0, %0, %1")
DEF_KERNEL(k_sub_u32, "v_sub_u32 %0, %0, %1")
DEF_KERNEL(k_sub_u32_clamp, "v_sub_u32 %0, %0, %1 clamp")
DEF_KERNEL(k_add3_u32, "v_add3_u32 %0, %0, %1, %2")
DEF_KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
DEF_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
DEF_KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 16, %1")
DEF_KERNEL(k_max_u16, "v_max_u16 %0, %0, %1")
DEF_KERNEL(k_min_u16, "v_min_u16 %0, %0, %1")
DEF_KERNEL(k_sub_u16_clamp, "v_sub_u16 %0, %0, %1 clamp")
DEF_KERNEL(k_sub_u16, "v_sub_u16 %0, %0, %1")
DEF_KERNEL(k_add_u16, "v_add_u16 %0, %0, %1")
DEF_KERNEL(k_max3_u16, "v_max3_u16 %0, %0, %1, %2")
DEF_KERNEL(k_max3_i16, "v_max3_i16 %0, %0, %1, %2")
DEF_KERNEL(k_med3_u16, "v_med3_u16 %0, %0, %1, %2")
DEF_KERNEL(k_max_f16, "v_max_f16 %0, %0, %1")
DEF_KERNEL(k_max_f32, "v_max_f32 %0, %0, %1")
DEF_KERNEL(k_max3_f32, "v_max3_f32 %0, %0, %1, %2")
DEF_KERNEL(k_max_i32, "v_max_i32 %0, %0, %1")
DEF_KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
DEF_KERNEL(k_max_u16_sdwa, "v_max_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0")
DEF_KERNEL(k_sad_u16, "v_sad_u16 %0, %0, %1, %2")
DEF_KERNEL(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
DEF_KERNEL(k_pk_max_f16, "v_pk_max_f16 %0, %0, %1")
DEF_KERNEL(k_pk_add_f16, "v_pk_add_f16 %0, %0, %1")
DEF_KERNEL(k_add_f16, "v_add_f16 %0, %0, %1")
DEF_KERNEL(k_maximum3_f32, "v_maximum3_f32 %0, %0, %1, %2")
DEF_KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
DEF_KERNEL(k_lshlrev, "v_lshlrev_b32 %0, 16, %0")
// round 2: the cost of hazard wait states and of the wave_shr hand-off for a
// lone wave (the config-2 loop has one DPP + s_nop 1 and ~4 s_nop 0 per step)
DEF_KERNEL(k_pk_add_f16_nop0, "v_pk_add_f16 %0, %0, %1\n s_nop 0")
DEF_KERNEL(k_pk_add_f16_nop1, "v_pk_add_f16 %0, %0, %1\n s_nop 1")
DEF_KERNEL(k_and_wave_shr, "v_and_b32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
DEF_KERNEL(k_and_row_shr, "v_and_b32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
DEF_KERNEL(k_pk_max3_f16_clamp_pair, "v_pk_maximum3_f16 %0, %0, %1, %2\n v_pk_add_f16 %0, %1, %0 clamp")

// Two independent chains per asm statement (v, w), 8 of each: the issue rate
// of a lone wave when two instruction types alternate (pipe co-issue).
#define DEF_MIX(NAME, ASM)                                                              \
template <int CHAINS>                                                                  \
__global__ void NAME(uint32_t* out, int iters, uint32_t seed) {                       \
    uint32_t v[8], w[8];                                                               \
    for (int k = 0; k < 8; ++k) { v[k] = seed * (threadIdx.x + k + 1); w[k] = v[k] ^ 0x55u; } \
    uint32_t b = seed ^ 0x1234u, c = seed ^ 0x777u;                                    \
    for (int i = 0; i < iters; ++i) {                                                  \
        _Pragma("unroll")                                                              \
        for (int r = 0; r < 8; ++r) {                                                  \
            _Pragma("unroll")                                                          \
            for (int k = 0; k < CHAINS; ++k) asm volatile(ASM : "+v"(v[k]), "+v"(w[k]) : "v"(b), "v"(c)); \
        }                                                                              \
    }                                                                                  \
    uint32_t s = 0;                                                                    \
    for (int k = 0; k < CHAINS; ++k) s ^= v[k] ^ w[k];                                 \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                    \
}
DEF_MIX(m_pkadd_pkadd, "v_pk_add_f16 %0, %0, %2\n v_pk_add_f16 %1, %1, %3")
DEF_MIX(m_pkadd_lshlor, "v_pk_add_f16 %0, %0, %2\n v_lshl_or_b32 %1, %1, 16, %3")
DEF_MIX(m_pkadd_perm, "v_pk_add_f16 %0, %0, %2\n v_perm_b32 %1, %1, %2, %3")
DEF_MIX(m_pkmax3_max3u, "v_pk_maximum3_f16 %0, %0, %2, %3\n v_max3_u32 %1, %1, %2, %3")
DEF_MIX(m_pkadd_xor, "v_pk_add_f16 %0, %0, %2\n v_xor_b32 %1, %1, %3")
DEF_MIX(m_pkadd_addu32, "v_pk_add_f16 %0, %0, %2\n v_add_u32 %1, %1, %3")
DEF_MIX(m_perm_perm, "v_perm_b32 %0, %0, %2, %3\n v_perm_b32 %1, %1, %2, %3")
DEF_MIX(m_lshlor_bfi, "v_lshl_or_b32 %0, %0, 16, %2\n v_bfi_b32 %1, %1, %2, %3")

template <typename K>
float run(K kern, int blocks, int threads, int iters, uint32_t* out) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 2, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, 3u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

#define BENCH(NAME)                                                                                   \
    {                                                                                                 \
        const int iters = 4096;                                                                       \
        float t8 = run(NAME<8>, 256 * 16, 256, iters, out);  /* 16 waves/SIMD, ILP 8 */              \
        float t1 = run(NAME<1>, 256 * 16, 256, iters, out);  /* 16 waves/SIMD, 1 chain */            \
        float l1 = run(NAME<1>, 256 * 4, 64, iters, out);    /* 1 wave/SIMD, 1 chain: latency */     \
        float i8 = run(NAME<8>, 256 * 4, 64, iters, out);    /* 1 wave/SIMD, ILP 8 */                \
        double ops8 = 256.0 * 16 * 256 / 64 * iters * 16 * 8;  /* wave-instructions */               \
        double ops1 = 256.0 * 16 * 256 / 64 * iters * 16;                                             \
        double lat_ops = 256.0 * 4 * iters * 16;                                                      \
        /* cycles per wave-instr per SIMD at 2.4 GHz (1024 SIMDs) */                                   \
        printf("%-16s full-ILP8 %.2f cyc/instr/SIMD | full-1chain %.2f | 1wave chain %.2f cyc/instr | 1wave ILP8 %.2f\n", \
               #NAME, t8 * 1e-3 * 2.4e9 * 1024 / ops8, t1 * 1e-3 * 2.4e9 * 1024 / ops1,              \
               l1 * 1e-3 * 2.4e9 * 1024 / lat_ops, i8 * 1e-3 * 2.4e9 * 1024 / (lat_ops * 8));        \
    }

#define BENCH_MIX(NAME)                                                                               \
    {                                                                                                 \
        const int iters = 4096;                                                                       \
        float i8 = run(NAME<8>, 256 * 4, 64, iters, out);    /* 1 wave/SIMD, 2 x 8 chains */          \
        float f8 = run(NAME<8>, 256 * 16, 256, iters, out);  /* 16 waves/SIMD */                      \
        double lat_ops = 256.0 * 4 * iters * 8 * 8 * 2;                                               \
        double ops8 = 256.0 * 16 * 256 / 64 * iters * 8 * 8 * 2;                                      \
        printf("%-16s mix: 1wave %.2f cyc/instr | full %.2f cyc/instr/SIMD\n", #NAME,                   \
               i8 * 1e-3 * 2.4e9 * 1024 / lat_ops, f8 * 1e-3 * 2.4e9 * 1024 / ops8);                  \
    }

int main() {
    uint32_t* out;
    CHK(hipMalloc(&out, 256 * 16 * 256 * 4));
    BENCH(k_xor_b32)
    BENCH(k_max_u32)
    BENCH(k_max3_u32)
    BENCH(k_pk_max_u16)
    BENCH(k_pk_max_i16)
    BENCH(k_max_i16)
    BENCH(k_pk_add_u16)
    BENCH(k_pk_sub_u16)
    BENCH(k_pk_max3_f16)
    BENCH(k_dpp_mov)
    BENCH(k_add_dpp)
    BENCH(k_add_u32)
    BENCH(k_sub_u32)
    BENCH(k_sub_u32_clamp)
    BENCH(k_add3_u32)
    BENCH(k_and_or)
    BENCH(k_perm)
    BENCH(k_lshl_or)
    BENCH(k_max_u16)
    BENCH(k_min_u16)
    BENCH(k_sub_u16_clamp)
    BENCH(k_sub_u16)
    BENCH(k_add_u16)
    BENCH(k_max3_u16)
    BENCH(k_max3_i16)
    BENCH(k_med3_u16)
    BENCH(k_max_f16)
    BENCH(k_max_f32)
    BENCH(k_max3_f32)
    BENCH(k_max_i32)
    BENCH(k_cndmask)
    BENCH(k_max_u16_sdwa)
    BENCH(k_sad_u16)
    BENCH(k_pk_min_u16)
    BENCH(k_pk_max_f16)
    BENCH(k_pk_add_f16)
    BENCH(k_add_f16)
    BENCH(k_maximum3_f32)
    BENCH(k_bfi)
    BENCH(k_lshlrev)
    BENCH(k_pk_add_f16_nop0)
    BENCH(k_pk_add_f16_nop1)
    BENCH(k_and_wave_shr)
    BENCH(k_and_row_shr)
    BENCH(k_pk_max3_f16_clamp_pair)
    BENCH_MIX(m_pkadd_pkadd)
    BENCH_MIX(m_pkadd_lshlor)
    BENCH_MIX(m_pkadd_perm)
    BENCH_MIX(m_pkmax3_max3u)
    BENCH_MIX(m_pkadd_xor)
    BENCH_MIX(m_pkadd_addu32)
    BENCH_MIX(m_perm_perm)
    BENCH_MIX(m_lshlor_bfi)
    CHK(hipDeviceSynchronize());
    return 0;
}
