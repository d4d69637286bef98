// Issue-rate microbenchmark for the integer VALU instructions the field
// kernels lean on (gfx950).  8 independent dependency chains per lane, inline
// asm so the exact instruction is issued.  Prints ns per wave-instruction per
// SIMD (lower is better) and the implied cycles at the measured clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096

#define CHAIN8(ASM)                                                                 \
    asm volatile(ASM : "+v"(a0) : "v"(k)); asm volatile(ASM : "+v"(a1) : "v"(k));  \
    asm volatile(ASM : "+v"(a2) : "v"(k)); asm volatile(ASM : "+v"(a3) : "v"(k));  \
    asm volatile(ASM : "+v"(a4) : "v"(k)); asm volatile(ASM : "+v"(a5) : "v"(k));  \
    asm volatile(ASM : "+v"(a6) : "v"(k)); asm volatile(ASM : "+v"(a7) : "v"(k));

template <int OP>
__global__ void kern(uint32_t *out, uint32_t seed) {
    uint32_t k = seed + threadIdx.x;
    uint32_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5, a6 = k + 6, a7 = k + 7;
    for (int i = 0; i < ITERS; i++) {
        if constexpr (OP == 0) { CHAIN8("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 1) { CHAIN8("v_sub_u32 %0, %0, %1") }
        if constexpr (OP == 2) { CHAIN8("v_or_b32 %0, %0, %1") }
        if constexpr (OP == 3) { CHAIN8("v_and_b32 %0, %0, %1") }
        if constexpr (OP == 4) { CHAIN8("v_xor_b32 %0, %0, %1") }
        if constexpr (OP == 5) { CHAIN8("v_lshrrev_b32 %0, %1, %0") }
        if constexpr (OP == 6) { CHAIN8("v_lshlrev_b32 %0, %1, %0") }
        if constexpr (OP == 7) { CHAIN8("v_add3_u32 %0, %0, %1, %0") }
        if constexpr (OP == 8) { CHAIN8("v_or3_b32 %0, %0, %1, %0") }
        if constexpr (OP == 9) { CHAIN8("v_mul_u32_u24 %0, %0, %1") }
        if constexpr (OP == 10) { CHAIN8("v_mad_u32_u24 %0, %0, %1, %0") }
        if constexpr (OP == 11) { CHAIN8("v_mad_i32_i24 %0, %0, %1, %0") }
        if constexpr (OP == 12) { CHAIN8("v_mul_hi_u32 %0, %0, %1") }
        if constexpr (OP == 13) { CHAIN8("v_mul_lo_u32 %0, %0, %1") }
        if constexpr (OP == 14) { CHAIN8("v_bcnt_u32_b32 %0, %0, %1") }
        if constexpr (OP == 15) { CHAIN8("v_bfe_u32 %0, %0, %1, 5") }
        if constexpr (OP == 16) { CHAIN8("v_lshl_add_u32 %0, %0, 3, %1") }
        if constexpr (OP == 17) { CHAIN8("v_min_u32 %0, %0, %1") }
        if constexpr (OP == 18) { CHAIN8("v_pk_add_u16 %0, %0, %1") }
        if constexpr (OP == 19) { CHAIN8("v_pk_mad_u16 %0, %0, %1, %0") }
        if constexpr (OP == 20) { CHAIN8("v_pk_lshrrev_b16 %0, %1, %0") }
        if constexpr (OP == 21) { CHAIN8("v_add_f32 %0, %0, %1") }
        if constexpr (OP == 22) { CHAIN8("v_fma_f32 %0, %0, %1, %0") }
        if constexpr (OP == 23) { CHAIN8("v_pk_add_u16 %0, %0, %1") }
        if constexpr (OP == 24) { CHAIN8("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 25) { CHAIN8("v_mov_b32 %0, %1") }
        if constexpr (OP == 26) { CHAIN8("v_add_u32_e64 %0, %0, %1") }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// 64-bit shift: separate kernel (64-bit operands)
__global__ void kern_shl64(uint64_t *out, uint32_t seed) {
    uint32_t k = (seed + threadIdx.x) & 63;
    uint64_t a0 = k, a1 = k + 1, a2 = k + 2, a3 = k + 3, a4 = k + 4, a5 = k + 5, a6 = k + 6, a7 = k + 7;
    for (int i = 0; i < ITERS; i++) {
#define S64(a) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(a) : "v"(k));
        S64(a0) S64(a1) S64(a2) S64(a3) S64(a4) S64(a5) S64(a6) S64(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
// LDS random ds_read_b64 vs conflict-free, as issued by 16 waves/CU
__global__ void kern_lds(uint64_t *out, uint32_t seed, int random) {
    __shared__ uint64_t tab[1600];
    for (int i = threadIdx.x; i < 1600; i += blockDim.x) tab[i] = i * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    uint32_t x = (seed + threadIdx.x * 2654435761u);
    uint64_t acc = 0;
    for (int i = 0; i < ITERS; i++) {
        uint32_t idx = random ? (x >> 16) % 1600 : (threadIdx.x + i) % 1600;
        x = x * 1664525u + 1013904223u;
        acc ^= tab[idx];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    uint64_t *buf;
    hipMalloc(&buf, 256 * 1024 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 8, block = 256;  // 8 WGs/CU -> 8 waves/SIMD
    const char *names[] = {"v_add_u32","v_sub_u32","v_or_b32","v_and_b32","v_xor_b32","v_lshrrev_b32","v_lshlrev_b32","v_add3_u32","v_or3_b32","v_mul_u32_u24","v_mad_u32_u24","v_mad_i32_i24","v_mul_hi_u32","v_mul_lo_u32","v_bcnt_u32_b32","v_bfe_u32","v_lshl_add_u32","v_min_u32","v_pk_add_u16","v_pk_mad_u16","v_pk_lshrrev_b16","v_add_f32","v_fma_f32","v_pk_add_u16_b","v_add_u32_b","v_mov_b32","v_add_u32_e64"};
    auto run = [&](auto launch, const char *name) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double winstr = (double)grid * block / 64 * ITERS * 8;  // wave-instructions
        double per_simd = winstr / 1024;
        printf("%-18s %8.3f ms  %.3f ns per wave-instr per SIMD (%.2f cyc @2.4GHz)\n", name, ms,
               ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
    };
#define RUN(OP) run([&] { hipLaunchKernelGGL(kern<OP>, dim3(grid), dim3(block), 0, 0, (uint32_t *)buf, 7u); }, names[OP]);
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15) RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25) RUN(26)
    run([&] { hipLaunchKernelGGL(kern_shl64, dim3(grid), dim3(block), 0, 0, buf, 7u); }, "v_lshlrev_b64");
    for (int r = 0; r < 2; r++) {
        hipLaunchKernelGGL(kern_lds, dim3(grid), dim3(block), 0, 0, buf, 7u, r);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern_lds, dim3(grid), dim3(block), 0, 0, buf, 7u, r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double lds_per_cu = (double)grid * block / 64 * ITERS / 256;
        printf("ds_read_b64 %s: %.3f ms, %.2f cyc per wave-read per CU @2.4GHz\n",
               r ? "random" : "linear", ms, ms * 1e6 * 2.4 / lds_per_cu);
    }
    return 0;
}
