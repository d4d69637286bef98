// LDS random-lookup microbenchmark (gfx950): cycles per wave-lookup of the
// table layouts considered for the b80-class FD kernel.
// Each lane walks a pseudo-random sequence of entry indices e < 6400 (the b80
// digit-pair table) and ORs what it reads into its mask words, 16 waves per CU
// (4 per SIMD, the b80 kernel's occupancy):
//   0  one ds_read_b128 of a 16-byte entry (102 KB table: production b80)
//   1  ds_read_b64 of an 8-byte low entry (51 KB) + ds_read_u16 of the high
//      16 bits (12.8 KB): the split layout
//   2  ds_read_b64 of an 8-byte entry only (the b40-class lookup, 6400 entries)
//   3  ds_read_u16 only
//   4  ds_read_b128 with every lane of a 16-lane group on its own 16-byte slot
//      column (lane-column replicated 80-entry digit table, 20 KB): conflict-free
//   5  16-byte entries read as ds_read_b64 at +0 and ds_read_u16 at +8 (same
//      stored limb, two immediate offsets)
//   6  ds_read_b64 stride 8 + ds_read_u16 stride 8 (two 51 KB regions)
//   7..9  the single reads of 5 and 6 alone
//   10 ds_read_b96 of a 12-byte entry (77 KB, 4-byte aligned: gfx950 DS
//      unaligned access), checked against a host recomputation
//   11 ds_read_b96 of a 16-byte entry (aligned)
//   12 ds_read_b64 stride 8 + ds_read_b32 stride 4 (two regions, 51 + 26 KB)
//   13 12-byte entries read as ds_read_b64 at +0 and ds_read_b32 at +8
// Prints ns and LDS-cycles per wave-lookup (clock from s_memtime), so the
// conflict cost of each layout is measured, not modelled.
//   hipcc --offload-arch=gfx950 -O3 -o lds_lookup lds_lookup.hip && ./lds_lookup
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
typedef uint32_t v3u __attribute__((ext_vector_type(3)));
constexpr uint32_t NE = 6400;

template <int MODE>
__global__ void __launch_bounds__(1024) kern(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) unsigned char t[NE * 16 + 16];  // 102 KB
    for (uint32_t i = threadIdx.x; i < (NE * 16 + 16) / 4; i += blockDim.x)
        ((uint32_t *)t)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = seed * 747796405u + threadIdx.x * 2891336453u + blockIdx.x;
    uint32_t m0 = 0, m1 = 0, m2 = 0;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int i = 0; i < ITERS; i++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t e = __umulhi(x, NE);  // uniform in [0, NE)
        if constexpr (MODE == 0) {
            const uint4 v = *(const uint4 *)(t + e * 16);
            m0 |= v.x; m1 |= v.y; m2 |= v.z;
            asm volatile("" ::"v"(v.w));
        } else if constexpr (MODE == 1) {
            const uint2 v = *(const uint2 *)(t + e * 8);
            const uint32_t h = *(const uint16_t *)(t + NE * 8 + e * 2);
            m0 |= v.x; m1 |= v.y; m2 |= h;
        } else if constexpr (MODE == 2) {
            const uint2 v = *(const uint2 *)(t + e * 8);
            m0 |= v.x; m1 |= v.y;
        } else if constexpr (MODE == 3) {
            m2 |= *(const uint16_t *)(t + e * 2);
        } else if constexpr (MODE == 5) {  // 16-B entries: b64 at +0, u16 at +8
            const uint2 v = *(const uint2 *)(t + e * 16);
            const uint32_t h = *(const uint16_t *)(t + e * 16 + 8);
            m0 |= v.x; m1 |= v.y; m2 |= h;
        } else if constexpr (MODE == 6) {  // b64 stride 8 + u16 stride 8 (own region)
            const uint2 v = *(const uint2 *)(t + e * 8);
            const uint32_t h = *(const uint16_t *)(t + NE * 8 + e * 8);
            m0 |= v.x; m1 |= v.y; m2 |= h;
        } else if constexpr (MODE == 7) {  // b64 stride 16 only
            const uint2 v = *(const uint2 *)(t + e * 16);
            m0 |= v.x; m1 |= v.y;
        } else if constexpr (MODE == 8) {  // u16 stride 8 only
            m2 |= *(const uint16_t *)(t + e * 8);
        } else if constexpr (MODE == 9) {  // u16 stride 16 only
            m2 |= *(const uint16_t *)(t + e * 16 + 8);
        } else if constexpr (MODE == 10) {  // 12-B entries, one ds_read_b96
            const v3u v = *(const v3u *)__builtin_assume_aligned(t + e * 12, 4);
            m0 |= v.x; m1 |= v.y; m2 |= v.z;
        } else if constexpr (MODE == 11) {  // 16-B entries, ds_read_b96
            const v3u v = *(const v3u *)(t + e * 16);
            m0 |= v.x; m1 |= v.y; m2 |= v.z;
        } else if constexpr (MODE == 12) {  // b64 stride 8 + b32 stride 4
            const uint2 v = *(const uint2 *)(t + e * 8);
            m0 |= v.x; m1 |= v.y; m2 |= *(const uint32_t *)(t + NE * 8 + e * 4);
        } else if constexpr (MODE == 13) {  // 12-B entries: b64 at +0, b32 at +8
            const uint2 v = *(const uint2 *)__builtin_assume_aligned(t + e * 12, 4);
            asm volatile("" ::"v"(v.x));
            m0 |= v.x; m1 |= v.y; m2 |= *(const uint32_t *)(t + e * 12 + 8);
        } else {
            const uint32_t d = __umulhi(x, 80);
            const uint4 v = *(const uint4 *)(t + (d * 16 + (lane & 15)) * 16);
            m0 |= v.x; m1 |= v.y; m2 |= v.z;
            asm volatile("" ::"v"(v.w));
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = m0 ^ m1 ^ m2;
    if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

template <int MODE>
static void run(const char *name, uint32_t *out, uint64_t *cyc, int cus) {
    const int grid = cus;  // one 1024-thread workgroup per CU (16 waves)
    hipLaunchKernelGGL(kern<MODE>, dim3(grid), dim3(1024), 0, 0, out, cyc, 1u);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(kern<MODE>, dim3(grid), dim3(1024), 0, 0, out, cyc, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint64_t h[1024];
    hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; i++) s += (double)h[i];
    s /= grid;
    // per CU: 16 waves x ITERS lookups share the CU's one LDS pipe
    const double per = s / (16.0 * ITERS);
    printf("%-44s %8.3f ms  %6.2f cycles per wave-lookup per CU (s_memtime)\n", name, ms, per);
    if (MODE == 10) {  // the unaligned b96 read returns the right words
        static uint32_t o[1024];
        hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
        int bad = 0;
        for (uint32_t tid = 0; tid < 1024; tid++) {
            uint32_t x = 2u * 747796405u + tid * 2891336453u + 0u, m0 = 0, m1 = 0, m2 = 0;
            for (int i = 0; i < ITERS; i++) {
                x = x * 1664525u + 1013904223u;
                const uint32_t e = (uint32_t)(((uint64_t)x * NE) >> 32);
                m0 |= (e * 3) * 2654435761u;
                m1 |= (e * 3 + 1) * 2654435761u;
                m2 |= (e * 3 + 2) * 2654435761u;
            }
            bad += o[tid] != (m0 ^ m1 ^ m2);
        }
        printf("  b96 unaligned check: %d of 1024 lanes differ\n", bad);
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&out, (size_t)cus * 1024 * 4);
    hipMalloc(&cyc, (size_t)cus * 8);
    run<0>("b128 16-B entries (production b80)", out, cyc, cus);
    run<1>("b64 8-B low + u16 high (split layout)", out, cyc, cus);
    run<2>("b64 8-B entries only", out, cyc, cus);
    run<3>("u16 2-B entries only", out, cyc, cus);
    run<4>("b128 lane-column digit table (no conflicts)", out, cyc, cus);
    run<5>("16-B entries: b64 +0 and u16 +8", out, cyc, cus);
    run<6>("b64 stride 8 + u16 stride 8", out, cyc, cus);
    run<7>("b64 stride 16 only", out, cyc, cus);
    run<8>("u16 stride 8 only", out, cyc, cus);
    run<9>("u16 stride 16 only", out, cyc, cus);
    run<10>("b96 12-B entries (unaligned)", out, cyc, cus);
    run<11>("b96 16-B entries", out, cyc, cus);
    run<12>("b64 stride 8 + b32 stride 4", out, cyc, cus);
    run<13>("12-B entries: b64 +0 and b32 +8", out, cyc, cus);
    printf("rc=%d\n", (int)hipGetLastError());
    return 0;
}
