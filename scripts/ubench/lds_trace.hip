// LDS lookups on the FD kernel's REAL index pattern (gfx950), per table
// layout: VERDICT r03 item 4 asks whether a bank swizzle of the 16-byte pair
// table (entry i stored at i ^ f(i >> 4) in its low 4 bits) cuts the b65-80
// kernels' conflicts.  scripts/ubench/lds_trace_gen.py writes, per layout,
// the stored positions the kernel's lookups would hit: per wave, 64 lanes
// `chunk` numbers apart, every looked-up limb of n^2 and n^3.  Here each wave
// loads its trace row into registers and issues those ds_read_b128 lookups
// ITERS times (16 waves per CU, the b80 kernel's occupancy); the CU's s_memtime
// span (first wave's start to last wave's end) per wave-lookup is what the
// layout costs on that pattern.  (Round 4's first version timed wave 0 alone:
// the oldest wave is favoured by the LDS arbiter and finishes well before the
// others, so for the 2-cycle ds_read_b64 it read about 2.3x too fast; both
// figures are printed.)
//   hipcc --offload-arch=gfx950 -O3 -o lds_trace lds_trace.hip && ./lds_trace trace.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ITERS 256
constexpr int MAXL = 32;          // looked-up limbs per step (b80: 24)
constexpr uint32_t NE = 6400 + 16;

// Read styles: 0 one ds_read_b128 of a 16-byte entry (production b65-80);
// 1 ds_read_b64 of an 8-byte entry (digits 0-63) + ds_read_b32 of a 4-byte
// entry (digits 64-) in a second region (the split layout); 2 ds_read_b64 of
// an 8-byte entry only (the b40-64 lookup); 3 ds_read_b64 + ds_read_u16.
template <int NL, int MODE>
__global__ void __launch_bounds__(1024) kern(const uint16_t *trace, uint32_t waves, uint32_t *out, uint64_t *cyc) {
    // cyc[2 * (blockIdx.x * 16 + wave)] = start, [+1] = end (s_memtime)
    __shared__ __attribute__((aligned(16))) unsigned char t[NE * 16];
    for (uint32_t i = threadIdx.x; i < NE * 4; i += blockDim.x) ((uint32_t *)t)[i] = i * 2654435761u;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) % waves;
    uint32_t a[NL];
#pragma unroll
    for (int l = 0; l < NL; l++) a[l] = (uint32_t)trace[((size_t)w * NL + l) * 64 + lane] * (MODE == 0 ? 16 : 8);
    __syncthreads();
    uint32_t m0 = 0, m1 = 0, m2 = 0;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        // the addresses pass through an empty asm every iteration: the
        // compiler cannot hoist the (loop-invariant) lookups out of the loop
#pragma unroll
        for (int l = 0; l < NL; l++) asm volatile("" : "+v"(a[l]));
#pragma unroll
        for (int l = 0; l < NL; l++) {
            if constexpr (MODE == 0) {
                const uint4 v = *(const uint4 *)(t + a[l]);
                m0 |= v.x;
                m1 |= v.y;
                m2 |= v.z;
                asm volatile("" ::"v"(v.w));
            } else {
                const uint2 v = *(const uint2 *)(t + a[l]);
                m0 |= v.x;
                m1 |= v.y;
                if constexpr (MODE == 1) m2 |= *(const uint32_t *)(t + NE * 8 + a[l] / 2);
                if constexpr (MODE == 3) m2 |= *(const uint16_t *)(t + NE * 8 + a[l] / 4);
            }
        }
        asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = m0 ^ m1 ^ m2;
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 16 + threadIdx.x / 64)] = c0;
        cyc[2 * (blockIdx.x * 16 + threadIdx.x / 64) + 1] = c1;
    }
}

struct Cost {
    double span, wave0;  // LDS cycles per wave-lookup per CU: CU span, wave 0 alone
};

template <int NL, int MODE>
static Cost run(const uint16_t *d, uint32_t waves, uint32_t *out, uint64_t *cyc, uint64_t *hc, int cus) {
    Cost best = {1e30, 1e30};
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL((kern<NL, MODE>), dim3(cus), dim3(1024), 0, 0, d, waves, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(hc, cyc, (size_t)cus * 32 * 8, hipMemcpyDeviceToHost);
        double span = 0, w0 = 0;
        for (int i = 0; i < cus; i++) {
            uint64_t lo = ~0ull, hi = 0;
            for (int w = 0; w < 16; w++) {
                lo = hc[2 * (i * 16 + w)] < lo ? hc[2 * (i * 16 + w)] : lo;
                hi = hc[2 * (i * 16 + w) + 1] > hi ? hc[2 * (i * 16 + w) + 1] : hi;
            }
            span += (double)(hi - lo);
            w0 += (double)(hc[2 * i * 16 + 1] - hc[2 * i * 16]);
        }
        const double per = cus * 16.0 * ITERS * NL;  // 16 waves share the CU's LDS pipe
        best.span = span / per < best.span ? span / per : best.span;
        best.wave0 = w0 / per < best.wave0 ? w0 / per : best.wave0;
    }
    return best;
}

template <int NL>
static void run_all(const char *name, const uint16_t *d, uint32_t waves, uint32_t *out, uint64_t *cyc,
                    uint64_t *hc, int cus) {
    const Cost c[4] = {run<NL, 0>(d, waves, out, cyc, hc, cus), run<NL, 1>(d, waves, out, cyc, hc, cus),
                       run<NL, 2>(d, waves, out, cyc, hc, cus), run<NL, 3>(d, waves, out, cyc, hc, cus)};
    printf("%-12s b128 %6.2f | b64+b32 %6.2f | b64 %6.2f | b64+u16 %6.2f  LDS cycles per wave-lookup per CU "
           "(CU span)\n", name, c[0].span, c[1].span, c[2].span, c[3].span);
    printf("%-12s b128 %6.2f | b64+b32 %6.2f | b64 %6.2f | b64+u16 %6.2f  (wave 0 alone)\n", "", c[0].wave0,
           c[1].wave0, c[2].wave0, c[3].wave0);
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t hdr[6];
    if (fread(hdr, 4, 6, f) != 6) return 2;
    const uint32_t nlay = hdr[0], waves = hdr[1], nl = hdr[2];
    if ((nl != 24 && nl != 12) || hdr[3] > 6400) {
        fprintf(stderr, "this build handles 12 or 24 limbs of a <= 6400-entry table\n");
        return 2;
    }
    printf("base %u chunk %u: %u waves x %u looked-up limbs (best of 3, s_memtime)\n", hdr[4], hdr[5], waves, nl);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t per = (size_t)waves * nl * 64;
    uint16_t *h = (uint16_t *)malloc(per * 2), *d;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&d, per * 2);
    (void)hipMalloc(&out, (size_t)cus * 1024 * 4);
    (void)hipMalloc(&cyc, (size_t)cus * 32 * 8);
    uint64_t *hc = (uint64_t *)malloc((size_t)cus * 32 * 8);
    for (uint32_t L = 0; L < nlay; L++) {
        char name[17] = {0};
        if (fread(name, 1, 16, f) != 16 || fread(h, 2, per, f) != per) return 2;
        (void)hipMemcpy(d, h, per * 2, hipMemcpyHostToDevice);
        if (nl == 24) run_all<24>(name, d, waves, out, cyc, hc, cus);
        else run_all<12>(name, d, waves, out, cyc, hc, cus);
    }
    printf("rc=%d\n", (int)hipGetLastError());
    return 0;
}
