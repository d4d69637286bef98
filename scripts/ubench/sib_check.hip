// Standalone A/B of one FD kernel configuration against the production b40
// configuration on the same field (no library, no finish): histograms summed
// over the copies on the host, near-miss counts compared, times printed.
// Build (CPU side):  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DXM=2 -DXWG=768
//   -DXVD=2049 -DXLG=-1 scripts/ubench/sib_check.hip -o scripts/ubench/sib_check
// Run: sib_check START COUNT [REPS]
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "../../nice_amd/csrc/fd2_kernel.hpp"

using namespace nice;
using namespace nice::fd2;
std::atomic<uint32_t> nice::fd2::g_force_sib_stride{0};  // (defined by fd2_detailed.hip in the library)
#ifndef XLG
#define XLG -1
#endif
#ifndef XPROBE
#define XPROBE 0
#endif
// XB / XND / XNE / XNE2: base and limb combo (default b40 4 8 5)
#ifndef XB
#define XB 40
#define XND 4
#define XNE 8
#define XNE2 5
#endif
// XREF 0: the regular big-field kernel of the base (b40: the round-4
// kernel); 1: the round-5 production b40 sibling kernel
#if defined(XREF) && XREF == 1
using Ref = Cfg<40, 4, 8, 5, 0, 512, 4097, 100, 0, 3>;
#elif !defined(XREFVD)
#define XREF 0
using Ref = Cfg<XB, XND, XNE, XNE2, 0, big_wg(XB), valu_limbs_big(XB, XND, XNE)>;
#endif
#ifndef XPERS
#define XPERS 0
#endif
// XREFVD: the reference is the variant's own configuration at VD = XREFVD
#ifdef XREFVD
#undef XREF
#define XREF 2
using Ref = Cfg<XB, XND, XNE, XNE2, 0, XWG, XREFVD, XLG, XPERS, XM>;
#endif
using Var = Cfg<XB, XND, XNE, XNE2, XPROBE, XWG, XVD, XLG, XPERS, XM>;

template <class P>
static double run(unsigned __int128 start, u64 count, std::vector<u64> &hist, u32 &nmiss, int reps) {
    u64 *d_hist;
    u32 *d_count;
    u64 *d_n;
    u32 *d_u;
    hipMalloc(&d_hist, kHistCopies * 129 * 8);
    hipMalloc(&d_count, 4);
    hipMalloc(&d_n, (1 << 20) * 16);
    hipMalloc(&d_u, (1 << 20) * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        hipMemset(d_hist, 0, kHistCopies * 129 * 8);
        hipMemset(d_count, 0, 4);
        DetailedLaunch p{};
        p.start_lo = (u64)start;
        p.start_hi = (u64)(start >> 64);
        p.count = count;
        p.base = XB;
        p.cutoff = (u32)(XB * 9 / 10);  // floor(b * 0.9) (number_stats.rs:15-17; exact for these bases)
        p.hist = d_hist;
        p.hist_copies = kHistCopies;
        p.out = NumOut{d_n, d_u, d_count, 1u << 20};
        p.fin = FieldFinish{nullptr, nullptr, 0, 0};
        hipEventRecord(e0, 0);
        hipError_t e = launch_cfg<P>(p, cus, 0);
        hipEventRecord(e1, 0);
        if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            printf("launch failed: %s\n", hipGetErrorString(e));
            exit(1);
        }
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    std::vector<u64> h(kHistCopies * 129);
    hipMemcpy(h.data(), d_hist, h.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&nmiss, d_count, 4, hipMemcpyDeviceToHost);
    hist.assign(129, 0);
    for (u32 c = 0; c < kHistCopies; c++)
        for (int b = 0; b < 129; b++) hist[b] += h[c * 129 + b];
    hipFree(d_hist);
    hipFree(d_count);
    hipFree(d_n);
    hipFree(d_u);
    return best;
}

int main(int argc, char **argv) {
    // START in decimal, up to 128 bits (b80 fields start above 2^64)
    unsigned __int128 start = 1916284264916ull;
    if (argc > 1) {
        start = 0;
        for (const char *c = argv[1]; *c; c++) start = start * 10 + (unsigned)(*c - '0');
    }
    const u64 count = argc > 2 ? strtoull(argv[2], 0, 10) : 100000000ull;
    const int reps = argc > 3 ? atoi(argv[3]) : 3;
    std::vector<u64> h0, h1;
    u32 m0 = 0, m1 = 0;
    // alternate the two kernels (a best-of per kernel over `reps` rounds),
    // so clock drift during the run charges both alike
    double t0 = 1e30, t1 = 1e30;
    for (int r = 0; r < reps; r++) {
        t0 = std::min(t0, run<Ref>(start, count, h0, m0, 1));
        t1 = std::min(t1, run<Var>(start, count, h1, m1, 1));
    }
    u64 s0 = 0, s1 = 0;
    int bad = 0;
    for (int b = 0; b < 129; b++) {
        s0 += h0[b];
        s1 += h1[b];
        if (h0[b] != h1[b]) {
            if (bad < 8) printf("bin %d: ref %llu var %llu\n", b, (unsigned long long)h0[b], (unsigned long long)h1[b]);
            bad++;
        }
    }
    printf("B=%d REF=%d PROBE=%d M=%d WG=%d VD=%d LG=%d start=%llu count=%llu: ref %.1f us var %.1f us, sums %llu %llu, "
           "near-miss %u %u, %s\n",
           XB, XREF, XPROBE, XM, XWG, XVD, XLG, (unsigned long long)start, (unsigned long long)count, t0 * 1e3, t1 * 1e3,
           (unsigned long long)s0, (unsigned long long)s1, m0, m1, bad || m0 != m1 ? "MISMATCH" : "match");
    return bad || m0 != m1;
}
