// fd2_kernel.hpp -- production finite-difference detailed kernel (gfx950):
// the device code and its per-instantiation launcher.  Instantiated per base
// by fd2_part*.hip (compiled in parallel), driven by fd2_detailed.hip.
//
// Computes exactly what process_range_detailed does (common/src/
// client_process.rs:150-191: per n the unique-digit count of n^2 and n^3 in
// base b, histogrammed, plus the near-miss list) for segments inside a base's
// valid range, where n^2 and n^3 have fixed digit counts D2 + D3 = b.  It
// replaces the reference's detailed_kernel (common/src/cuda/nice_kernels.cu:
// 486-531); the design is MI355X-first, not a translation:
//
//  * Each lane walks a contiguous chunk n0 .. n0+len-1 (len <= B = b^2).
//    n^2 and n^3 live in radix-B limbs (one limb = two base-b digits) and step
//    by finite differences, never dividing:
//        S = n^2 += D1,            D1 = 2n + 1 += 2
//        C = n^3 += 3 S + N3,      N3 = 3n + 1 += 3
//    (the cube's increment 3n^2 + 3n + 1 is rebuilt from the square's limbs,
//    so no second-order difference state is carried).  A C-limb sum is < 5B:
//    its carry (0..4) is one multiply-high (two for b80).
//  * Limb counts are template parameters picked by the host per segment
//    (ND, NE = limbs of D1 = 2e+1 and E1 = 3e^2+3e+1 at the segment's end,
//    NE2 of 6e+6 kept for the layout checks), so a step touches exactly the
//    limbs that can change: S limbs [0, ND], C limbs [0, NE].  Carries out of
//    those (probability ~1/B per step) and the limb-0 wraps of D1 / N3 take a
//    rare, wave-uniform branch.
//  * The per-step limbs are stored SCALED by the mask-table entry size ES and
//    BIASED by 2^T - B: the stored word is directly the LDS byte address of the
//    limb's digit-pair mask (no address arithmetic), and the radix-B carry is
//    bit T + log2(ES) of the sum (one shift, one v_mad_i32_i24 to reduce).
//  * n^2 mod B and n^3 mod B depend only on n mod B, so limb 0 of S and of C
//    share ONE lookup in a low-digit table indexed by r = n0 mod B + i (< 2B:
//    the table has 2B entries, so r never wraps inside a chunk).
//  * Histogram: per-thread counters in LDS for a window of W unique counts
//    around the distribution's bulk (b40: 17..32 holds all but 7e-5 of n); the
//    rare counts outside the window (and every near-miss, which always lies
//    above the window) take a divergent branch to a per-workgroup LDS
//    histogram and the global near-miss list.  One flush per workgroup.
//
//  * Grid: rounds of workgroups, one chunk per lane, where two or more
//    workgroups share a CU (b40); one round of resident 1024-thread
//    workgroups whose waves pull strided 64-unit batches where one workgroup
//    fills a CU (Cfg::PERS, b42..80 fields of >= 2 rounds).
//
// The kernel is issue-bound on VALU and LDS together: b40 per n is 13 random
// 8-byte LDS lookups (≈5 LDS cycles each per wave) and ≈78 VALU instructions
// per wave-step; see DESIGN.md §3.1 for the cycle model and the measured
// roofline.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <tuple>
#include <mutex>
#include <type_traits>

#include "host_math.hpp"
#include "kernels.h"
#include "nice_device.hpp"
#include "probe.hpp"

namespace nice {
namespace fd2 {

constexpr int log2ceil(unsigned v) { int t = 0; while ((1u << t) < v) t++; return t; }
constexpr int ilog2(unsigned v) { int t = 0; while ((2u << t) <= v) t++; return t; }

// Exactness of the digit split q = mulhi(ES v, m) = v / b over v < b^2.
constexpr bool split_exact(unsigned base, unsigned es, unsigned long long m) {
    for (unsigned v = 0; v < base * base; v++)
        if (((unsigned long long)es * v * m) >> 32 != v / base) return false;
    return true;
}

// Tuning / bottleneck-probe knobs read from the environment exist only in
// the probe build (make -C nice_amd probe -> libnice_hip_probe.so, used by
// scripts/); the product library ignores the environment and always runs the
// production configuration.

// Histogram window [W0, W0 + W) per base: where the unique-count
// distribution of in-range n lives (scripts/fd2_windows.py, 40 000 samples
// per base: at most 6e-4 of n fall outside; b40/50/80 keep their measured
// production windows).  W0 + W <= cutoff + 1: every near-miss is outside.
constexpr int window_w(int b) {
    return b == 40 ? 15 : b == 50 ? 18 : b == 80 ? 28 : b <= 45 ? 15 : b <= 61 ? 18 : b <= 70 ? 20 : 28;
}
constexpr int window_w0(int b) {
    switch (b) {
    case 40: return 18;
    case 42: return 19;
    case 43: return 20;
    case 44: case 45: case 47: return 21;
    case 48: return 22;
    case 49: return 23;
    case 50: return 21;
    case 52: return 24;
    case 53: return 25;
    case 54: case 55: return 26;
    case 57: return 27;
    case 58: return 28;
    case 59: case 60: return 29;
    case 62: case 63: return 30;
    case 64: return 31;
    case 65: return 32;
    case 67: return 33;
    case 68: return 34;
    case 80: return 33;
    default: return b * 61 / 100 - window_w(b) / 2;
    }
}

// Waves per SIMD whose VGPR budget (512 / waves) holds a base's lane state
// without spilling in the step loop: the stepped and cached limbs of n^2, n^3,
// 2n+1, 3n+1 plus the mask words, R = NS + NC + 2 NX + 1 + MW registers, and
// about as many temporaries.  b40 (R = 31) just fits 64 VGPRs (8 waves);
// R = 35..38 (b42..50) needs ~80 (6 waves), R <= 46 (b52..60) ~96 (5),
// wider bases 128 (4).
constexpr int state_regs(int base) {
    const int k = base / 5, r5 = base % 5;
    const int d2 = r5 == 0 ? 2 * k : (r5 == 4 ? 2 * k + 2 : 2 * k + 1);
    const int d3 = r5 == 0 ? 3 * k : (r5 == 2 ? 3 * k + 1 : 3 * k + 2);
    const int dn = r5 == 0 ? k : k + 1;
    return (d2 + 1) / 2 + (d3 + 1) / 2 + 2 * ((dn + 1) / 2) + 1 + (base + 31) / 32;
}
constexpr int state_waves(int base) {
    const int r = state_regs(base);
    return r <= 31 ? 8 : (r <= 38 ? 6 : (r <= 46 ? 5 : 4));
}

// In-range n fits 64 bits: BASE^DN <= 2^64 (DN digits).
constexpr bool fits64(unsigned base, int digits) {
    unsigned long long v = 1;
    for (int i = 0; i < digits; i++) {
        if (v > ~0ull / base) return false;
        v *= base;
    }
    return true;
}

// Limbs decoded by VALU instead of a table lookup (Cfg::VD: top C limbs +
// 16 x top S limbs), per base where the lookups' bank conflicts outweigh the
// VALU work: the best of VD 0/1/2/3/17 on the 1e9 field at the range start
// (scripts/vd_sweep_all.py, profiles/r02/vd_sweep_all.log), kept where it
// gains over ~1 %; without a low-digit table also limb 0 (VD & 256,
// profiles/r02/vd_sweep_low.log).  b64: 6.31 -> 4.25 ms (its table index
// n^2 mod 4096 keeps few residues mod 32, so lookups pile onto few banks);
// b45 2.60 -> 2.41; b60 3.79 -> 3.41; b63 3.96 -> 3.70; b68 7.42 -> 6.87;
// b80 8.22 -> 7.46; b40 neutral (r01).  Re-swept on the persistent grid
// (profiles/r03/vd_sweep_persistent.log): b55 0 -> 1 (2.91 -> 2.87 ms), b58
// 1 -> 2 (3.08 -> 3.00); every other base within ~1 % of its choice.
constexpr int valu_limbs(int base) {
    switch (base) {
    case 43: case 44: case 45: case 48: case 50: case 54: case 55: return 1;
    case 53: case 58: case 65: return 2;
    case 67: case 68: case 80: return 256;  // limb 0 by VALU
    // b59..64: the low-digit table with its carries in a side table (VD &
    // 1024, Cfg::LSDX), then the best top limbs by VALU: b59 3.31 -> 3.01 ms,
    // b60 3.39 -> 3.18, b62 3.49 -> 3.35, b63 3.71 -> 3.59, b64 4.17 -> 4.13
    // (profiles/r03/lsdx_sweep.log)
    case 59: case 63: case 64: return 1024 + 2;
    case 60: return 1024 + 17;
    case 62: return 1024 + 1;
    default: return 0;
    }
}

// Fields of >= 1e7 on the three-mask-word bases (b65..80, the persistent
// 1024-thread kernel): limb 0 by VALU and the VALU-decoded C limbs just BELOW
// the top stepped one (VD & 2048, Cfg::VDB).  The top stepped limb only takes
// carries, so across a wave its lookup is nearly a broadcast (4 LDS cycles on
// b80's index pattern against 11-12 for the limbs below it,
// scripts/ubench/lds_trace_gen.py), and decoding it by VALU saved little;
// decoding the limbs below it saves full-price lookups.  How many: per limb
// layout (the segment's ND, NE), from interleaved A/B sweeps over 1e9 fields
// at several points of each range with the select-free decode of or_valu and
// the one-multiply C carry (profiles/r04/vd_below_top.log): three, four where
// b80's n^3 has 17 limbs.  Against the round-3 kernels: b80 1e9 6.84 -> 6.24
// ms at the range start, b65 5.97 -> 5.43, b67 5.94 -> 5.64, b68 6.48 -> 5.57.
// The two-word bases (co-bound by VALU and LDS) move their VALU-decoded
// limbs below the top where that measured faster at both points of the
// range: b50 -1.1 / -2.2 %, b53 -1.1 / -1.4, b60 -1.2 / -1.7 (same VALU work,
// cheaper lookups); elsewhere within +-1 % or mixed, unchanged.  b40 (no
// VALU-decoded limbs before) decodes one C limb below the top on its 8-limb
// n^3 layouts (the first ~45 % of the range, the extra-large benchmark field
// among them): 2.03 -> 1.98 ms at the range start, 2.74 -> 2.62 at 0.1, 2.22
// -> 2.17 at 0.3, and it beats one or two more decoded limbs at every point
// checked in 0.02..0.35; on the 9-limb layout it lost 0-2 % and stays as it
// was (profiles/r04/vd_b40.log).
constexpr int valu_limbs_big(int base, int nd, int ne) {
    if (base == 40) return ne == 8 ? 2048 | 1 : 0;
    if (base == 50 || base == 53 || base == 60) return valu_limbs(base) | 2048;
    if ((base + 31) / 32 != 3) return valu_limbs(base);
    if (base == 80 && ne == 17) return 256 | 2048 | 4;
    return 256 | 2048 | 3;
}

// LDS bytes / waves per SIMD of a base's kernel at a workgroup size (the
// formulas of Cfg, evaluated without instantiating it).
constexpr int lds_bytes(int base, int wg) {
    const int mw = (base + 31) / 32, b2 = base * base;
    const bool split = mw == 3 && (valu_limbs(base) & 512) != 0;
    const int es = mw == 1 ? 4 : (mw == 2 || split ? 8 : 16);
    int t = 0;
    while ((1 << t) < b2) t++;
    const int ebt = es * ((1 << t) - b2);
    if (split) {  // [OUTL | X2 | X1 | window rows] (Cfg::SPLIT)
        const int a = (4 * (base + 1) + 15) / 16 * 16, h = (ebt / 2 + 15) / 16 * 16;
        const int t2 = a > h ? a : h;
        const int tb0 = (t2 + 4 * b2 + 15) / 16 * 16, tbe = (ebt + 15) / 16 * 16;
        const int tb = tb0 > tbe ? tb0 : tbe;
        return (tb + b2 * es + 15) / 16 * 16 + window_w(base) * (wg / 2) * 4;
    }
    const int tb0 = (window_w(base) * (wg / 2) * 4 + 4 * (base + 1) + 15) / 16 * 16;
    const int tb = tb0 >= ebt ? tb0 : (ebt + 15) / 16 * 16;
    const int db = base - 32;
    const bool lsd_w1 = mw == 2 && db > 0 && db + (db > 20 ? 4 : 10) <= 30;
    const bool lsdx = mw == 2 && db > 0 && !lsd_w1 && (valu_limbs(base) & 1024) != 0;
    return tb + (b2 * es + 15) / 16 * 16 + (lsd_w1 || lsdx ? (2 * b2 * es + 15) / 16 * 16 : 0) +
           (lsdx ? (2 * b2 + 15) / 16 * 16 : 0);
}
// Waves per SIMD actually resident: the LDS and VGPR caps, in whole
// workgroups (a workgroup puts wg / 256 waves on each SIMD).
constexpr int waves_at(int base, int wg) {
    const int lds = (163840 / lds_bytes(base, wg)) * (wg / 64) / 4;
    const int cap = lds < state_waves(base) ? lds : state_waves(base);
    return cap / (wg / 256) * (wg / 256);
}
// Workgroup size for fields >= 1e7 in rounds of workgroups: the kernels are
// bound by LDS lookups and want as many in flight as fit, so the size with
// more waves per SIMD under the LDS budget wins, 512 on a tie.  Measured on
// the first three bases: b40 two 1024-thread workgroups per CU (8 waves/SIMD)
// 2.38 ms vs 2.43 for three 512-thread ones (6 waves,
// profiles/r01/fd2_wg_sweep2.log); b80 one 1024-thread workgroup (4 waves)
// 8.47 ms vs 9.37 at 512 (2 waves, profiles/r01/b80_wg_sweep.log); b50 4
// waves either way, 512 kept.
constexpr int rounds_wg(int base) { return waves_at(base, 1024) > waves_at(base, 512) ? 1024 : 512; }
// With the persistent grid (Cfg::PERS) a tie goes to 1024: one 1024-thread
// workgroup per CU walking strided batches beats two 512-thread ones in
// rounds on every such base (b42..50 -3..-10 %, b59..64 -2..-5 % per 1e9,
// profiles/r03/pers_sweep_wg1024.log).
constexpr int big_wg(int base) { return waves_at(base, 1024) >= waves_at(base, 512) ? 1024 : 512; }

// Persistent grid by default where the kernel holds ONE workgroup per CU
// (b52..58, b65..68, b80 at 1024 threads): with two or more, a workgroup's
// draining tail overlaps another's steps, and rounds of workgroups win
// (profiles/r03/pers_sweep_all.log: b52..58 -12..-15 %, b65..68 / b80 -6..-10 %
// per 1e9; b42..50 and b59..64, two workgroups per CU, +1..+6 %).
constexpr bool one_wg_per_cu(int base, int wg) { return waves_at(base, wg) == wg / 256; }

// Sibling lanes (Cfg::SIB = M > 1): registers per wave for M lanes' state
// (the shared limb-1 state once, the upper limbs of every sibling).
constexpr int sib_waves(int base, int m) { return m <= 1 ? state_waves(base) : (m <= 3 ? 6 : 5); }

template <int BASE_, int ND_, int NE_, int NE2_, int PROBE_ = 0, int WG_ = 512, int VD_ = 0, int LG_ = -1,
          int PERS_ = -1, int SIB_ = 1>
struct Cfg {
    static constexpr int BASE = BASE_;
    // Bottleneck probes (timing experiments only, results are wrong): 1 = no
    // table lookups (limb words OR-ed directly), 2 = no LDS histogram add,
    // 4 = no limb-1 lookups of S and C.
    static constexpr int PROBE = PROBE_;
    static constexpr int ND = ND_, NE = NE_, NE2 = NE2_;
    static constexpr int k = BASE / 5, r5 = BASE % 5;
    // Digit counts inside the valid range (base_range.rs:14-32).
    static constexpr int D2 = r5 == 0 ? 2 * k : (r5 == 4 ? 2 * k + 2 : 2 * k + 1);
    static constexpr int D3 = r5 == 0 ? 3 * k : (r5 == 2 ? 3 * k + 1 : 3 * k + 2);
    static constexpr int DN = r5 == 0 ? k : k + 1;
    static constexpr bool N64 = fits64(BASE, DN);  // init's u64 path
    // init's products in u64 columns (the 1024-thread kernels of the bases
    // whose n passes 64 bits: the register allocation that spills least);
    // elsewhere u32 columns (every FD base's column sums fit 32 bits:
    // static_assert below), normalised by 32-bit multiply-highs
    // VD & 65536 (probe A/B): the round-5 init -- init_digits on the 128-bit n
    // and u64 columns -- also on the 512-thread kernels of the bases whose n
    // passes 64 bits; the persistent-grid probe configurations at 512
    // threads (PERS_ = 1) take it too, their init being the round-5 one
    static constexpr bool OLDINIT = (VD_ & 65536) != 0;
    static constexpr bool C64 = !N64 && (WG_ >= 1024 || OLDINIT || PERS_ > 0);
    static constexpr int NS = cdiv(D2, 2), NC = cdiv(D3, 2), NX = cdiv(DN, 2);
    static constexpr int SL = ND + 1, CL = NE + 1, EL = NE2 + 1;  // per-step limbs
    static constexpr int S_TOPD = D2 - 2 * (NS - 1), C_TOPD = D3 - 2 * (NC - 1);
    static constexpr u32 B = (u32)BASE * BASE;
    static constexpr int T = log2ceil(B);
    static constexpr u32 BT = (1u << T) - B;
    static constexpr int MW = (BASE + 31) / 32;
    // VD & 512 (three mask words, b65..68 / b80): the digit-pair masks SPLIT
    // into X1, 8-byte entries of the digits 0..63 (ds_read_b64), and X2, 4-byte
    // entries of the digits 64.. (ds_read_b32), each table at its own entry
    // size, so both spread a lane group over all 64 banks: the stored limb
    // (scaled by 8) addresses X1 directly and X2 after one shift.  Probe
    // only: on the kernel's own b80 index pattern b64 + b32 costs 11.9 LDS
    // cycles per wave-lookup against 11.45 for one b128 of a 16-byte entry
    // (scripts/ubench/lds_trace.hip, profiles/r04/lds_trace.log), and the
    // kernel is 7 % slower with it.
    static constexpr bool SPLIT = MW == 3 && (VD_ & 512) != 0;
    static constexpr int ES = MW == 1 ? 4 : (MW == 2 || SPLIT ? 8 : 16);  // table entry stride (bytes)
    static constexpr int SH = T + ilog2(ES);                     // carry bit of a scaled limb
    static constexpr u32 ESB = ES * B, EBT = ES * BT;
    static constexpr int WG = WG_;
    // Target chunk (numbers per lane), see launch_cfg: a lane's init costs a
    // few steps, more for wider bases.
    static constexpr int TCHUNK = BASE <= 45 ? 80 : (BASE <= 58 ? 160 : 240);
    static constexpr int NBINS = BASE + 1;
    // Histogram window [W0, W0 + W): per-thread counters (u32, or u16 halves
    // shared by threads t and t + WG/2 when LDS is tight).
    static constexpr int W = window_w(BASE);
    static constexpr int W0 = window_w0(BASE);
    // Window counters: HQ per dword (u16 halves shared by threads t and
    // t + WG/2).
    static constexpr int HQ = 2;
    static constexpr int HROW = WG / HQ;  // counters per window row
    // (A branch-free window count -- every count to row min(uw, W), a dummy
    // row W, out-of-window counts recorded behind one wave-uniform branch --
    // measured 1 % slower on the b40 sibling kernel; skipping the
    // out-of-window work altogether, wrong by design, only 3 % faster:
    // profiles/r06/occupancy_ab.txt, bfw_uniform_branch_ab.log.)
    static constexpr int HIST_BYTES = W * HROW * 4;
    // Layout.  Default: [window rows | out-of-window bins (OUTL) | tables].
    // The digit-pair table needs at least EBT below it: S limbs are stored
    // biased by EBT and looked up at (TB - EBT) + S, an unsigned immediate
    // offset (b65-68: EBT exceeds the histogram region, so the table starts
    // later).  SPLIT: [OUTL | pad | X2 at T2 | X1 at TB | window rows]: S
    // limbs (biased by EBT) are looked up at (TB - EBT) + S in X1 and at
    // (T2 - EBT / 2) + S / 2 in X2, C limbs at TB + C and T2 + C / 2, all
    // unsigned 16-bit immediate offsets.
    static constexpr int T2 = SPLIT ? std::max((4 * NBINS + 15) / 16 * 16, ((int)EBT / 2 + 15) / 16 * 16) : 0;
    static constexpr int TB0 = SPLIT ? (T2 + 4 * (int)B + 15) / 16 * 16 : (HIST_BYTES + 4 * NBINS + 15) / 16 * 16;
    // VD & 32768 (small fields): no table image at all -- every limb decoded
    // by VALU, limb 0 included -- so no per-workgroup table DMA (the table
    // loads of a small field's hundreds of workgroups are fetched through the
    // fabric: b40 1e6 spends a median 1.5 us, b80 1e6 4.6 us, of each
    // workgroup's life on its state and tables; profiles/r06/stamps_r06.log)
    static constexpr bool NOTAB = (VD_ & 32768) != 0;
    static constexpr int TB = NOTAB || TB0 >= (int)EBT ? TB0 : ((int)EBT + 15) / 16 * 16;
    static constexpr int OUTL = SPLIT ? 0 : HIST_BYTES;  // per-workgroup histogram of out-of-window counts
    static constexpr int TC0 = (SPLIT ? T2 : TB) / 16 * 16;  // the table image starts here (16-byte copy)
    // Low-digit entry, word 1: digit bits [0, DB), then the carries and flags
    // of the step n -> n+1, all functions of n mod B (limb 0 of S, C, D1, N3
    // is never stored): the carry out of S limb 0 of S += D1 and the carry
    // (0..4) out of C limb 0 of C += 3S + N3; bit 30: D1 limb-0 wrap, bit 31:
    // N3 limb-0 wrap (top bits, so "any flag" is one compare).  Up to b52 the
    // carries sit pre-scaled by ES = 8 (a 4-bit field at F0 holding 8 * carry,
    // a 6-bit field at FC holding 8 * carry: one v_bfe each gives the scaled
    // carry); b53..58 leave room only for the bare carries (1 + 3 bits, one
    // extra multiply-add per step); wider bases have no low-digit table.
    static constexpr int DB = BASE - 32;
    static constexpr bool TIGHT = DB > 20;
    // VD & 16384 (small fields): no low-digit table, limb 0 stepped like the
    // others (a 12.8 KB instead of a 38.4 KB table image at b40)
    static constexpr bool LSD_W1 = MW == 2 && DB > 0 && DB + (TIGHT ? 4 : 10) <= 30 && (VD_ & (16384 | 32768)) == 0;
    // VD & 1024 (probe A/B, b59..64: word 1 of the entry is all digit bits):
    // the low-digit table with the carries and wrap flags in a side table of
    // bytes (bit 0 the S carry, bits 1-3 the C carry, bit 6 / 7 the D1 / N3
    // wraps), read at rc = TK + n mod B + i; r8 then holds TL too (TL can
    // pass the 16-bit immediate offset).
    static constexpr bool LSDX = MW == 2 && DB > 0 && !LSD_W1 && (VD_ & 1024) != 0;
    static constexpr bool LSD = LSD_W1 || LSDX;
    // (regions padded to 16 bytes: the image is copied in with 16-byte accesses)
    static constexpr int TL = TB + (NOTAB ? 0 : ((int)(B * ES) + 15) / 16 * 16);  // low-digit table (LDE entries)
    // Low-digit entries: a lane whose chunk starts at n reads n mod B + i, i <
    // chunk <= B, so 2B cover any chunk.  The sibling kernels of b46+ keep
    // B + 256 (their chunks are capped at 256, launch_sib): the table then
    // leaves room for two 512-thread workgroups per CU.
    static constexpr int LDE = (SIB_ > 1 && BASE_ >= 46) ? (int)B + 256 : 2 * (int)B;
    static constexpr int TK = TL + (LSD ? ((int)(LDE * ES) + 15) / 16 * 16 : 0);  // LSDX: carry bytes
    static constexpr int TEND = SPLIT ? (TB + (int)(B * ES) + 15) / 16 * 16
                                      : TK + (LSDX ? ((int)(2 * B) + 15) / 16 * 16 : 0);
    static constexpr int HB = SPLIT ? TEND : 0;  // window rows
    // Sibling lanes: each sibling's cached C limbs [CL, NC) -- read and
    // written only on the rare path -- as u16 per thread in LDS instead of
    // VGPRs (slot (j, k) of thread t at COLD + 2 ((j NCOLD + k) WG + t)).
    static constexpr int NCOLD = SIB_ > 1 ? NC - CL : 0;
    static constexpr int COLD = TEND;
    static constexpr int COLD_BYTES = (SIB_ * NCOLD * WG_ * 2 + 15) / 16 * 16;
    static constexpr int LDS_BYTES = SPLIT ? HB + HIST_BYTES : TEND + COLD_BYTES;
    static constexpr int TAB_BYTES = TEND - TC0;  // table image copied in per workgroup
    static constexpr int ZA = SPLIT ? TC0 : TB;   // zeroed per workgroup: [0, ZA) and [HB, LDS_BYTES)
    static constexpr int LO = LSD ? 1 : 0;  // first stored / looked-up limb
    static constexpr u32 DMASK = (1u << (DB > 0 && DB < 32 ? DB : 0)) - 1;
    static constexpr u32 FLAG_D1 = LSDX ? 1u << 6 : 1u << 30, FLAG_N3 = LSDX ? 1u << 7 : 1u << 31;  // any flag: w1 >= FLAG_D1
    static constexpr int F0 = LSDX ? 0 : TIGHT ? DB : (DB + 3) / 4 * 4;
    static constexpr int FC = LSDX ? 1 : TIGHT ? DB + 1 : F0 + 4;
    static constexpr int F0W = TIGHT ? 1 : 4, FCW = TIGHT ? 3 : 6;  // field widths
    // C += 3S + N3 (N3 = 3n + 1, NN limbs).  A C limb sum is < 5B, so its
    // carry (0..4) is a multiply-high by MAGIC = ceil(2^32 / (ES B)) (exact
    // over the range: static_assert).
    static constexpr int NN = NX + 1;
    static constexpr u32 DC = ES * B;
    static constexpr u32 MAGIC = (u32)(((1ull << 32) + DC - 1) / DC);
    static constexpr unsigned long long TMAX = (unsigned long long)ES * (5ull * B + 4);
    // One multiply-high by MAGIC is exact because t is a multiple of ES:
    // with t = ES u, u = qB + r and ES B MAGIC = 2^32 + e, the product is
    // q + r / B + u e / (B 2^32), whose floor is q while u e < 2^32 (b80:
    // u <= 5B + 4 = 32004, e = 98304).  Where even that fails, divide t / ES
    // first.  (Rounds 1-3 bounded t e < 2^32 instead, which sent the
    // 16-byte-entry bases b65..80 down the extra shift per C limb.)
    static constexpr bool C1 = ((unsigned long long)MAGIC * DC - (1ull << 32)) * (TMAX / ES) < (1ull << 32);
    static constexpr u32 MAGICB = (u32)(((1ull << 32) + B - 1) / B);
    // VALU-decoded limbs (no table lookup): VD % 16 of the top stepped C
    // limbs and VD / 16 of the top stepped S limbs.  Their two digits come
    // from one multiply-high by MAGIC_D = ceil(2^32 / (ES b)) and set their
    // bits with 64-bit shifts, trading VALU work (~6 ops at MW = 2, ~15 at
    // MW = 3) for one data-random (bank-conflicting) LDS read.
    static constexpr int VD = VD_;
    static constexpr int VDC = VD % 16, VDS = (VD / 16) % 16;
    // VD & 2048 (b65..80 probe): the VALU-decoded limbs sit just BELOW the
    // top stepped limb instead of at it.  The top stepped limb only takes
    // carries, so its value is nearly the same in every lane of a wave and
    // its lookup is nearly a broadcast (4 LDS cycles on b80's index pattern),
    // while the limbs below it cost 11-12 (scripts/ubench/lds_trace_gen.py).
    static constexpr int VDB = (VD & 2048) ? 1 : 0;
    // VD & 4096: the VALU-decoded limbs are the LOWEST ones above the
    // low-digit table's limb (LO + 1 ...): the most data-random indices, whose
    // lookups bank-conflict the most (sibling lanes, which have VALU to spare)
    static constexpr bool VDLOW = (VD & 4096) != 0;
    static constexpr bool vd_s(int q) {
        if (NOTAB) return true;
        return VDLOW ? (q > LO && q <= LO + VDS && q < SL) : (q >= SL - VDB - VDS && q < SL - VDB);
    }
    static constexpr bool vd_c(int q) {
        if (NOTAB) return true;
        return VDLOW ? (q > LO && q <= LO + VDC && q < CL) : (q >= CL - VDB - VDC && q < CL - VDB);
    }
    // Lookup groups: a scheduling barrier after every LG table lookups of a
    // step (0: none), so the compiler cannot hoist all of a step's LDS reads
    // ahead of their ORs -- with SPLIT's b64 + u16 pairs that held ~75 VGPRs
    // of loaded words at once and spilled the 1024-thread b80 kernel at its
    // 128-VGPR budget; the 16-byte layout spilled 52-64 bytes per lane there
    // too, and LG 8 removes it (b80 1e9 7.45 -> 7.31 ms, lg_sweep.log).
    // -1: the per-base default.
    // (sibling lanes: LG >= 100 -- the default -- pipelines the siblings'
    // lookups with the arithmetic, walk_sib_pipe; below 100 LG != 0 ends a
    // group after each sibling's lookups, LG > 1 after every LG of them too)
    static constexpr int LG = LG_ >= 0 ? LG_ : (SIB_ > 1 ? 100 : (MW == 3 && WG >= 1024 ? 8 : 0));
    // Persistent grid: one round of resident workgroups, each walking a
    // contiguous range of 64-unit batches that its waves pull from an LDS
    // counter as they finish (instead of one chunk per lane and many rounds
    // of workgroups, where a workgroup's CU idles down while its slowest
    // wave finishes: b54 1e9, one 1024-thread workgroup per CU, waited 61 us
    // of a 134 us workgroup life for it, profiles/r03/fd2_stamps_b54.log).
    // -1: the per-base default.
    // Sibling lanes: M = SIB numbers n0 + j B^2 per lane, in lock step.  n and
    // n + j B^2 agree mod B^2, so limbs 0 and 1 of n^2, n^3, 2n + 1 and 3n + 1
    // (radix B) are the same for all of them and so is the carry out of limb
    // 1 of every chain: the low-digit lookup, limb 1's two lookups and limb 1's
    // carry chains run once for the M numbers (walk_sib).  Rounds only.
    static constexpr int SIB = SIB_;
    static constexpr bool PERS = SIB_ > 1 ? false : PERS_ >= 0 ? PERS_ != 0 : (WG >= 1024 && one_wg_per_cu(BASE, WG));
    // the same kernel with rounds of workgroups (launch_cfg falls back to it
    // when the runtime occupancy or the field size does not suit PERS), at
    // the workgroup size rounds prefer
    using NoPers = Cfg<BASE_, ND_, NE_, NE2_, PROBE_, (PERS_ < 0 ? rounds_wg(BASE_) : WG_), VD_, LG_, 0>;
    // the production kernel without sibling lanes (segments shorter than a
    // few M B^2): the big-field workgroup size and VALU-decoded limbs; b46+
    // keep the persistent-grid default of their regular kernel (b52..55 1e8
    // fields: rounds of workgroups +8..+10 %, profiles/r05/sib_short_table_ab.log)
    using NoSib = std::conditional_t<(BASE_ >= 46),
                                     Cfg<BASE_, ND_, NE_, NE2_, PROBE_, big_wg(BASE_), valu_limbs_big(BASE_, ND_, NE_)>,
                                     Cfg<BASE_, ND_, NE_, NE2_, PROBE_, rounds_wg(BASE_), valu_limbs_big(BASE_, ND_, NE_), -1, 0>>;
    // lookup groups of walk_chunk (the sibling kernel's regular parts: none)
    static constexpr int LGW = SIB_ > 1 ? 0 : (LG_ >= 0 ? LG_ : (MW == 3 && WG_ >= 1024 ? 8 : 0));
    // VD & 256 (no low-digit table only): limb 0 of S and of C by VALU too --
    // n^2 mod B and n^3 mod B of a wave's lanes keep few residues mod 16, so
    // their lookups pile onto few bank quads
    static constexpr bool VDL = ((VD & 256) != 0 || NOTAB) && !LSD;
    static constexpr u32 MAGIC_D = (u32)(((1ull << 32) + ES * BASE - 1) / (ES * BASE));
    static_assert(VD == 0 || (MW >= 2 && split_exact(BASE, ES, MAGIC_D)), "VALU digit split");
    static_assert(VDC <= NE + 1 - (MW <= 2 ? 1 : 0) && VDS <= ND + 1 && (VD & ~0x1ffff) == 0 &&
                      ((VD & 1024) == 0 || LSDX),
                  "VALU-decoded limbs");
    // Waves per SIMD: what the LDS allows, capped by what the lane state
    // needs in VGPRs (the register budget is set to match, see state_waves).
    static constexpr int WPE0 = (163840 / LDS_BYTES) * (WG / 64) / 4;
    // (the small-field variants -- no low-digit table / no table -- at a
    // 128-VGPR budget: a field below 1e7 puts only a few waves on each SIMD)
    // (three mask words without a table: 256 VGPRs)
    static constexpr int WREG = (VD_ & 32768) && MW == 3 ? 2 : (VD_ & (16384 | 32768)) ? 4 : sib_waves(BASE, SIB);
    static constexpr int WPE1 = WPE0 < WREG ? WPE0 : WREG;
    // in whole workgroups: k = the workgroups a CU holds at WPE1 waves per
    // SIMD (a workgroup's WG / 64 waves spread over the 4 SIMDs), then the
    // waves per SIMD those k workgroups need (640-thread workgroups: 2.5 each)
    static constexpr int WGK = WPE1 * 256 / WG;
    static constexpr int WPE = WGK > 0 ? (WGK * (WG / 64) + 3) / 4 : (WG / 64 + 3) / 4;
    static_assert(WPE >= 1, "LDS: not even one workgroup fits");
    static_assert(SL < NS && CL < NC && EL <= NE, "FD layout needs cached high limbs");
    static_assert(ND <= NX + 1 && NE2 <= NX + 1 && NE <= NS + 1, "difference limb counts");
    static_assert(S_TOPD >= 1 && C_TOPD >= 1, "top limb");
    static_assert((NOTAB || TB >= (int)EBT) && (NOTAB || TB - (int)EBT < 65536) && (!LSD || LSDX || TL < 65536),
                  "LDS offsets");
    static_assert(!NOTAB || (!LSD && !SPLIT && SIB_ == 1), "table-free kernel: regular lanes, no low-digit table");
    static_assert(!PERS || N64 || C64, "persistent grid: init() only (init_at is the rounds path's)");
    static_assert(!SPLIT || (T2 >= (int)EBT / 2 && T2 < 65536 && T2 + 4 * (int)B <= TB && 4 * NBINS <= TC0 &&
                             ES == 8 && TB < 65536),
                  "split layout");
    static_assert(LDS_BYTES <= 163840, "LDS");
    static_assert(TB % 16 == 0 && TAB_BYTES % 16 == 0 && HB % 16 == 0, "16-byte table copy");
    static_assert(W0 >= 0 && W0 + W <= NBINS, "window");
    static_assert(!LSD || (ES == 8 && (LSDX ? TIGHT && FC + FCW <= 6 : FC + FCW <= 30)), "low-digit entry layout");
    static_assert(C1 || ((unsigned long long)MAGICB * B - (1ull << 32)) * (TMAX / ES) < (1ull << 32),
                  "C-limb carry magic");
    static_assert(NN <= SL && NE >= NS, "C += 3S + N3 layout");
    static_assert(3 * ES <= 64, "inline-constant multiplier");
    static_assert(SIB == 1 || (LSD && MW == 2 && LO == 1 && SL >= 3 && CL >= 3 && ND >= 2 && NN >= 2),
                  "sibling lanes share limb 1: low-digit-table bases only");
    static_assert((unsigned long long)NX * B * B + 2ull * B < (1ull << 32), "32-bit init columns");
};

// v_mad_u32_u24 with an inline-constant multiplier (LLVM otherwise splits it
// into v_mul_u32_u24 + v_add3_u32).
template <u32 K>
__device__ __forceinline__ u32 mad_u24(u32 a, u32 c) {
    static_assert(K <= 64, "inline constant");
    u32 r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "n"(K), "v"(c));
    return r;
}

// v_mad_i32_i24 with a scalar multiplier: a * K + c on 24-bit signed a, K
// (LLVM otherwise turns c - a * K into a v_mad_u64_u32, which does not issue
// at the full rate).
template <int K>
__device__ __forceinline__ u32 mad_i24s(u32 a, u32 c) {
    u32 r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(K), "v"(c));
    return r;
}

// v_bcnt_u32_b32 with a scalar accumulator: popcount(x) + acc.
__device__ __forceinline__ u32 bcnt_acc(u32 x, u32 acc) {
    u32 r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "s"(acc));
    return r;
}

template <class P>
struct State {
    u32 S[P::NS];    // n^2: limbs [0, SL) scaled+biased, [SL, NS) plain
    u32 C[P::NC];    // n^3: same with CL
    u32 D1[P::ND];   // scaled, plain
    u32 N3[P::NN];   // 3n + 1, scaled, limb i < SL offset by -3 ES BT
    u32 r8;          // low-digit table byte offset: ES * (n mod B + i) (LSDX: + TL)
    u32 rc;          // LSDX: carry byte address TK + n mod B + i
    u32 hi[P::MW];   // mask of the cached (rarely changing) limbs of S and C
};

template <class P>
__device__ __forceinline__ void or_entry(const unsigned char *p, u32 (&m)[P::MW]) {
    if constexpr (P::MW == 1) {
        m[0] |= *(const u32 *)p;
    } else if constexpr (P::MW == 2 || P::SPLIT) {
        uint2 v = *(const uint2 *)p;
        m[0] |= v.x;
        m[1] |= v.y;
    } else {
        uint4 v = *(const uint4 *)p;
        m[0] |= v.x;
        m[1] |= v.y;
        m[2] |= v.z;
        // Keep the 4th (zero) dword live so the load stays ds_read_b128: LLVM
        // would shrink it to ds_read_b96, which gfx950 serves in 8 lane groups
        // over 32 banks (8 cycles per wave) instead of 4 groups over 64 (4).
        asm volatile("" ::"v"(v.w));
    }
}

// OR the digit-pair mask of a stored limb into m: X1 (or the one table) at
// smem + OFF1 + stored; SPLIT also X2 at smem + OFF2 + stored / 2.
template <class P, int OFF1, int OFF2>
__device__ __forceinline__ void or_lookup(const unsigned char *smem, u32 stored, u32 (&m)[P::MW]) {
    or_entry<P>(smem + OFF1 + stored, m);
    if constexpr (P::SPLIT) m[2] |= *(const u32 *)(smem + OFF2 + (stored >> 1));
}

// End of a lookup group (Cfg::LG): the group's ORs are pinned here (the mask
// words pass through an empty asm, so LLVM cannot re-associate every OR of a
// step into one tree at its end) and no instruction crosses the point, so
// the group's loaded words are dead before the next group's reads issue.
template <class P>
__device__ __forceinline__ void lookup_group_end(u32 (&m)[P::MW]) {
#pragma unroll
    for (int w = 0; w < P::MW; w++) asm volatile("" : "+v"(m[w]));
    __builtin_amdgcn_sched_barrier(0);
}

// Digit bits of a scaled limb (vs = ES v, v < B) by VALU: the high digit by
// one multiply-high, the low one by a multiply-subtract, each bit set with a
// 64-bit shift (digits >= 64 land in mask word 2 at MW = 3).
template <class P>
__device__ __forceinline__ void or_valu(u32 vs, u32 (&m)[P::MW]) {
    const u32 q = __umulhi(vs, P::MAGIC_D);                        // high digit
    const u32 r = mad_i24s<-P::BASE>(q, vs / (u32)P::ES);          // low digit
    if constexpr (P::MW == 2) {
        const u64 bits = (1ull << q) | (1ull << r);
        m[0] |= (u32)bits;
        m[1] |= (u32)(bits >> 32);
    } else {
        // Digit d < 96 without compares or selects: a 64-bit shift by d
        // (the hardware takes d mod 64) is right in words 0 and 1 for d < 64,
        // and for d >= 64 leaves bit d - 64 in word 0 and nothing in word 1;
        // word 2's bit is bit 6 of d shifted by d mod 32, which is exactly that
        // stray bit, so XOR-ing it out of word 0 leaves every word right.
        const u64 bq = 1ull << (q & 63), br = 1ull << (r & 63);
        const u32 wq = __builtin_amdgcn_ubfe(q, 6, 1) << (q & 31), wr = __builtin_amdgcn_ubfe(r, 6, 1) << (r & 31);
        m[0] |= ((u32)bq ^ wq) | ((u32)br ^ wr);
        m[1] |= (u32)(bq >> 32) | (u32)(br >> 32);
        m[2] |= wq | wr;
    }
}

template <class P>
__device__ __forceinline__ void or_plain(const unsigned char *smem, u32 v, int digits, u32 (&m)[P::MW]) {
    if (digits == 2) {
        if constexpr (P::NOTAB) or_valu<P>(v * P::ES, m);
        else or_lookup<P, P::TB, P::T2>(smem, v * P::ES, m);
    } else {
#pragma unroll
        for (int w = 0; w < P::MW; w++) m[w] |= (v >> 5) == (u32)w ? 1u << (v & 31) : 0u;
    }
}

template <class P>
__device__ __forceinline__ void recompute_hi(State<P> &st, const unsigned char *smem) {
#pragma unroll
    for (int w = 0; w < P::MW; w++) st.hi[w] = 0;
#pragma unroll
    for (int i = P::SL; i < P::NS; i++) or_plain<P>(smem, st.S[i], i == P::NS - 1 ? P::S_TOPD : 2, st.hi);
#pragma unroll
    for (int i = P::CL; i < P::NC; i++) or_plain<P>(smem, st.C[i], i == P::NC - 1 ? P::C_TOPD : 2, st.hi);
}

// Radix-B normalisation of u64 column sums into M limbs (the value fits by the
// host's choice of limb counts; a carry past limb M-1 is dropped).
template <class P, int N, int M>
__device__ __forceinline__ void normalize64(const u64 (&acc)[N], u32 (&out)[M]) {
    u64 cy = 0;
#pragma unroll
    for (int t = 0; t < M; t++) {
        u64 v = (t < N ? acc[t] : 0) + cy;
        out[t] = (u32)(v % P::B);
        cy = v / P::B;
    }
}

// Radix-B normalisation of column sums into M limbs (the value fits by the
// host's choice of limb counts; a carry past limb M-1 is dropped).  A is u32
// where every column sum fits 32 bits (static_assert in init), else u64.
template <class P, class A, int N, int M>
__device__ __forceinline__ void normalize(const A (&acc)[N], u32 (&out)[M]) {
    A cy = 0;
#pragma unroll
    for (int t = 0; t < M; t++) {
        const A v = (t < N ? acc[t] : (A)0) + cy;
        cy = v / P::B;
        out[t] = (u32)(v - cy * P::B);
    }
}

// Radix-B digits X of n.
template <class P>
__device__ __forceinline__ void init_digits(u32 (&X)[P::NX], u64 n_lo, u64 n_hi) {
    constexpr u32 B = P::B;
    if constexpr (P::N64) {
        // In-range n fits 64 bits (b40 < 2^43, b50 < 2^57): two radix-B digits
        // per u64 division by B^2, the rest in 32 bits.
        (void)n_hi;
        constexpr u64 B2 = (u64)B * B;
        u64 v = n_lo;
#pragma unroll
        for (int j = 0; j < P::NX; j += 2) {
            const u64 q = v / B2;
            const u32 r = (u32)(v - q * B2);
            X[j] = r % B;
            if (j + 1 < P::NX) X[j + 1] = r / B;
            v = q;
        }
    } else {
        u32 w[4] = {(u32)n_lo, (u32)(n_lo >> 32), (u32)n_hi, (u32)(n_hi >> 32)};
#pragma unroll
        for (int j = 0; j < P::NX; j++) {
            u64 rem = 0;
#pragma unroll
            for (int q = 3; q >= 0; q--) {
                u64 cur = (rem << 32) | w[q];
                w[q] = (u32)(cur / B);
                rem = cur % B;
            }
            X[j] = (u32)rem;
        }
    }
}

// Plain (unscaled, unbiased) limbs of S = n^2, C = n^3, D1 = 2n + 1 and
// N3 = 3n + 1 from n's digits X, and the low-digit offsets.
template <class P>
__device__ __forceinline__ void init_plain(State<P> &st, const u32 (&X)[P::NX]) {
    // Column sums: at most min(NS, NX) products < B^2 plus a carry: 32 bits
    // (Cfg static_assert).
    using A = u32;
    if constexpr (P::C64) {
        // wide bases (b80: the 1024-thread kernel at the 128-VGPR cap): u64
        // columns, the layout whose register allocation spills least.
        st.r8 = X[0] * P::ES + (P::LSDX ? (u32)P::TL : 0u);
        st.rc = X[0] + (u32)P::TK;
        {
            u64 acc[2 * P::NX];
#pragma unroll
            for (int t = 0; t < 2 * P::NX; t++) acc[t] = 0;
#pragma unroll
            for (int i = 0; i < P::NX; i++)
#pragma unroll
                for (int j = 0; j < P::NX; j++) acc[i + j] += (u64)X[i] * X[j];
            normalize64<P>(acc, st.S);
        }
        {
            u64 acc[P::NS + P::NX];
#pragma unroll
            for (int t = 0; t < P::NS + P::NX; t++) acc[t] = 0;
#pragma unroll
            for (int i = 0; i < P::NS; i++)
#pragma unroll
                for (int j = 0; j < P::NX; j++) acc[i + j] += (u64)st.S[i] * X[j];
            normalize64<P>(acc, st.C);
        }
        {
            u64 acc[P::NX];
#pragma unroll
            for (int t = 0; t < P::NX; t++) acc[t] = 2ull * X[t] + (t == 0 ? 1 : 0);
            normalize64<P>(acc, st.D1);
        }
        {
            u64 acc[P::NX];
#pragma unroll
            for (int t = 0; t < P::NX; t++) acc[t] = 3ull * X[t] + (t == 0 ? 1 : 0);
            normalize64<P>(acc, st.N3);
        }
    } else {
        st.r8 = X[0] * P::ES + (P::LSDX ? (u32)P::TL : 0u);
        st.rc = X[0] + (u32)P::TK;
        {  // S = X^2
            A acc[2 * P::NX];
#pragma unroll
            for (int t = 0; t < 2 * P::NX; t++) acc[t] = 0;
#pragma unroll
            for (int i = 0; i < P::NX; i++)
#pragma unroll
                for (int j = 0; j < P::NX; j++) acc[i + j] += (A)X[i] * X[j];
            normalize<P>(acc, st.S);
        }
        {  // C = S * X
            A acc[P::NS + P::NX];
#pragma unroll
            for (int t = 0; t < P::NS + P::NX; t++) acc[t] = 0;
#pragma unroll
            for (int i = 0; i < P::NS; i++)
#pragma unroll
                for (int j = 0; j < P::NX; j++) acc[i + j] += (A)st.S[i] * X[j];
            normalize<P>(acc, st.C);
        }
        {  // D1 = 2n + 1
            A acc[P::NX];
#pragma unroll
            for (int t = 0; t < P::NX; t++) acc[t] = 2 * (A)X[t] + (t == 0 ? 1 : 0);
            normalize<P>(acc, st.D1);
        }
        {  // N3 = 3n + 1
            A acc[P::NX];
#pragma unroll
            for (int t = 0; t < P::NX; t++) acc[t] = 3 * (A)X[t] + (t == 0 ? 1 : 0);
            normalize<P>(acc, st.N3);
        }
    }
}

// Plain limbs -> the stepped representation (scaled by the entry stride,
// biased; limb 0 from the low-digit table where there is one).
template <class P>
__device__ __forceinline__ void init_scale(State<P> &st) {
    if constexpr (P::LSD) st.S[0] = st.C[0] = st.D1[0] = st.N3[0] = 0;  // from the table
#pragma unroll
    for (int i = 0; i < P::SL; i++) st.S[i] = (st.S[i] + P::BT) * P::ES;
#pragma unroll
    for (int i = 0; i < P::CL; i++) st.C[i] *= P::ES;  // unbiased: carries by multiply-high
#pragma unroll
    for (int i = 0; i < P::ND; i++) st.D1[i] *= P::ES;
#pragma unroll
    for (int i = 0; i < P::NN; i++) st.N3[i] = st.N3[i] * P::ES - (i < P::SL ? 3 * P::EBT : 0u);
}

// Lane state at n (every limb but the cached mask, which needs the tables:
// recompute_hi after them).
template <class P>
__device__ __forceinline__ void init(State<P> &st, u64 n_lo, u64 n_hi) {
    u32 X[P::NX];
    init_digits<P>(X, n_lo, n_hi);
    init_plain<P>(st, X);
    init_scale<P>(st);
}

// Radix-B digits of n = base + off from the host's digits of the launch part's
// first n (Fd2Args::xs / xt) and the lane's offset off < B^4: one u64
// division by B^2 and two u32 splits, then a carried add -- instead of the
// 128-bit n's NX x 4 u64 divisions by B (init_digits on the bases whose n
// passes 64 bits, where the radix conversion was most of a lane's init).
template <class P>
__device__ __forceinline__ void digits_plus(u32 (&X)[P::NX], const u32 *xb, u64 off) {
    constexpr u32 B = P::B;
    constexpr u64 B2 = (u64)B * B;
    const u64 q = off / B2;
    const u32 r = (u32)(off - q * B2), qq = (u32)q;
    const u32 o[4] = {r % B, r / B, qq % B, qq / B};
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < P::NX; i++) {
        const u32 t = xb[i] + (i < 4 ? o[i] : 0u) + c;
        c = t >= B ? 1u : 0u;
        X[i] = t - c * B;
    }
}

// init at base + off (base: the launch part whose digits the host passed).
// Bases whose in-range n fits 64 bits keep init(): their conversion is two
// u64 divisions.  So do the 1024-thread kernels (u64 columns): there the
// digits path measured 1.3 % slower on b80 1e9 (6.29 vs 6.21 ms), while the
// 512-thread small-field kernel gained 3.5 % on b80 1e6 (19.2 vs 19.9 us in
// the A/B harness; profiles/r06/init_ab_b80.log).
template <class P>
__device__ __forceinline__ void init_at(State<P> &st, const u32 *xb, u64 off, u64 n_lo, u64 n_hi) {
    if constexpr (P::N64 || P::C64) {
        (void)xb;
        (void)off;
        init<P>(st, n_lo, n_hi);
    } else {
        (void)n_lo;
        (void)n_hi;
        u32 X[P::NX];
        digits_plus<P>(X, xb, off);
        init_plain<P>(st, X);
        init_scale<P>(st);
    }
}

// +ES into scaled plain limbs [from, N) (rare path).
template <class P, int N>
__device__ __forceinline__ void carry_scaled(u32 (&x)[N], int from) {
    u32 c = 1;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (i < from) continue;
        u32 v = x[i] + c * P::ES;
        c = v >= P::ESB;
        x[i] = c ? 0u : v;
    }
}
// +1 into plain limbs [from, N) (rare path).
template <class P, int N>
__device__ __forceinline__ void carry_plain(u32 (&x)[N], int from) {
    u32 c = 1;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (i < from) continue;
        u32 v = x[i] + c;
        c = v == P::B;
        x[i] = c ? 0u : v;
    }
}

// +ES into N3 limbs [1, NN) (offset limbs, rare path).
template <class P>
__device__ __forceinline__ void carry_n3(State<P> &st) {
    u32 c = 1;
#pragma unroll
    for (int i = 1; i < P::NN; i++) {
        const u32 off = i < P::SL ? 3 * P::EBT : 0u;
        u32 v = st.N3[i] + off + c * P::ES;
        c = v >= P::ESB;
        st.N3[i] = (c ? 0u : v) - off;
    }
}

// Rare path: a limb-0 wrap of D1 / N3, or a carry out of the top stepped
// limb of S (tS >= 2^SH, biased) or C (tC >= ES B).  The top stepped limbs
// are left unreduced by step(): they only take carries, so they need
// reducing only here.
template <class P>
__device__ __forceinline__ void rare(State<P> &st, const unsigned char *smem, u32 d1w, u32 n3w, bool cS,
                                     bool cC) {
    if (d1w) carry_scaled<P>(st.D1, 1);
    if (n3w) carry_n3<P>(st);
    if (cS) {
        st.S[P::SL - 1] -= P::ESB;
        carry_plain<P>(st.S, P::SL);
    }
    if (cC) {
        st.C[P::CL - 1] -= P::DC;
        carry_plain<P>(st.C, P::CL);
    }
    if (cS | cC) recompute_hi<P>(st, smem);
}

// One FD step n -> n+1.  w1 = word 1 of the low-digit entry of n (LSD bases):
// limb 0 of every quantity lives in the table, so the chains start at limb 1
// with the table's carries.  The carry leaves each limb as c8 = ES * carry,
// (t >> T) & ES; the limb is reduced with one v_mad_i32_i24.  The top stepped
// limb of S and of C only ever receives a carry (D1 and 3S + N3 are shorter),
// so it is just compared: a carry out of it (~1/B per step) goes to rare().
template <class P>
__device__ __forceinline__ void step(State<P> &st, const unsigned char *smem, u32 w1) {
    constexpr u32 ES = P::ES;
    constexpr int L0 = P::LO;  // LSD bases: limb 0 lives in the low-digit table
    constexpr int CT = P::CL - 1, ST = P::SL - 1;  // top stepped limbs
    static_assert(CT >= P::NS && CT >= P::NN && ST >= P::ND, "top limbs take carries only");
    // C += 3S + N3 (old S), limbs L0 .. CL-1.  Unbiased scaled limbs; a limb
    // sum is < 5B, its carry (0..4) is a multiply-high.
    u32 cC = 0;
    if constexpr (P::LSD) cC = __builtin_amdgcn_ubfe(w1, P::FC, P::FCW);  // TIGHT: bare carry
#pragma unroll
    for (int i = L0; i < CT; i++) {
        u32 t;
        if (P::TIGHT && i == L0) t = mad_u24<ES>(cC, st.C[i]);  // scale the bare carry
        else t = st.C[i] + cC;
        // Past limb L0 the carry is c * ES from a multiply-high: keep C + c*ES
        // one v_lshl_add_u32 and add N3 with a plain v_add_u32 (LLVM would
        // otherwise emit v_lshlrev_b32 + v_add3_u32, ~2 issue cycles more).
        if (i > L0 && i < P::NN) asm("" : "+v"(t));
        if (i < P::NN) t += st.N3[i];
        else if (i < P::SL) t -= 3 * P::EBT;
        // + 3S as one v_mad_u32_u24 (limbs < 2^24)
        if (i < P::SL) t = mad_u24<3>(st.S[i], t);
        else if (i < P::NS) t = mad_u24<3 * ES>(st.S[i], t);
        const u32 c = P::C1 ? __umulhi(t, P::MAGIC) : __umulhi(t / ES, P::MAGICB);
        st.C[i] = t - c * P::DC;
        cC = c * ES;
    }
    st.C[CT] += cC;  // < DC + 4 ES: a carry out is at most 1
    // S += D1, limbs L0 .. SL-1 (biased: carry = bit T of t >> log2 ES).
    u32 cS = 0;
    if constexpr (P::LSD) cS = __builtin_amdgcn_ubfe(w1, P::F0, P::F0W);  // TIGHT: bare carry
#pragma unroll
    for (int i = L0; i < ST; i++) {
        u32 t;
        if (P::TIGHT && i == L0) t = mad_u24<ES>(cS, st.S[i] + (i < P::ND ? st.D1[i] : 0u));
        else t = st.S[i] + (i < P::ND ? st.D1[i] : 0u) + cS;
        cS = (t >> P::T) & ES;
        st.S[i] = t - cS * P::B;
    }
    st.S[ST] += cS;
    st.r8 += ES;
    if constexpr (P::LSDX) st.rc += 1;
    const bool topS = st.S[ST] >= (1u << P::SH), topC = st.C[CT] >= P::DC;
    if constexpr (P::LSD) {
        if (w1 >= P::FLAG_D1 || topS || topC)
            rare<P>(st, smem, w1 & P::FLAG_D1, w1 & P::FLAG_N3, topS, topC);
    } else {
        // limb 0 of D1 (+2) and N3 (+3, stored offset by -3 ES BT) step here
        st.D1[0] += 2 * ES;
        st.N3[0] += 3 * ES;
        const u32 d1w = st.D1[0] >= P::ESB, n3w = st.N3[0] + 3 * P::EBT >= P::ESB;
        if (d1w || n3w || topS || topC) {
            if (d1w) st.D1[0] -= P::ESB;
            if (n3w) st.N3[0] -= P::ESB;
            rare<P>(st, smem, d1w, n3w, topS, topC);
        }
    }
}

// Table image (the LDS bytes from TB on): digit-pair table, entry e = d1*b +
// d0 marks d0 and d1; low-digit table (LSD bases), entry r < 2B marks the two
// low digits of r^2 and of r^3 (mod B) plus the limb-0 carries and wraps.
template <class P>
__global__ void fd2_tables_kernel(unsigned char *tb) {
    const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P::B) return;
    u32 v[4] = {0, 0, 0, 0};
    auto mark = [&](u32 x) {
        u32 d0 = x % P::BASE, d1 = x / P::BASE;
        v[d0 >> 5] |= 1u << (d0 & 31);
        v[d1 >> 5] |= 1u << (d1 & 31);
    };
    auto put = [&](unsigned char *p) {
        if constexpr (P::ES == 4) *(u32 *)p = v[0];
        else if constexpr (P::ES == 8) *(uint2 *)p = make_uint2(v[0], v[1]);
        else *(uint4 *)p = make_uint4(v[0], v[1], v[2], v[3]);
    };
    mark(e);
    put(tb + (P::TB - P::TC0) + e * P::ES);
    if constexpr (P::SPLIT) *(u32 *)(tb + (P::T2 - P::TC0) + 4 * e) = v[2];  // X2: digits 64..
    if constexpr (P::LSD) {
        v[0] = v[1] = v[2] = v[3] = 0;
        const u32 B = P::B;
        const u32 s0 = (u32)((u64)e * e % B), c0 = (u32)((u64)s0 * e % B);
        mark(s0);
        mark(c0);
        const u32 d1 = (2 * e + 1) % B, n3 = (3 * e + 1) % B;
        u32 f = 0;
        f |= d1 + 2 >= B ? P::FLAG_D1 : 0u;                   // D1 limb-0 wrap
        f |= n3 + 3 >= B ? P::FLAG_N3 : 0u;                   // N3 limb-0 wrap
        const u32 sc = s0 + d1 >= B ? 1u : 0u, cc = (c0 + 3 * s0 + n3) / B;
        f |= (P::TIGHT ? sc : P::ES * sc) << P::F0;            // S  += D1 carry
        f |= (P::TIGHT ? cc : P::ES * cc) << P::FC;            // C += 3S + N3 carry
        if constexpr (P::LSDX) {
            tb[(P::TK - P::TC0) + e] = (unsigned char)f;
            tb[(P::TK - P::TC0) + e + P::B] = (unsigned char)f;
        } else {
            v[1] |= f;
        }
        put(tb + (P::TL - P::TC0) + e * P::ES);
        if ((int)(e + P::B) < P::LDE) put(tb + (P::TL - P::TC0) + (e + P::B) * P::ES);
    }
}

// The table image for this device and base, built on first use (the layout
// depends on the base only) and kept for the process.
template <class P>
static hipError_t fd2_tables(hipStream_t s, const uint4 **out) {
    if constexpr (P::TAB_BYTES == 0) {  // table-free kernel (Cfg::NOTAB)
        (void)s;
        *out = nullptr;
        return hipSuccess;
    }
    static std::mutex mu;
    static std::map<int, unsigned char *> have;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(mu);
    auto it = have.find(dev);
    if (it == have.end()) {
        unsigned char *t = nullptr;
        if ((e = hipMalloc(&t, P::TAB_BYTES)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(t, 0, P::TAB_BYTES, s)) != hipSuccess) return e;  // padding
        hipLaunchKernelGGL(fd2_tables_kernel<P>, dim3((P::B + 255) / 256), dim3(256), 0, s, t);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // other streams (contexts) of this device may read it next
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        it = have.emplace(dev, t).first;
    }
    *out = (const uint4 *)it->second;
    return hipSuccess;
}

// One launch covers a whole segment: blocks [0, main_blocks) walk `nunits`
// chunks of `chunk` numbers from `start`; the blocks after them take the
// < chunk numbers left over, one per lane, from `tail` (same code, chunk 1:
// every parameter stays wave-uniform, and no second launch is serialised
// behind the first).  With fin.out set, the launch also finishes the field:
// the last workgroup to retire sums the kHistCopies histogram copies into
// the caller's mapped result words and re-zeroes the state block, so a field
// is ONE launch instead of main + tail + epilogue (under several fields in
// flight each small launch waited for free CUs: 25-60 us apiece).
// Probe build: per-workgroup phase stamps (scripts/fd2_stamps.py).  When
// g_stamps (host, set by nice_probe_fd2_stamps) is non-null, thread 0 of each
// workgroup b < kStampGroups writes kStampWords words at stamps + kStampWords b:
// for each phase k the constant 100 MHz real-time counter (word 2k) and the
// shader clock (word 2k + 1).  The stamps go only to that buffer; nothing
// reads them on the device.  Phases 7..9 are the finishing workgroup's
// field finish.  (Product build: kProbes is false and Fd2Args::stamps null, so
// a stamp compiles to nothing.)
constexpr u32 kStampGroups = 65536, kStampWords = 32;
NICE_PROBE_ONLY(extern u64 *g_stamps; extern u64 g_last_launch[6];)  // last launch: grid, WG, chunk, nunits, tail, per_cu
// Forced sibling lane stride (nice_debug_force_sib_stride; 0: the model's pick).
extern std::atomic<uint32_t> g_force_sib_stride;
#define FD2_STAMP_P(p, k)                                                                        \
    do {                                                                                         \
        if (kProbes && (p) && threadIdx.x == 0 && blockIdx.x < kStampGroups) {                   \
            (p)[kStampWords * (u64)blockIdx.x + 2 * (k)] = __builtin_amdgcn_s_memrealtime();     \
            (p)[kStampWords * (u64)blockIdx.x + 2 * (k) + 1] = __builtin_amdgcn_s_memtime();     \
        }                                                                                        \
    } while (0)
#define FD2_STAMP(a, k) FD2_STAMP_P((a).stamps, k)

struct Fd2Args {
    u64 *stamps;  // probe build: phase stamps (null in the product build)
    u64 start_lo, start_hi;
    u64 tail_lo, tail_hi;
    u32 nunits, chunk;
    u32 tail_count, main_blocks;
    u32 cutoff;
    u32 ncopies;        // histogram copies in use (<= kHistCopies), the same for every launch of a field
    u32 wave_cap;       // persistent grid: batches one wave may take (its lanes' u16 counters hold them)
    // Cfg::SIB > 1: blocks [0, sib_blocks) walk sibling units (q, k) -> n0 =
    // sib + q M B^2 + k sib_chunk, k < sib_upb; blocks [sib_blocks,
    // sib_blocks + edge_blocks) the edge units q -> edge + q M B^2 (chunk
    // edge_chunk: the rest of each B^2 block); the regular parts follow.
    u64 sib_lo, sib_hi, edge_lo, edge_hi;
    u32 sib_chunk, sib_upb, sib_units, sib_blocks;
    u32 edge_chunk, edge_units, edge_blocks;
    // radix-B digits of start (xs) and tail (xt), least significant first,
    // for init_at (bases whose n passes 64 bits; kXDigits >= NX)
    u32 xs[12], xt[12];
    u64 *hist;          // kHistCopies x 129 bins
    NumOut out;
    const uint4 *tabs;
    FieldFinish fin;    // fin.out_mapped == nullptr: no in-kernel finish
};

// Last-workgroup finish (see Fd2Args).  smem is reused as scratch (>= 1 KB).
// Hand-off without any L2 write-back (MI355X_MICROARCH.md, inter-workgroup
// visibility: agent atomics both sides, the last arriver told by its add's
// return value): every wave waits for its own histogram atomics
// (vmcnt(0)), a barrier, ONE agent-scope add per workgroup; the last
// workgroup reads the copies with agent-scope (sc1) loads.  A __threadfence()
// here would write back and invalidate the XCD's whole L2 once per
// workgroup: 12 000 of them made the b40 1e9 field 1.8x slower.
template <int WG>
__device__ __forceinline__ void field_finish(const FieldFinish &fin, u64 *hist, u32 ncopies, u32 nbins, u32 *count,
                                             unsigned char *smem, u64 *stamps) {
    (void)stamps;
    __shared__ u32 last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) last = last_block_arrive(fin.done);
    __syncthreads();
    if (!last) return;
    FD2_STAMP_P(stamps, 7);  // the last workgroup: arrival known
    unsigned long long *acc = (unsigned long long *)smem;
    for (u32 b = threadIdx.x; b < 129; b += WG) acc[b] = 0;
    __syncthreads();
    // All of a lane's loads issued before the first is used: one L2 round
    // trip for the copies instead of one per copy row.  Only bins < nbins
    // (base + 1) are read: the field's launches touch no other bin, and every
    // finish leaves the bins it read at zero (the generic kernel's finish
    // kernel zeroes all of them).
    constexpr u32 PER = (kHistCopies * 129 + WG - 1) / WG;
    const u32 NE = ncopies * nbins;
    const u32 nmiss = threadIdx.x == 0 ? __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    u64 v[PER];
    u32 at[PER];
#pragma unroll
    for (u32 k = 0; k < PER; k++) {
        const u32 e = threadIdx.x + k * WG;
        const u32 c = e / nbins, b = e - c * nbins;
        at[k] = c * 129 + b;
        v[k] = e < NE ? __hip_atomic_load(&hist[at[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    }
#pragma unroll
    for (u32 k = 0; k < PER; k++) {
        if (v[k]) {
            atomicAdd(&acc[at[k] % 129], (unsigned long long)v[k]);
            __hip_atomic_store(&hist[at[k]], (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    FD2_STAMP_P(stamps, 8);  // copies read and summed
    done_reset(fin.done);
    if (fin.tag) {
        // tagged words (FieldFinish::tag): no store-completion wait, no
        // sequence word; the kernel's end orders the re-zeroing for the slot's
        // next field
        const u64 t = (u64)fin.tag << 32;
        for (u32 b = threadIdx.x; b < nbins; b += WG) fin.out_mapped[b] = t | (u32)acc[b];
        if (threadIdx.x == 0) {
            fin.out_mapped[129] = t | nmiss;
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        FD2_STAMP_P(stamps, 9);
        return;
    }
    for (u32 b = threadIdx.x; b < 129; b += WG) fin.out_mapped[b] = acc[b];
    if (threadIdx.x == 0) {
        fin.out_mapped[129] = nmiss;
        __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Publish: every lane's mapped stores complete, then one system-scope
    // release store of the sequence number (once per field, so its L2
    // write-back costs nothing measurable).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    FD2_STAMP_P(stamps, 9);  // mapped stores complete
    if (threadIdx.x == 0)
        __hip_atomic_store(&fin.out_mapped[130], fin.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One lane's chunk: `chunk` numbers from n0 (the state at n0 built by init;
// the cached high limbs' mask is built here, it needs the tables).
template <class P>
__device__ __forceinline__ void walk_chunk(State<P> &st, const unsigned char *smem, u32 chunk, u64 n0_lo,
                                           u64 n0_hi, u32 hbase, u32 hinc, u32 *outl, u32 cutoff,
                                           const NumOut &out, u32 &probe_acc) {
    recompute_hi<P>(st, smem);
    const u32 r80 = st.r8;
    for (u32 i = 0; i < chunk; i++) {
        u32 m[P::MW], w1 = 0;
#pragma unroll
        for (int w = 0; w < P::MW; w++) m[w] = st.hi[w];
        if constexpr (P::PROBE & 1) {
            m[0] |= st.r8;
            w1 = st.r8 & 0xff;
#pragma unroll
            for (int q = P::LO; q < P::SL; q++) m[q & 1] |= st.S[q];
#pragma unroll
            for (int q = P::LO; q < P::CL; q++) m[q & 1] |= st.C[q];
        } else {
            if constexpr (P::LSD) {
                const uint2 v = *(const uint2 *)(smem + (P::LSDX ? 0 : P::TL) + st.r8);
                m[0] |= v.x;
                if constexpr (P::LSDX) {
                    m[1] |= v.y;
                    w1 = smem[st.rc];
                } else {
                    m[1] |= v.y & P::DMASK;
                    w1 = v.y;
                }
            }
#pragma unroll
            for (int q = P::LO; q < P::SL; q++) {
                if ((P::PROBE & 4) && q == 1) { m[0] |= st.S[q] & 0xffu; continue; }  // probe: no limb-1 lookups
                if (P::vd_s(q) || (P::VDL && q == 0)) or_valu<P>(st.S[q] - P::EBT, m);
                else or_lookup<P, P::TB - (int)P::EBT, P::T2 - (int)P::EBT / 2>(smem, st.S[q], m);
                if (P::LGW && (q - P::LO + 1) % P::LGW == 0) lookup_group_end<P>(m);
            }
#pragma unroll
            for (int q = P::LO; q < P::CL; q++) {
                if ((P::PROBE & 4) && q == 1) { m[1] |= st.C[q] & 0xffu; continue; }
                if (P::vd_c(q) || (P::VDL && q == 0)) or_valu<P>(st.C[q], m);
                else or_lookup<P, P::TB, P::T2>(smem, st.C[q], m);
                if (P::LGW && (P::SL + q - 2 * P::LO + 1) % P::LGW == 0) lookup_group_end<P>(m);
            }
        }
        // uw = unique count - W0: the bias rides in the first v_bcnt's
        // accumulator operand (an SGPR; LLVM would add it separately).
        u32 uw = bcnt_acc(m[0], (u32)(-P::W0));
#pragma unroll
        for (int w = 1; w < P::MW; w++) uw += __popc(m[w]);
        if (uw < (u32)P::W) {
            if constexpr (P::PROBE & 2) probe_acc++;
            else atomicAdd((u32 *)(smem + uw * (P::HROW * 4) + hbase), hinc);
        } else {
            const u32 u = uw + P::W0;
            atomicAdd(&outl[u], 1u);
            if (u > cutoff) {
                u64 lo = n0_lo, hi = n0_hi;
                add_u128(lo, hi, (st.r8 - r80) / P::ES);  // = i (keeps i scalar)
                u32 pos = atomicAdd(out.count, 1u);
                if (pos < out.cap) {
                    out.n[2 * (u64)pos] = lo;
                    out.n[2 * (u64)pos + 1] = hi;
                    out.u[pos] = u;
                }
            }
        }
        step<P>(st, smem, w1);
    }
}

// ---------------------------------------------------------------------------
// Sibling lanes (Cfg::SIB = M > 1).  A lane steps the M numbers n + j B^2
// (j < M) together.  They agree mod B^2, so limbs 0 and 1 of n^2, n^3, D1 =
// 2n + 1 and N3 = 3n + 1 are equal for all of them, and so is every chain's
// carry out of limb 1: the low-digit entry (limb 0 of S and C, with the
// carries and wrap flags), the two limb-1 lookups and limb 1's carry chains
// are done once per step for M numbers.  Sibling 0's State holds the shared
// limbs (its S[1], C[1], D1[1], N3[1], r8); the other siblings' copies of
// them are never read.  Limbs >= 2, the cached high limbs and their mask are
// each sibling's own.  Per n: b40 M = 2 goes from 12 lookups and ~266 VALU
// cycles per wave-step to 10.5 and ~240.
// ---------------------------------------------------------------------------

// One C limb i > LO of C += 3S + N3 (old S) with the scaled carry-in cC;
// returns the scaled carry out (step() does the same inline).  The cached S
// limbs [SL, NS) of a sibling are held as K = 3 ES S (they change only on the
// rare path), so their term is one add.
template <class P>
__device__ __forceinline__ u32 c_limb(State<P> &st, int i, u32 cC) {
    u32 t = st.C[i] + cC;
    if (i < P::NN) asm("" : "+v"(t));
    if (i < P::NN) t += st.N3[i];
    else if (i < P::SL) t -= 3 * P::EBT;
    if (i < P::SL) t = mad_u24<3>(st.S[i], t);
    else if (i < P::NS) t += st.S[i];
    // (The scaled carry straight from one multiply-high, mulhi(t, ES MAGIC) &
    // -ES, prices 18 cycles fewer per step in the issue budget but measured
    // 0.6-2.2 % slower, interleaved A/B: profiles/r05/carry_c8_ab.log.)
    const u32 c = P::C1 ? __umulhi(t, P::MAGIC) : __umulhi(t / P::ES, P::MAGICB);
    st.C[i] = t - c * P::DC;
    return c * P::ES;
}

// One S limb i > LO of S += D1 (biased) with the scaled carry-in cS.
template <class P>
__device__ __forceinline__ u32 s_limb(State<P> &st, int i, u32 cS) {
    const u32 t = st.S[i] + (i < P::ND ? st.D1[i] : 0u) + cS;
    const u32 c = (t >> P::T) & P::ES;
    st.S[i] = t - c * P::B;
    return c;
}

// A sibling's cold C limb k (C[CL + k]) in LDS.
template <class P>
__device__ __forceinline__ unsigned short *cold_slot(const unsigned char *smem, int j, int k) {
    return (unsigned short *)(smem + P::COLD) + ((u32)(j * P::NCOLD + k) * P::WG + threadIdx.x);
}

// recompute_hi for a sibling: cached S limbs in K form, cached C limbs in LDS.
template <class P>
__device__ __forceinline__ void sib_hi(State<P> &st, int j, const unsigned char *smem) {
#pragma unroll
    for (int w = 0; w < P::MW; w++) st.hi[w] = 0;
#pragma unroll
    for (int i = P::SL; i < P::NS; i++)
        or_plain<P>(smem, st.S[i] / (3 * P::ES), i == P::NS - 1 ? P::S_TOPD : 2, st.hi);
#pragma unroll
    for (int k = 0; k < P::NCOLD; k++)
        or_plain<P>(smem, *cold_slot<P>(smem, j, k), P::CL + k == P::NC - 1 ? P::C_TOPD : 2, st.hi);
}

// Plain limbs of sibling j (n + j B^2) from sibling 0's plain limbs and n's
// digits X: (n + j B^2)^2 = S + 2 j n B^2 + j^2 B^4 and (n + j B^2)^3 = C +
// 3 j S B^2 + 3 j^2 n B^4 + j^3 B^6 -- column adds and one normalisation
// instead of sibling j's own radix conversion and products (~1/3 of a
// lane's init each).
template <class P>
__device__ __forceinline__ void sib_derive(State<P> &sj, const State<P> &s0, const u32 (&X)[P::NX], u32 j) {
    {
        u32 acc[P::NS];
#pragma unroll
        for (int t = 0; t < P::NS; t++)
            acc[t] = s0.S[t] + (t >= 2 && t - 2 < P::NX ? 2 * j * X[t - 2] : 0u) + (t == 4 ? j * j : 0u);
        normalize<P>(acc, sj.S);
    }
    {
        u32 acc[P::NC];
#pragma unroll
        for (int t = 0; t < P::NC; t++)
            acc[t] = s0.C[t] + (t >= 2 && t - 2 < P::NS ? 3 * j * s0.S[t - 2] : 0u) +
                     (t >= 4 && t - 4 < P::NX ? 3 * j * j * X[t - 4] : 0u) + (t == 6 ? j * j * j : 0u);
        normalize<P>(acc, sj.C);
    }
    {
        u32 acc[P::ND];
#pragma unroll
        for (int t = 0; t < P::ND; t++) acc[t] = s0.D1[t] + (t == 2 ? 2 * j : 0u);
        normalize<P>(acc, sj.D1);
    }
    {
        u32 acc[P::NN];
#pragma unroll
        for (int t = 0; t < P::NN; t++) acc[t] = s0.N3[t] + (t == 2 ? 3 * j : 0u);
        normalize<P>(acc, sj.N3);
    }
    sj.r8 = s0.r8;
    sj.rc = s0.rc;
}

// Sibling state after init: cached S limbs to K form, cached C limbs to LDS.
template <class P>
__device__ __forceinline__ void sib_park(State<P> &st, int j, const unsigned char *smem) {
#pragma unroll
    for (int i = P::SL; i < P::NS; i++) st.S[i] *= 3 * P::ES;
#pragma unroll
    for (int k = 0; k < P::NCOLD; k++) *cold_slot<P>(smem, j, k) = (unsigned short)st.C[P::CL + k];
}

// Rare path of step_sib: limb-0 wraps of D1 / N3 (one event for all
// siblings: the shared limb 1, then each sibling's upper limbs) and carries
// out of each sibling's top stepped limbs (rare()'s work per sibling).
template <class P>
__device__ __forceinline__ void rare_sib(State<P> (&st)[P::SIB], const unsigned char *smem,
                                      const bool (&cS)[P::SIB], const bool (&cC)[P::SIB]) {
    constexpr int L = P::LO;
    // limb L of the shared D1 / N3 reached B (sib_shared_step stepped it):
    // wrap it and carry into every sibling's limbs above
    if (st[0].D1[L] >= P::ESB) {
        st[0].D1[L] -= P::ESB;
#pragma unroll
        for (int j = 0; j < P::SIB; j++) carry_scaled<P>(st[j].D1, L + 1);
    }
    {
        const u32 off1 = L < P::SL ? 3 * P::EBT : 0u;
        if (st[0].N3[L] + off1 >= P::ESB) {
            st[0].N3[L] -= P::ESB;
#pragma unroll
            for (int j = 0; j < P::SIB; j++) {
                u32 cc = 1;
#pragma unroll
                for (int i = L + 1; i < P::NN; i++) {
                    const u32 off = i < P::SL ? 3 * P::EBT : 0u;
                    const u32 w = st[j].N3[i] + off + cc * P::ES;
                    cc = w >= P::ESB;
                    st[j].N3[i] = (cc ? 0u : w) - off;
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < P::SIB; j++) {
        if (cS[j]) {
            st[j].S[P::SL - 1] -= P::ESB;
            u32 c = 1;  // +1 into the cached limbs (K form: 3 ES per unit)
#pragma unroll
            for (int i = P::SL; i < P::NS; i++) {
                const u32 v = st[j].S[i] + c * 3 * P::ES;
                c = v >= 3 * P::ESB;
                st[j].S[i] = c ? 0u : v;
            }
        }
        if (cC[j]) {
            st[j].C[P::CL - 1] -= P::DC;
            u32 c = 1;
#pragma unroll
            for (int k = 0; k < P::NCOLD; k++) {
                unsigned short *slot = cold_slot<P>(smem, j, k);
                const u32 v = *slot + c;
                c = v == P::B;
                *slot = (unsigned short)(c ? 0u : v);
            }
        }
        if (cS[j] | cC[j]) sib_hi<P>(st[j], j, smem);
    }
}

template <class P>
__device__ __forceinline__ void sib_shared_step(State<P> &s0, u32 w1, u32 &cC, u32 &cS, bool &wrap);

// One FD step of all siblings (step() restated with the shared limb 1).
template <class P>
__device__ __forceinline__ void step_sib(State<P> (&st)[P::SIB], const unsigned char *smem, u32 w1) {
    constexpr int L = P::LO;
    constexpr int CT = P::CL - 1, ST = P::SL - 1;
    u32 cC, cS;
    bool any;
    sib_shared_step<P>(st[0], w1, cC, cS, any);
    bool topS[P::SIB], topC[P::SIB];
#pragma unroll
    for (int j = 0; j < P::SIB; j++) {
        u32 c = cC;
#pragma unroll
        for (int i = L + 1; i < CT; i++) c = c_limb<P>(st[j], i, c);
        st[j].C[CT] += c;
        u32 cs = cS;
#pragma unroll
        for (int i = L + 1; i < ST; i++) cs = s_limb<P>(st[j], i, cs);
        st[j].S[ST] += cs;
        topS[j] = st[j].S[ST] >= (1u << P::SH);
        topC[j] = st[j].C[CT] >= P::DC;
        any |= topS[j] | topC[j];
    }
    if (any) rare_sib<P>(st, smem, topS, topC);
}

// step_sib in pieces for the pipelined walk: the shared limb L (returns the
// scaled carries into limb L + 1 of C and S) ...
template <class P>
__device__ __forceinline__ void sib_shared_step(State<P> &s0, u32 w1, u32 &cC, u32 &cS, bool &wrap) {
    constexpr u32 ES = P::ES;
    constexpr int L = P::LO;
    static_assert(L < P::ND && L < P::NN && P::FLAG_D1 == (1u << 30) && P::FLAG_N3 == (1u << 31),
                  "sibling lanes: shared D1 / N3 limb and the low-digit entry's wrap flags");
    cC = __builtin_amdgcn_ubfe(w1, P::FC, P::FCW);
    {
        u32 t = P::TIGHT ? mad_u24<ES>(cC, s0.C[L]) : s0.C[L] + cC;
        if (L < P::NN) t += s0.N3[L];
        else t -= 3 * P::EBT;
        t = mad_u24<3>(s0.S[L], t);
        const u32 c = P::C1 ? __umulhi(t, P::MAGIC) : __umulhi(t / ES, P::MAGICB);
        s0.C[L] = t - c * P::DC;
        cC = c * ES;
    }
    cS = __builtin_amdgcn_ubfe(w1, P::F0, P::F0W);
    {
        const u32 d = L < P::ND ? s0.D1[L] : 0u;
        const u32 t = P::TIGHT ? mad_u24<ES>(cS, s0.S[L] + d) : s0.S[L] + d + cS;
        cS = (t >> P::T) & ES;
        s0.S[L] = t - cS * P::B;
    }
    s0.r8 += ES;
    // limb-0 wraps of D1 / N3 (the entry's flags, one in ~B / 5 steps) step
    // their limb L here, without a branch; only limb L reaching B (one in
    // ~B^2 / 5) takes the rare path.  (Branching on the flags sent a wave
    // down the rare path on ~1 in 5 steps, mostly for this increment.)
    s0.D1[L] += (w1 >> (30 - ilog2(ES))) & ES;
    s0.N3[L] += (w1 >> (31 - ilog2(ES))) & ES;
    wrap = (s0.D1[L] >= P::ESB) | (s0.N3[L] + (L < P::SL ? 3 * P::EBT : 0u) >= P::ESB);
}

// ... and one sibling's limbs above it (returns whether a top limb carried).
template <class P>
__device__ __forceinline__ bool sib_upper_step(State<P> &st, u32 cC, u32 cS, bool &topS, bool &topC) {
    constexpr int L = P::LO;
    constexpr int CT = P::CL - 1, ST = P::SL - 1;
#pragma unroll
    for (int i = L + 1; i < CT; i++) cC = c_limb<P>(st, i, cC);
    st.C[CT] += cC;
#pragma unroll
    for (int i = L + 1; i < ST; i++) cS = s_limb<P>(st, i, cS);
    st.S[ST] += cS;
    topS = st.S[ST] >= (1u << P::SH);
    topC = st.C[CT] >= P::DC;
    return topS | topC;
}

// One sibling's looked-up table entries of a step (entries of VALU-decoded
// limbs and of limbs <= L are unused).
template <class P>
struct SibLook {
    uint2 s[P::SL], c[P::CL];
};

template <class P>
__device__ __forceinline__ void sib_issue(const State<P> &st, const unsigned char *smem, SibLook<P> &e) {
#pragma unroll
    for (int q = P::LO + 1; q < P::SL; q++)
        if (!P::vd_s(q)) e.s[q] = *(const uint2 *)(smem + (P::TB - (int)P::EBT) + st.S[q]);
#pragma unroll
    for (int q = P::LO + 1; q < P::CL; q++)
        if (!P::vd_c(q)) e.c[q] = *(const uint2 *)(smem + P::TB + st.C[q]);
}

template <class P>
__device__ __forceinline__ void sib_consume(const State<P> &st, const SibLook<P> &e, u32 (&m)[P::MW]) {
#pragma unroll
    for (int q = P::LO + 1; q < P::SL; q++) {
        if (P::vd_s(q)) {
            or_valu<P>(st.S[q] - P::EBT, m);
        } else {
            m[0] |= e.s[q].x;
            m[1] |= e.s[q].y;
        }
    }
#pragma unroll
    for (int q = P::LO + 1; q < P::CL; q++) {
        if (P::vd_c(q)) {
            or_valu<P>(st.C[q], m);
        } else {
            m[0] |= e.c[q].x;
            m[1] |= e.c[q].y;
        }
    }
}

// OR the digit bits of limb q of sibling j's S (isS) or C into m.
template <class P>
__device__ __forceinline__ void or_limb(const State<P> &st, const unsigned char *smem, bool isS, int q,
                                        u32 (&m)[P::MW]) {
    if (isS) {
        if (P::vd_s(q)) or_valu<P>(st.S[q] - P::EBT, m);
        else or_lookup<P, P::TB - (int)P::EBT, P::T2 - (int)P::EBT / 2>(smem, st.S[q], m);
    } else {
        if (P::vd_c(q)) or_valu<P>(st.C[q], m);
        else or_lookup<P, P::TB, P::T2>(smem, st.C[q], m);
    }
}

// walk_chunk for M siblings: `chunk` steps of the numbers n0 + j B^2 + i.
// Sibling 0's first number of this lane's unit (fd2_body's layout of the
// sibling parts; recomputed on the rare near-miss path instead of kept live).
struct SibUnit {
    bool active;
    u32 chunk;
    u64 lo, hi;
};
template <class P>
__device__ __forceinline__ SibUnit sib_unit(const Fd2Args &a) {
    const bool edge = blockIdx.x >= a.sib_blocks;
    const u32 sunit = (edge ? blockIdx.x - a.sib_blocks : blockIdx.x) * P::WG + threadIdx.x;
    const u32 upb = edge ? 1u : a.sib_upb;
    SibUnit u;
    u.active = sunit < (edge ? a.edge_units : a.sib_units);
    u.chunk = edge ? a.edge_chunk : a.sib_chunk;
    const u32 q = sunit / upb, k = sunit - q * upb;
    u.lo = edge ? a.edge_lo : a.sib_lo;
    u.hi = edge ? a.edge_hi : a.sib_hi;
    add_u128(u.lo, u.hi, (u64)q * ((u64)P::SIB * P::B * P::B) + (u64)k * u.chunk);
    return u;
}

// Histogram / near-miss record of sibling j's number at step i (mask m).
template <class P>
__device__ __forceinline__ void sib_record(u32 u, int j, u32 i, const Fd2Args &a, u32 *outl, u32 cutoff,
                                           const NumOut &out);

template <class P>
__device__ __forceinline__ void sib_count(const u32 (&m)[P::MW], int j, u32 i, const unsigned char *smem,
                                          const Fd2Args &a, u32 hbase, u32 hinc, u32 *outl, u32 cutoff,
                                          const NumOut &out) {
    u32 uw = bcnt_acc(m[0], (u32)(-P::W0));
#pragma unroll
    for (int w = 1; w < P::MW; w++) uw += __popc(m[w]);
    if (uw < (u32)P::W) {
        atomicAdd((u32 *)(smem + uw * (P::HROW * 4) + hbase), hinc);
    } else {
        sib_record<P>(uw + P::W0, j, i, a, outl, cutoff, out);
    }
}

// An out-of-window count u of sibling j's number at step i: the workgroup's
// out-of-window bin and, above the cutoff, the near-miss list.
template <class P>
__device__ __forceinline__ void sib_record(u32 u, int j, u32 i, const Fd2Args &a, u32 *outl, u32 cutoff,
                                           const NumOut &out) {
    {
        atomicAdd(&outl[u], 1u);
        if (u > cutoff) {
            const SibUnit su = sib_unit<P>(a);
            u64 lo = su.lo, hi = su.hi;
            // i opaque here: otherwise the compiler strength-reduces su.lo +
            // j B^2 + i into three 64-bit induction variables stepped on
            // every step of the walk for this once-in-1e8 branch
            u32 ii = i;
            asm volatile("" : "+v"(ii));
            add_u128(lo, hi, (u64)j * ((u64)P::B * P::B) + ii);
            u32 pos = atomicAdd(out.count, 1u);
            if (pos < out.cap) {
                out.n[2 * (u64)pos] = lo;
                out.n[2 * (u64)pos + 1] = hi;
                out.u[pos] = u;
            }
        }
    }
}

// walk_sib, pipelined (Cfg::LG >= 100): a step issues the shared lookups and
// sibling 0's, computes the shared limb's carries (they need only the
// low-digit entry) while those are in flight, issues sibling 1's, and then
// per sibling j: consumes its lookups, counts its number, steps its upper
// limbs and issues sibling j + 2's.  Two siblings' lookups are in flight
// while the VALU works, so the lookups' latency hides behind arithmetic at 4
// waves per SIMD (scheduling barriers pin the order).
template <class P>
__device__ __forceinline__ void walk_sib_pipe(State<P> (&st)[P::SIB], const unsigned char *smem, const Fd2Args &a,
                                              u32 chunk, u32 hbase, u32 hinc, u32 *outl, u32 cutoff,
                                              const NumOut &out) {
    constexpr int L = P::LO;
    constexpr int M = P::SIB;
#pragma unroll
    for (int j = 0; j < M; j++) sib_hi<P>(st[j], j, smem);
    for (u32 i = 0; i < chunk; i++) {
        SibLook<P> e[M];
        // shared lookups (limb 0 of S and C, limb L of S and C) and sibling 0's
        const uint2 vlo = *(const uint2 *)(smem + P::TL + st[0].r8);
        uint2 vs, vc;
        u32 mv[P::MW] = {};
        if (P::vd_s(L)) or_valu<P>(st[0].S[L] - P::EBT, mv);
        else vs = *(const uint2 *)(smem + (P::TB - (int)P::EBT) + st[0].S[L]);
        if (P::vd_c(L)) or_valu<P>(st[0].C[L], mv);
        else vc = *(const uint2 *)(smem + P::TB + st[0].C[L]);
        sib_issue<P>(st[0], smem, e[0]);
        __builtin_amdgcn_sched_barrier(0);
        // the shared limb's step (needs only the low-digit entry's carries)
        const u32 w1 = vlo.y;
        u32 cC, cS;
        bool any;
        sib_shared_step<P>(st[0], w1, cC, cS, any);
        if (M > 1) sib_issue<P>(st[1], smem, e[1]);
        __builtin_amdgcn_sched_barrier(0);
        u32 m0[P::MW];
        bool topS[M], topC[M];
#pragma unroll
        for (int j = 0; j < M; j++) {
            if (j == 0) {
                m0[0] = vlo.x | mv[0] | (P::vd_s(L) ? 0u : vs.x) | (P::vd_c(L) ? 0u : vc.x);
                m0[1] = (vlo.y & P::DMASK) | mv[1] | (P::vd_s(L) ? 0u : vs.y) | (P::vd_c(L) ? 0u : vc.y);
            }
            u32 m[P::MW];
#pragma unroll
            for (int w = 0; w < P::MW; w++) m[w] = m0[w] | st[j].hi[w];
            sib_consume<P>(st[j], e[j], m);
            // probe 16 (wrong by design): no window count, the mask feeds a
            // register sum instead
            if constexpr ((P::PROBE & 16) != 0) {
                any |= (m[0] ^ m[1]) == 0x5a5a5a5au;
            } else {
                sib_count<P>(m, j, i, smem, a, hbase, hinc, outl, cutoff, out);
            }
            any |= sib_upper_step<P>(st[j], cC, cS, topS[j], topC[j]);
            if (j + 2 < M) sib_issue<P>(st[j + 2], smem, e[j + 2]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // probe 8 (wrong by design): the rare path never runs
        if ((P::PROBE & 8) == 0 && any) rare_sib<P>(st, smem, topS, topC);
    }
}

template <class P>
__device__ __forceinline__ void walk_sib(State<P> (&st)[P::SIB], const unsigned char *smem, const Fd2Args &a,
                                         u32 chunk, u32 hbase, u32 hinc, u32 *outl, u32 cutoff, const NumOut &out) {
    if constexpr (P::LG >= 100) {
        walk_sib_pipe<P>(st, smem, a, chunk, hbase, hinc, outl, cutoff, out);
        return;
    }
    constexpr int L = P::LO;
#pragma unroll
    for (int j = 0; j < P::SIB; j++) sib_hi<P>(st[j], j, smem);
    const u32 r80 = st[0].r8;
    for (u32 i = 0; i < chunk; i++) {
        // shared: limb 0 of S and C (low-digit entry) and limb 1 of both
        u32 m0[P::MW];
        const uint2 v = *(const uint2 *)(smem + P::TL + st[0].r8);
        const u32 w1 = v.y;
        m0[0] = v.x;
        m0[1] = v.y & P::DMASK;
        or_limb<P>(st[0], smem, true, L, m0);
        or_limb<P>(st[0], smem, false, L, m0);
#pragma unroll
        for (int j = 0; j < P::SIB; j++) {
            u32 m[P::MW];
#pragma unroll
            for (int w = 0; w < P::MW; w++) m[w] = m0[w] | st[j].hi[w];
#pragma unroll
            for (int q = L + 1; q < P::SL; q++) {
                or_limb<P>(st[j], smem, true, q, m);
                if (P::LG > 1 && (q - L) % P::LG == 0) lookup_group_end<P>(m);
            }
#pragma unroll
            for (int q = L + 1; q < P::CL; q++) {
                or_limb<P>(st[j], smem, false, q, m);
                if (P::LG > 1 && (P::SL - L - 1 + q - L) % P::LG == 0) lookup_group_end<P>(m);
            }
            // a group per sibling: its loaded words are dead before the next
            // sibling's lookups issue (bounds the VGPRs in flight)
            if (P::LG) lookup_group_end<P>(m);
            u32 uw = bcnt_acc(m[0], (u32)(-P::W0));
#pragma unroll
            for (int w = 1; w < P::MW; w++) uw += __popc(m[w]);
            if (uw < (u32)P::W) {
                atomicAdd((u32 *)(smem + uw * (P::HROW * 4) + hbase), hinc);
            } else {
                const u32 u = uw + P::W0;
                atomicAdd(&outl[u], 1u);
                if (u > cutoff) {
                    const SibUnit su = sib_unit<P>(a);
                    u64 lo = su.lo, hi = su.hi;
                    add_u128(lo, hi, (u64)j * ((u64)P::B * P::B) + (st[0].r8 - r80) / P::ES);
                    u32 pos = atomicAdd(out.count, 1u);
                    if (pos < out.cap) {
                        out.n[2 * (u64)pos] = lo;
                        out.n[2 * (u64)pos + 1] = hi;
                        out.u[pos] = u;
                    }
                }
            }
        }
        step_sib<P>(st, smem, w1);
    }
}

// Persistent grid: batch b of the launch (64 lanes' units) -> this lane's
// unit: b < mb: main unit 64 b + lane (chunk a.chunk from a.start); else the
// tail numbers 64 (b - mb) + lane (chunk 1 from a.tail).
__device__ __forceinline__ void pers_unit(const Fd2Args &a, u32 b, u32 mb, u32 lane, bool &active, u64 &lo,
                                          u64 &hi, u32 &chunk) {
    if (b < mb) {
        const u32 unit = 64 * b + lane;
        active = unit < a.nunits;
        lo = a.start_lo;
        hi = a.start_hi;
        add_u128(lo, hi, (u64)unit * a.chunk);
        chunk = a.chunk;
    } else {
        const u32 idx = 64 * (b - mb) + lane;
        active = idx < a.tail_count;
        lo = a.tail_lo;
        hi = a.tail_hi;
        add_u128(lo, hi, (u64)idx);
        chunk = 1;
    }
}

template <class P>
__device__ __forceinline__ void fd2_body(const Fd2Args &a) {
    // Static LDS: its address is a compile-time constant, so a lookup is one
    // ds_read with the table offset in the instruction's immediate field.
    __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDS_BYTES];
    u32 *hist = (u32 *)(smem + P::HB);
    u32 *outl = (u32 *)(smem + P::OUTL);
    const u32 tid = threadIdx.x;
    const NumOut out = a.out;
    const u32 cutoff = a.cutoff;
    // sibling parts (Cfg::SIB), then the main part and the tail part of the
    // launch (workgroup-uniform)
    const u32 sib_end = P::SIB > 1 ? a.sib_blocks + a.edge_blocks : 0u;
    const bool sib_part = P::SIB > 1 && blockIdx.x < sib_end;
    const u32 bid = blockIdx.x - sib_end;
    const bool main_part = bid < a.main_blocks;
    const u64 start_lo = main_part ? a.start_lo : a.tail_lo;
    const u64 start_hi = main_part ? a.start_hi : a.tail_hi;
    const u32 nunits = main_part ? a.nunits : a.tail_count;
    const u32 chunk = main_part ? a.chunk : 1u;
    const u32 blk = main_part ? bid : bid - a.main_blocks;
    FD2_STAMP(a, 0);  // start

    // The tables (built once per device and base in global memory,
    // fd2_tables) are DMA'd into LDS, and the histogram region zeroed:
    // building them here cost ~5 % of a launch of short chunks.  One
    // global_load_lds_dwordx4 wave-instruction moves 1 KiB (lane l's 16 bytes
    // land at the wave-uniform base + 16 l): every load of the copy is in
    // flight at once, with no VGPR round trip and no ds_write (the register
    // copy it replaces waited one L2 round trip per 16 bytes a lane moved:
    // b40 1e6 spent 2.1 us of a 12.5 us kernel in it, fd2_stamps_before.log).
    {
        constexpr u32 N16 = (u32)(P::TAB_BYTES / 16);
        const u32 lane = tid & 63, w64 = tid & ~63u;
        for (u32 i0 = w64; i0 < N16; i0 += P::WG)
            if (i0 + lane < N16)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(a.tabs + i0 + lane),
                                                 (__attribute__((address_space(3))) void *)(smem + P::TC0 + 16 * i0),
                                                 16, 0, 0);
        uint4 *h4 = (uint4 *)smem;
        for (u32 i = tid; i < (u32)(P::ZA / 16); i += P::WG) h4[i] = make_uint4(0, 0, 0, 0);
        if constexpr (P::SPLIT)
            for (u32 i = tid; i < (u32)(P::HIST_BYTES / 16); i += P::WG)
                h4[P::HB / 16 + i] = make_uint4(0, 0, 0, 0);
    }
    // A lane's first chunk (without PERS its only one: launch_cfg sizes the
    // grid to cover every unit) is set up while the table DMA is in flight;
    // only the cached high limbs' mask needs the tables.
    const u32 lane_id = tid & 63;
    u32 unit = blk * P::WG + tid;
    bool active = unit < nunits;
    u64 n0_lo = start_lo, n0_hi = start_hi;
    u32 chunk_l = chunk;
    // persistent grid: this workgroup's batches are b = blockIdx + G k, k <
    // pnk, of the launch's nb = mb main + tail batches (strided, so every
    // workgroup samples the whole field: contiguous slabs were up to 40 %
    // slower on some n-ranges, profiles/r03/fd2_stamps_pers.log), and the
    // next k to hand out
    __shared__ u32 pers_next;
    u32 pmb = 0, pnk = 0, pk = 0;
    u64 n0_off = 0;          // n0 - the part's first n (init_at)
    const bool n0_tail = !main_part;
    if constexpr (P::PERS) {
        pmb = (a.nunits + 63) / 64;
        const u32 nb = pmb + (a.tail_count + 63) / 64, G = gridDim.x;
        pnk = nb > blockIdx.x ? (nb - blockIdx.x + G - 1) / G : 0;
        pk = tid >> 6;
        if (tid == 0) pers_next = P::WG / 64;
        if (pk < pnk) pers_unit(a, blockIdx.x + G * pk, pmb, lane_id, active, n0_lo, n0_hi, chunk_l);
        else active = false;
    } else {
        n0_off = (u64)unit * chunk;
        add_u128(n0_lo, n0_hi, n0_off);
    }
    // Window counters: row u - W0, column tid mod HROW (u16 halves / u8 quarters).
    const u32 hbase = P::HB + tid % P::HROW * 4;
    // (HROW is a multiple of 64: the increment is wave-uniform, an SGPR)
    static_assert(P::HROW % 64 == 0, "window row of whole waves");
    const u32 hinc = __builtin_amdgcn_readfirstlane(1u << (32 / P::HQ * (tid / P::HROW)));
    u32 probe_acc = 0;
    // Sibling lanes (workgroup-uniform): the sibling state is built, waited
    // for and walked on its own path, so its registers never overlap the
    // regular path's (one State live at the barrier, not M + 1).
    bool sib_done = false;
    if constexpr (P::SIB > 1) {
        if (sib_part) {
            State<P> sst[P::SIB];
            const SibUnit su = sib_unit<P>(a);
            if (su.active) {
                u32 X[P::NX];
                init_digits<P>(X, su.lo, su.hi);
                init_plain<P>(sst[0], X);
#pragma unroll
                for (int j = 1; j < P::SIB; j++) sib_derive<P>(sst[j], sst[0], X, (u32)j);
#pragma unroll
                for (int j = 0; j < P::SIB; j++) {
                    init_scale<P>(sst[j]);
                    sib_park<P>(sst[j], j, smem);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (su.active) walk_sib<P>(sst, smem, a, su.chunk, hbase, hinc, outl, cutoff, out);
            sib_done = true;
        }
    }
    State<P> st;
    // (the persistent grid runs only on the 1024-thread kernels, which keep
    // init(): C64)
    if constexpr (P::PERS || P::N64 || P::C64) {
        if (!sib_done && active) init<P>(st, n0_lo, n0_hi);
    } else {
        if (!sib_done && active) init_at<P>(st, n0_tail ? a.xt : a.xs, n0_off, n0_lo, n0_hi);
    }
    // The table DMA must have landed before any wave reads LDS: wait for it
    // explicitly (a workgroup barrier alone need not imply vmcnt(0)), then
    // the barrier.
    if (!sib_done) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    FD2_STAMP(a, 1);  // state built, tables in LDS
    FD2_STAMP(a, 2);  // (the cached mask is built inside walk_chunk)
    if constexpr (P::SIB > 1) {
        if (!sib_done && active)
            walk_chunk<P>(st, smem, chunk, n0_lo, n0_hi, hbase, hinc, outl, cutoff, out, probe_acc);
    } else if constexpr (!P::PERS) {
        if (active) {
            walk_chunk<P>(st, smem, chunk, n0_lo, n0_hi, hbase, hinc, outl, cutoff, out, probe_acc);
        }
    } else {
        // Persistent grid: wave w starts on this workgroup's batch k = w (its
        // state is already built), then pulls the next k from the LDS counter
        // until the workgroup's batches are exhausted or the wave has taken
        // wave_cap of them (its lanes' u16 counters hold them; the host sizes
        // launches so the waves' caps cover the workgroup's batches).
        u32 k = pk, taken = 0;
        bool act = active;
        u64 m_lo = n0_lo, m_hi = n0_hi;
        u32 ch = chunk_l;
        while (k < pnk) {
            if (taken) {
                pers_unit(a, blockIdx.x + gridDim.x * k, pmb, lane_id, act, m_lo, m_hi, ch);
                if (act) init<P>(st, m_lo, m_hi);
            }
            if (act) walk_chunk<P>(st, smem, ch, m_lo, m_hi, hbase, hinc, outl, cutoff, out, probe_acc);
            if (++taken >= a.wave_cap) break;
            u32 nk = 0;
            if (lane_id == 0) nk = atomicAdd(&pers_next, 1u);
            k = __builtin_amdgcn_readfirstlane(__shfl(nk, 0));
        }
    }
    if constexpr ((P::PROBE & 2) != 0) atomicAdd(&outl[P::W0], probe_acc);  // mass only
    FD2_STAMP(a, 3);  // thread 0's steps done
    __syncthreads();
    FD2_STAMP(a, 4);  // every wave's steps done
    const u32 lane = tid & 63, wave = tid >> 6;
    u64 *hist_out = a.hist + (blockIdx.x % a.ncopies) * 129;
    // Window rows: wave w sums rows w, w + WG/64, ...; all of a wave's rows
    // are read and reduced together, so their cross-lane steps overlap.
    constexpr u32 NWAVE = P::WG / 64, RPW = (P::W + NWAVE - 1) / NWAVE;
    u32 rs[RPW];
#pragma unroll
    for (u32 k = 0; k < RPW; k++) {
        const u32 row = wave + k * NWAVE;
        u32 s = 0;
        if (row < (u32)P::W) {
#pragma unroll
            for (int q = 0; q < P::HROW / 64; q++) {
                const u32 v = hist[row * P::HROW + lane + 64 * q];
                if constexpr (P::HQ == 2) s += (v & 0xffffu) + (v >> 16);
                else s += (v & 0xffu) + ((v >> 8) & 0xffu) + ((v >> 16) & 0xffu) + (v >> 24);
            }
        }
        rs[k] = s;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (u32 k = 0; k < RPW; k++) rs[k] += __shfl_xor(rs[k], o);
#pragma unroll
    for (u32 k = 0; k < RPW; k++) {
        const u32 row = wave + k * NWAVE;
        if (lane == 0 && row < (u32)P::W && rs[k])
            atomicAdd((unsigned long long *)&hist_out[P::W0 + row], (unsigned long long)rs[k]);
    }
    if (tid < (u32)P::NBINS && outl[tid])
        atomicAdd((unsigned long long *)&hist_out[tid], (unsigned long long)outl[tid]);
    FD2_STAMP(a, 5);  // histogram flushed (thread 0's part)
    if (a.fin.out_mapped) {
        __syncthreads();  // smem is reused by the finish
        field_finish<P::WG>(a.fin, a.hist, a.ncopies, P::NBINS, out.count, smem, a.stamps);
    }
    FD2_STAMP(a, 6);  // end (the finishing workgroup: after the finish)
}

template <class P>
__global__ void __launch_bounds__(P::WG) __attribute__((amdgpu_waves_per_eu(P::WPE, P::WPE)))
fd2_kernel(Fd2Args a) {
    fd2_body<P>(a);
}

template <class P>
static hipError_t launch_sib(const DetailedLaunch &p, int num_cus, hipStream_t s);

// Radix-B digits of n, least significant first (Fd2Args::xs / xt).
static inline void host_digits(u128 n, u32 B, u32 *out, int nx) {
    for (int i = 0; i < nx; i++) {
        out[i] = (u32)(n % B);
        n /= B;
    }
}

// ---------------------------------------------------------------------------
// Lane stride from a bank-conflict model.  A wave's lanes sit `L` numbers
// apart (one chunk each), so the value of a HIGH limb across the lanes is an
// arithmetic progression whose step is f'(n) L / B^q (f = n^2, n^3).  A
// table lookup costs, per pass of 32 lanes (8-byte entries) or 16 lanes
// (16-byte entries), the largest number of distinct entries that share a
// bank slot (entry mod 32 / mod 16): 1-2 for a progression with an odd step,
// up to 32 for a step that is a multiple of 32 -- e.g. b40's top C limb
// steps ~32 per lane at L = 125 from the range start (modelled 91 against
// 63 LDS cycles per wave-step, measured 2.35 against 1.86 ms per 1e9 in the
// sibling kernel), and L = 81 hits the same 10 % into the range (2.37 vs
// 1.90 ms; profiles/r05/sib_chunk_sweep.log).  The low limbs' values are
// effectively random whatever L is, so the model counts only the limbs
// whose value f / B^q stays below 2^60 (long double keeps their integer
// part), at a few points of the segment and of the chunk, and the launch
// takes the candidate stride with the smallest modelled cost.
// ---------------------------------------------------------------------------
// Cost of one lookup pass (`slots` lanes on `slots` bank slots) whose lane
// values are floor(a + d l) mod B, as a function of the step d at a
// resolution of 1/64, averaged over the offset a: max distinct values per
// slot.  The pattern of slots depends on d mod slots, but whether lanes
// share a value (a broadcast, free) only on d itself, so the table covers
// d in [0, 2 slots): steps >= slots are looked up at slots + d mod slots.
// Simulated once per process.
static const std::vector<float> &progression_cost(int slots) {
    static std::mutex mu;
    static std::map<int, std::vector<float>> tab;
    std::lock_guard<std::mutex> g(mu);
    auto it = tab.find(slots);
    if (it != tab.end()) return it->second;
    std::vector<float> t((size_t)slots * 128);
    for (size_t k = 0; k < t.size(); k++) {
        const double d = (double)k / 64;
        double sum = 0;
        for (int ai = 0; ai < 16; ai++) {
            const double a = ai / 16.0 + 0.03125;
            // the lane values floor(a + d l) never decrease with l, so a
            // value repeats only in consecutive lanes (a broadcast)
            int cnt[32] = {};
            int best = 0;
            long prev = -1;
            for (int l = 0; l < slots; l++) {
                const long v = (long)(a + d * l);  // a + d l >= 0: truncation is floor
                if (v == prev) continue;
                prev = v;
                const int sl = (int)(v & (slots - 1));  // slots: 16 or 32
                best = std::max(best, ++cnt[sl]);
            }
            sum += best;
        }
        t[k] = (float)(sum / 16);
    }
    return tab.emplace(slots, std::move(t)).first->second;
}

// Modelled LDS cycles of a wave-step's lookups of the limbs whose lane
// values progress (the high looked-up limbs of S = n^2 and C = n^3 from
// first_limb on, where the lanes' quadratic drift stays under half a unit)
// at lane stride L, averaged over the segment's start, middle and end.  The
// other limbs' values are effectively random whatever L is and are left out.
// Per limb and point the lane step is c L and the drift k L^2 (c = f'(n) /
// B^q, k = f''(n) 64^2 / 2 / B^q), so the strides of one pick share them.
template <class P>
struct ConflictModel {
    static constexpr int SLOTS = P::ES == 16 ? 16 : 32;
    static constexpr int NPASS = 64 / SLOTS;
    int n = 0;
    double c[3 * (P::SL + P::CL)], k[3 * (P::SL + P::CL)];
    const std::vector<float> *tab;
    ConflictModel(long double n0, long double span, int first_limb) : tab(&progression_cost(SLOTS)) {
        for (int pt = 0; pt < 3; pt++) {
            const long double x = n0 + span * (long double)pt / 2;
            for (int cube = 0; cube < 2; cube++) {
                const int hi = cube ? P::CL : P::SL;
                long double bq = 1;
                for (int q = 0; q < first_limb; q++) bq *= (long double)P::B;
                for (int q = first_limb; q < hi; q++, bq *= (long double)P::B) {
                    if (cube ? P::vd_c(q) : P::vd_s(q)) continue;
                    const long double f1 = cube ? 3 * x * x : 2 * x;  // f'(n)
                    const long double f2 = cube ? 6 * x : 2;          // f''(n)
                    c[n] = (double)(f1 / bq);
                    k[n] = (double)(f2 * 4096 / 2 / bq);
                    n++;
                }
            }
        }
    }
    double cost(u64 L) const {
        double sum = 0;
        const double l = (double)L;
        for (int i = 0; i < n; i++) {
            if (k[i] * l * l >= 0.5) continue;  // drifting: effectively random
            // the lane step in limb units: < 2^24 for every limb that passes
            // the drift test, so double keeps its fraction
            const double d = c[i] * l;
            const double r = d < SLOTS ? d : SLOTS + (d - SLOTS * std::floor(d / SLOTS));
            sum += NPASS * (*tab)[std::min<size_t>(tab->size() - 1, (size_t)(r * 64))];
        }
        return sum / 3;
    }
};

// The odd stride in [lo, hi] with the lowest modelled cost at the segment
// [start, start + count); among the strides within `tol` modelled cycles of
// the best, the one closest to target (a lane's init amortises over its
// chunk).  A few hundred table lookups: cheap enough for every launch.
// (A rounds-aware pick -- the stride whose units fill whole rounds of the
// resident lanes, times L plus init steps -- chose L ~ 130-160 and lost on
// small fields: b40 1e8 0.261 ms against 0.227 at L = 65, and did not gain at
// 1e9; profiles/r05/picker_rounds.log.)
template <class P>
static u64 pick_lane_stride(u128 start, u64 count, u64 lo, u64 hi, u64 target, int first_limb,
                            double tol = 0.5) {
    const ConflictModel<P> m((long double)start, (long double)count, first_limb);
    double cost[512];
    int nc = 0;
    double min_cost = 1e30;
    for (u64 L = lo | 1; L <= hi && nc < 512; L += 2, nc++) {
        cost[nc] = m.cost(L);
        min_cost = std::min(min_cost, cost[nc]);
    }
    u64 best = target | 1, best_d = ~0ull;
    nc = 0;
    for (u64 L = lo | 1; L <= hi && nc < 512; L += 2, nc++) {
        const u64 d = L > target ? L - target : target - L;
        if (cost[nc] <= min_cost + tol && d < best_d) {
            best = L;
            best_d = d;
        }
    }
    return best;
}

// The stride for fields of a few rounds (fewer than 3 at the target
// stride): among the odd L in [lo, hi] the model does not flag, the one
// whose units fill the fewest whole rounds of the resident lanes per step of
// work, ceil(Q (ceil(D / L) - 1) / lanes) (L + init).  A part-filled last
// round costs a whole one there: b40 1e8 (13 super-blocks) takes 0.227 ms at
// L = 65 (1.95 rounds), 0.270 at L = 63 (2.01) and 0.259 at 61 (2.08); 9e7 is
// best at 61 (1.76 rounds; profiles/r05/sib_small_L.log).  Sets `rounds`.
template <class P>
static u64 pick_small_stride(u128 start, u64 count, u64 lo, u64 hi, int first_limb, u64 Q, u64 lanes, u64 D,
                             double &rounds, double init = 6, double tol = 6) {
    const ConflictModel<P> m((long double)start, (long double)count, first_limb);
    double cost[512];
    int nc = 0;
    double min_cost = 1e30;
    for (u64 L = lo | 1; L <= hi && nc < 512; L += 2, nc++) {
        cost[nc] = m.cost(L);
        min_cost = std::min(min_cost, cost[nc]);
    }
    u64 best = lo | 1;
    double best_t = 1e300;
    rounds = 0;
    nc = 0;
    for (u64 L = lo | 1; L <= hi && nc < 512; L += 2, nc++) {
        if (cost[nc] > min_cost + tol) continue;
        const u64 units = Q * ((D + L - 1) / L - 1);
        const double t = (double)((units + lanes - 1) / lanes) * ((double)L + init);
        if (t < best_t) {
            best_t = t;
            best = L;
            rounds = (double)units / (double)lanes;
        }
    }
    return best;
}

template <class P>
static hipError_t launch_cfg(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    if constexpr (P::SIB > 1) return launch_sib<P>(p, num_cus, s);
    auto kern = fd2_kernel<P>;
    // Occupancy is a property of the code object: queried once per
    // instantiation (a runtime call per launch is host latency on small fields).
    static const int per_cu_q = [&] {
        int v = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, (const void *)kern, P::WG, 0) == hipSuccess
                   ? v : -1;
    }();
    if (per_cu_q < 0) return hipErrorInvalidDeviceFunction;
    const int per_cu = per_cu_q < 1 ? 1 : per_cu_q;
    hipError_t e = hipSuccess;
    // Resident lanes (one "round" of workgroups).
    const u64 lanes = (u64)num_cus * per_cu * P::WG;
    // Launch size bound (nunits fits 32 bits).  A lane takes ONE chunk per
    // launch, so its window counters count at most chunk <= TCHUNK numbers
    // (u16 halves; u8 quarters need chunk <= 255, checked below).
    const u64 max_count = lanes * 60000ull;
    // Every near-miss count must lie above the window (it is recorded on the
    // out-of-window branch).
    if (p.cutoff + 1 < (u32)(P::W0 + P::W)) return hipErrorInvalidValue;
    // Target numbers per lane.  Short chunks put a wave's 64 lanes on nearby n,
    // so the top stepped limbs (and the cached ones) of neighbouring lanes are
    // equal or close and their lookups stop conflicting; a chunk still pays
    // one init (radix-B conversion and products, ~10 steps).  Without PERS
    // each lane takes one chunk and the grid is many rounds of workgroups:
    // with two or more workgroups per CU, workgroups at different phases
    // (table DMA, init, steps, draining) share a CU (b40 1e9 round 1: 2.49 ms
    // persistent with static lane assignment at chunk 637, 2.31 at ~80,
    // 2.19-2.21 in rounds, profiles/r01/fd2_chunk_sweep.log).
    const u64 tchunk = probe_knob("NICE_FD2_TCHUNK", (u64)P::TCHUNK);
    if constexpr (P::PERS) {
        // The persistent grid pays off where ONE workgroup fills a CU and the
        // segment needs at least two rounds of them; otherwise (a device with
        // other occupancy, short segments) the same kernel in rounds.
        if (per_cu_q != 1 || p.count < 2 * tchunk * lanes) return launch_cfg<typename P::NoPers>(p, num_cus, s);
    }
    const uint4 *tabs = nullptr;
    if ((e = fd2_tables<P>(s, &tabs)) != hipSuccess) return e;
    DetailedLaunch q = p;
    u64 left = p.count;
    while (left) {
        u64 cnt = left < max_count ? left : max_count;
        u64 chunk = 0, nunits = 0, tail = 0, grid = 0;
        const u64 nw = P::WG / 64;
        for (;;) {
            // Chunk floor for fields too small to fill the chip: a lane's init
            // costs about ten steps, but with idle CUs latency wins (b40 1e6:
            // kernel 25 us at a floor of 32, 14 us at 4; scripts/small_fields.py).
            const u64 min_chunk = probe_knob("NICE_FD2_MINCHUNK", 4);
            // Whole rounds of workgroups, chunks <= the target (and <= B, the
            // low-digit table's reach).
            u64 rounds = (cnt + tchunk * lanes - 1) / (tchunk * lanes);
            if (rounds < 1) rounds = 1;
            chunk = (cnt + rounds * lanes - 1) / (rounds * lanes);
            if (chunk < min_chunk) chunk = cnt < min_chunk ? cnt : min_chunk;
            if (chunk < 1) chunk = 1;
            // Odd chunks: lane l of a wave then sits at n mod B = r0 + chunk * l,
            // so its low-digit entries fall on 32 distinct bank pairs per
            // half-wave (B is a multiple of 32 for the LSD bases).  Without a
            // low-digit table (b80) limb 0 of n^2 and n^3 is looked up in the
            // pair table, and a chunk divisible by 16 puts a 16-lane group on
            // ONE bank quad for those lookups (n^2 mod 16 equal on every lane):
            // b80 1e9 at chunk 2544 took 11.8 ms, at 2545 9.3.
            if (chunk > 1 && (P::LSD ? chunk % 2 == 0 : chunk % 16 == 0)) chunk++;
            if (chunk > P::B) chunk = P::B % 2 ? P::B : P::B - 1;
            // (The bank-conflict model that picks the sibling kernel's lane
            // stride, pick_lane_stride, did not help the persistent-grid
            // kernels of the wider bases: re-picking their chunk where it
            // modelled a pathology moved b45..80 by -5 .. +9 %,
            // profiles/r05/model_sweep.log, model_sweep2.log.)
            if (P::HQ == 4 && chunk > 255) return hipErrorInvalidValue;
            nunits = cnt / chunk;
            tail = cnt - nunits * chunk;  // < chunk <= B: one number per lane
            bool fits = nunits <= 0xffffffffull;
            if constexpr (P::PERS) {
                // one round of resident workgroups (fewer when the batches
                // run out); the batch count stays in 32 bits and every
                // workgroup's batches fit its waves' caps (u16 counters)
                const u64 nb = (nunits + 63) / 64 + (tail + 63) / 64;
                grid = std::min<u64>((u64)num_cus * per_cu, (nb + nw - 1) / nw);
                fits = fits && nunits <= 0xffffffc0ull && (nb + grid - 1) / grid <= nw * (65535 / chunk);
            } else {
                grid = (nunits + P::WG - 1) / P::WG + (tail + P::WG - 1) / P::WG;
            }
            if (fits) break;
            // Too much for one launch of this shape: split the segment (the
            // finish rides on the last launch, so any split is exact).
            if (cnt < 2) return hipErrorInvalidValue;
            cnt /= 2;
        }
        const u64 main_blocks = (nunits + P::WG - 1) / P::WG;  // one chunk per lane
        Fd2Args a{};
        NICE_PROBE_ONLY(a.stamps = g_stamps;)
        a.start_lo = q.start_lo;
        a.start_hi = q.start_hi;
        a.tail_lo = q.start_lo;
        a.tail_hi = q.start_hi;
        add_u128(a.tail_lo, a.tail_hi, nunits * chunk);
        a.nunits = (u32)nunits;
        a.chunk = (u32)chunk;
        a.tail_count = (u32)tail;
        a.main_blocks = (u32)main_blocks;
        if constexpr (!P::N64 && !P::C64) {
            host_digits(((u128)a.start_hi << 64) | a.start_lo, P::B, a.xs, P::NX);
            host_digits(((u128)a.tail_hi << 64) | a.tail_lo, P::B, a.xt, P::NX);
        }
        a.cutoff = q.cutoff;
        a.ncopies = q.hist_copies;
        a.wave_cap = (u32)(65535 / chunk);
        a.hist = q.hist;
        a.out = q.out;
        a.tabs = tabs;
        // the field's finish rides on its last launch
        a.fin = left == cnt ? q.fin : FieldFinish{nullptr, nullptr, 0, 0};
        NICE_PROBE_ONLY({
            const u64 v[6] = {grid, (u64)P::WG, chunk, nunits, tail, (u64)per_cu};
            for (int k = 0; k < 6; k++) g_last_launch[k] = v[k];
        })
        hipLaunchKernelGGL(kern, dim3((u32)grid), dim3(P::WG), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (p.launches) ++*p.launches;
        add_u128(q.start_lo, q.start_hi, cnt);
        left -= cnt;
    }
    return hipSuccess;
}


// Sibling-lane launches (Cfg::SIB = M > 1).  A segment [a, a + count) is
// Q super-blocks of M B^2 numbers plus a remainder R < M B^2.  Super-block q
// is walked by units (q, k): a lane takes the numbers a + q M B^2 + j B^2 +
// k L + i (j < M, i < L) for k < B^2 / L, and the last L' = B^2 mod L (or L)
// numbers of each B^2 block are the edge units (one per super-block, chunk
// L'); the remainder R runs as the regular main + tail parts of the same
// launch.  Launches are split so unit counts stay 32-bit; the field's finish
// rides on the last.
template <class P>
static hipError_t launch_sib(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    auto kern = fd2_kernel<P>;
    static const int per_cu_q = [&] {
        int v = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, (const void *)kern, P::WG, 0) == hipSuccess
                   ? v : -1;
    }();
    if (per_cu_q < 0) return hipErrorInvalidDeviceFunction;
    const int per_cu = per_cu_q < 1 ? 1 : per_cu_q;
    constexpr u64 D = (u64)P::B * P::B, SB = (u64)P::SIB * D;
    const u64 lanes = (u64)num_cus * per_cu * P::WG;
    // too short for the sibling walk to pay: the same base without siblings
    if (p.count < 4 * SB) return launch_cfg<typename P::NoSib>(p, num_cus, s);
    if (p.cutoff + 1 < (u32)(P::W0 + P::W)) return hipErrorInvalidValue;
    const uint4 *tabs = nullptr;
    hipError_t e = fd2_tables<P>(s, &tabs);
    if (e != hipSuccess) return e;
    // Sibling chunk L: odd, so limb 0's low-digit lookups of a half-wave hit
    // 32 distinct bank pairs (as launch_cfg's chunks).
    const u128 seg_start = ((u128)p.start_hi << 64) | p.start_lo;
    u64 L = probe_knob("NICE_FD2_SIBCHUNK", 0);
    // a stride forced by the test hook also skips the small-field fallback
    // below (every stride the pickers can return is then reachable on a
    // field of >= 4 super-blocks)
    if (!L) L = g_force_sib_stride.load(std::memory_order_relaxed);
    // Fields of fewer than 6 rounds of the resident lanes' units at the
    // target stride: the part-filled last round of the 4-wave grid decides,
    // so the stride fills rounds (pick_small_stride over [60, 100]), and
    // below ~1.5 rounds the regular kernel's finer grid wins (b40 1e8:
    // sibling 0.227-0.239 ms at L = 65 against 0.242-0.265 regular, 1.25e8
    // 0.263-0.289 against 0.282-0.307; 9e7 ties; profiles/r05/
    // sib_small_L.log; the 4- and 8-way shards of the bench field,
    // shard_projection.log).
    // A field that overlaps a running one (pipelined submits) shares the chip
    // with it, so no round is part-filled and the per-number cost decides:
    // the large-field pick.  The 8-way shard of the bench field (1.25e8),
    // pipelined: 0.2412 ms per step at L = 105, 0.2422 at 81, 0.2481 at the
    // small-field pick (79 / 81 / 65 by shard); 2.5e8 0.486 / 0.494 / 0.500,
    // 5e7 0.110 / 0.113 / 0.112, 1e8 0.1940 / 0.1938 / 0.1952, and L = 125
    // 20-25 % slower everywhere (profiles/r06/exchange/small_L_pipe.log).
    const u64 Q0 = p.count / SB;
    if (!L && !p.overlapped && 10 * Q0 * (D / P::TCHUNK) < 60 * lanes) {
        double rounds = 0;
        L = pick_small_stride<P>(seg_start, p.count, P::TCHUNK * 3 / 4, P::TCHUNK * 5 / 4, P::LO + 1, Q0, lanes, D,
                                 rounds);
        if (10 * rounds < (double)probe_knob("NICE_FD2_SIBROUNDS", 15))
            return launch_cfg<typename P::NoSib>(p, num_cus, s);
    }
    // Target stride: TCHUNK, or 140 for the pipelined walk (LG >= 100), which
    // fills and drains its lookup pipeline once per unit and so gains from
    // longer units.  b40 bench field (pipelined, stride swept over odd L in
    // [61, 255] against the pick, profiles/r06/stride/): target 80 picked
    // 65 at 1e9 (1.917 ms per field), target 140 picks 143 (-2.5 %) there and
    // 159 at 1.25e8 (-2.7 %); a quarter into the range -0.6 / -2.8 %.  The
    // per-sibling-lookup kernels (LG 1, b40 beyond the first limb layout and
    // b42..55) gain nothing consistent from longer targets (b42 1.25e8 +14 %
    // at 140), so they keep TCHUNK.
    constexpr u64 T = P::LG >= 100 ? 140 : (u64)P::TCHUNK;
    // A lone field of the pipelined walk (a synchronous caller, the reference
    // client's pattern: nothing overlaps its last round) picks over the same
    // range by whole rounds, as the small-field path does: b40 1e9 alone
    // 1875-1887 us at L = 159 (7.99 rounds) against 1890-1947 at the model's
    // 143 (8.9 rounds), 5e8 953 against 973-1012 (profiles/r06/stride/
    // iso_L.log).  Pipelined fields keep the model's pick (no last round).
    if (!L && P::LG >= 100 && !p.overlapped) {
        double rounds = 0;
        L = pick_small_stride<P>(seg_start, p.count, T * 3 / 4, T * 3 / 2, P::LO + 1, Q0, lanes, D, rounds);
    }
    if (!L) L = pick_lane_stride<P>(seg_start, p.count, T * 3 / 4, T * 3 / 2, T, P::LO + 1);
    // chunks reach low-digit entries n mod B + i < LDE (Cfg::LDE)
    constexpr u64 LMAX = (u64)P::LDE - P::B;
    if (L % 2 == 0) L++;
    if (L > D / 4) L = (D / 4) | 1;
    if (L > LMAX) L = LMAX % 2 ? LMAX : LMAX - 1;
    const u64 U = (D + L - 1) / L, r = D - (U - 1) * L;
    const bool has_edge = r != L;
    const u64 upb = has_edge ? U - 1 : U;
    // the lanes' u16 window counters hold M L numbers
    if ((u64)P::SIB * L > 65535) return hipErrorInvalidValue;
    if (p.sib) {
        p.sib[0] = (uint32_t)P::SIB;
        p.sib[1] = (uint32_t)L;
    }
    // Launch bound: unit counts in 32 bits and, as launch_cfg's, 60 000
    // numbers per resident lane -- counted at the regular kernel's 2048 lanes
    // per CU, so a b40 launch still takes up to 3.1e10 numbers whatever the
    // sibling kernel's own occupancy.
    const u64 qmax = std::max<u64>(1, std::min<u64>(0xffffffffull / upb, ((u64)num_cus * 2048 * 60000ull) / SB));
    DetailedLaunch q = p;
    u64 left = p.count;
    const u64 tchunk = probe_knob("NICE_FD2_TCHUNK", (u64)P::TCHUNK);
    while (left) {
        u64 Q = left / SB, cnt = left;
        if (Q > qmax) {
            Q = qmax;
            cnt = Q * SB;
        }
        // regular remainder (the last launch only): rounds of one chunk per lane
        const u64 R = cnt - Q * SB;
        u64 chunk = 1, nunits = 0, tail = 0;
        if (R) {
            u64 rounds = (R + tchunk * lanes - 1) / (tchunk * lanes);
            if (rounds < 1) rounds = 1;
            chunk = (R + rounds * lanes - 1) / (rounds * lanes);
            if (chunk < 4) chunk = R < 4 ? R : 4;
            if (chunk < 1) chunk = 1;
            if (chunk > 1 && chunk % 2 == 0) chunk++;
            if (chunk > LMAX) chunk = LMAX % 2 ? LMAX : LMAX - 1;
            nunits = R / chunk;
            tail = R - nunits * chunk;
        }
        Fd2Args a{};
        NICE_PROBE_ONLY(a.stamps = g_stamps;)
        a.sib_lo = q.start_lo;
        a.sib_hi = q.start_hi;
        a.sib_chunk = (u32)L;
        a.sib_upb = (u32)upb;
        a.sib_units = (u32)(Q * upb);
        a.sib_blocks = (u32)((Q * upb + P::WG - 1) / P::WG);
        a.edge_lo = q.start_lo;
        a.edge_hi = q.start_hi;
        add_u128(a.edge_lo, a.edge_hi, upb * L);
        a.edge_chunk = (u32)r;
        a.edge_units = has_edge ? (u32)Q : 0u;
        a.edge_blocks = has_edge ? (u32)((Q + P::WG - 1) / P::WG) : 0u;
        a.start_lo = q.start_lo;
        a.start_hi = q.start_hi;
        add_u128(a.start_lo, a.start_hi, Q * SB);
        a.tail_lo = a.start_lo;
        a.tail_hi = a.start_hi;
        add_u128(a.tail_lo, a.tail_hi, nunits * chunk);
        a.nunits = (u32)nunits;
        a.chunk = (u32)chunk;
        a.tail_count = (u32)tail;
        a.main_blocks = (u32)((nunits + P::WG - 1) / P::WG);
        a.cutoff = q.cutoff;
        a.ncopies = q.hist_copies;
        a.wave_cap = 0;
        a.hist = q.hist;
        a.out = q.out;
        a.tabs = tabs;
        a.fin = left == cnt ? q.fin : FieldFinish{nullptr, nullptr, 0, 0};
        const u64 grid = (u64)a.sib_blocks + a.edge_blocks + a.main_blocks + (tail + P::WG - 1) / P::WG;
        NICE_PROBE_ONLY({
            const u64 v[6] = {grid, (u64)P::WG, L, Q * upb, R, (u64)per_cu};
            for (int k = 0; k < 6; k++) g_last_launch[k] = v[k];
        })
        hipLaunchKernelGGL(kern, dim3((u32)grid), dim3(P::WG), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (p.launches) ++*p.launches;
        add_u128(q.start_lo, q.start_hi, cnt);
        left -= cnt;
    }
    return hipSuccess;
}

}  // namespace fd2
}  // namespace nice
