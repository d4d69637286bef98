// fd2_detailed.hip -- host side of the production FD detailed kernel: the
// limb-count cuts of each base's range, the per-segment dispatch to the
// per-base launchers (fd2_part*.hip) and the entry points of kernels.h.
#include <stdlib.h>

#include <map>
#include <mutex>

#include "fd2_kernel.hpp"
#include "fd2_combos.h"

namespace nice {
namespace fd2 {

NICE_PROBE_ONLY(u64 *g_stamps = nullptr; u64 g_last_launch[6] = {};)  // phase stamps, last launch (probe build)
std::atomic<uint32_t> g_force_sib_stride{0};  // nice_debug_force_sib_stride

// ---------------------------------------------------------------------------
// Host: limb counts per segment.  For a segment [a, e) the last FD state a
// lane builds is for n = e (one step past its last number), so D1(e) = 2e+1,
// E1(e) = 3e^2+3e+1 and E2(e) = 6e+6 must fit ND, NE, NE2 radix-b^2 limbs.
// ---------------------------------------------------------------------------
struct Combo {
    int nd, ne, ne2;
};

static int limbs_of(const Nat &x, const std::vector<Nat> &pw) {
    int k = 0;
    while (k < (int)pw.size() && x.cmp(pw[k]) >= 0) k++;
    return k;  // smallest k with x < B^k
}

static Combo combo_at(uint32_t base, u128 e, const std::vector<Nat> &pw) {
    Nat n = Nat::from(e);
    Nat d1 = n;
    d1.mul_small(2);
    Nat one = Nat::from(1);
    auto add = [](Nat a, const Nat &b) {
        a.l.resize(std::max(a.l.size(), b.l.size()) + 1, 0);
        uint64_t c = 0;
        for (size_t i = 0; i < a.l.size(); i++) {
            uint64_t t = (uint64_t)a.l[i] + (i < b.l.size() ? b.l[i] : 0) + c;
            a.l[i] = (uint32_t)t;
            c = t >> 32;
        }
        a.trim();
        return a;
    };
    d1 = add(d1, one);
    Nat n3 = n;
    n3.mul_small(3);
    Nat e1 = add(add(n3.mul(n), n3), one);  // 3n^2 + 3n + 1
    Nat e2 = n;
    e2.mul_small(6);
    e2 = add(e2, Nat::from(6));
    (void)base;
    return Combo{limbs_of(d1, pw), limbs_of(e1, pw), limbs_of(e2, pw)};
}

struct BaseThresholds {
    std::vector<Nat> pw;       // B^k
    std::vector<u128> cuts;    // n where the combo changes, ascending, inside the range
    std::vector<Combo> combos; // combos[i]: segments ending in (cuts[i-1], cuts[i]]
};

static const BaseThresholds &thresholds(uint32_t base) {
    static std::mutex mu;
    static BaseThresholds cache[129];
    static bool have[129] = {};
    std::lock_guard<std::mutex> g(mu);
    BaseThresholds &t = cache[base];
    if (have[base]) return t;
    const uint32_t B = base * base;
    for (int k = 0; k < 40; k++) t.pw.push_back(Nat::pow(B, k));
    u128 rs = 0, re = 0;
    base_range(base, rs, re);
    // Walk the range: binary-search each change of combo_at.
    u128 a = rs;
    Combo cur = combo_at(base, a + 1, t.pw);
    t.combos.push_back(cur);
    while (true) {
        Combo last = combo_at(base, re, t.pw);
        if (last.nd == cur.nd && last.ne == cur.ne && last.ne2 == cur.ne2) break;
        u128 lo = a + 1, hi = re;  // smallest e in (a, re] whose combo differs
        while (lo < hi) {
            u128 mid = lo + (hi - lo) / 2;
            Combo c = combo_at(base, mid, t.pw);
            if (c.nd == cur.nd && c.ne == cur.ne && c.ne2 == cur.ne2) lo = mid + 1;
            else hi = mid;
        }
        // Segments ending at e <= lo - 1 use `cur`; the cut is at n = lo - 1
        // (a segment [x, lo-1) ends at e = lo - 1).
        t.cuts.push_back(lo - 1);
        a = lo - 1;
        cur = combo_at(base, lo, t.pw);
        t.combos.push_back(cur);
    }
    have[base] = true;
    return t;
}

// Per-base launchers, one object per part (fd2_part.hip).
hipError_t launch_part0(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
hipError_t launch_part1(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
hipError_t launch_part2(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
hipError_t launch_part3(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
hipError_t launch_part4(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
hipError_t launch_part5(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
static_assert(FD2_NPARTS == 6, "launch_part declarations");

// c: the limb counts of the segment's cut interval (cached in thresholds(),
// no bignum work per launch).
static hipError_t launch_segment(const DetailedLaunch &p, const Combo &c, int num_cus, hipStream_t s) {
    const int probe = (int)probe_knob("NICE_FD2_PROBE", 0);
#include NICE_PROBE_INC("fd2_detailed_probe_dispatch.inc")
    // Fields too small to fill the chip keep 512-thread workgroups (the
    // per-workgroup table build dominates there: b80 1e6 kernel 30 vs 38 us);
    // probe 20 forces them for b80 comparisons.
    const bool force512 = probe_knob("NICE_FD2_WG512", 0) != 0;
    const u64 small = probe_knob("NICE_FD2_SMALL", 10000000ull);  // probe: small-field threshold
    const bool wg512 = force512 || p.count < small || (probe == 20 && p.base == 80);
    using Fn = hipError_t (*)(const DetailedLaunch &, int, int, int, bool, int, hipStream_t);
    static const Fn parts[FD2_NPARTS] = {launch_part0, launch_part1, launch_part2,
                                         launch_part3, launch_part4, launch_part5};
    const hipError_t e = parts[fd2_part_of((int)p.base)](p, c.nd, c.ne, c.ne2, wg512, num_cus, s);
    return e == hipErrorNotFound ? hipErrorInvalidValue : e;
}

}  // namespace fd2

void fd2_force_sib_stride(uint32_t L) { fd2::g_force_sib_stride.store(L, std::memory_order_relaxed); }

bool fd2_supported(uint32_t base) {
    switch (base) {
#define X(b) case b:
        FD2_BASES(X)
#undef X
        return true;
    default: return false;
    }
}

size_t fd2_cuts(uint32_t base, unsigned __int128 *out, size_t cap) {
    if (!fd2_supported(base)) return 0;
    const fd2::BaseThresholds &t = fd2::thresholds(base);
    for (size_t i = 0; i < t.cuts.size() && i < cap; i++) out[i] = t.cuts[i];
    return t.cuts.size();
}

// In-range segment [start, start + count): split at the limb-count cuts, one
// launch (plus a tail launch) per piece.
hipError_t launch_detailed_fd2(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    if (!fd2_supported(p.base)) return hipErrorInvalidValue;
    const fd2::BaseThresholds &t = fd2::thresholds(p.base);
    u128 a = ((u128)p.start_hi << 64) | p.start_lo;
    const u128 e = a + p.count;
    DetailedLaunch q = p;
    // p.hist_copies: the same for every launch of the field (enqueue_detailed)
    if (p.hist_copies < kHistCopies) q.hist_copies = (uint32_t)probe_knob("NICE_FD2_COPIES", p.hist_copies);
    if (q.hist_copies < 1 || q.hist_copies > kHistCopies) q.hist_copies = kHistCopies;
    for (size_t i = 0; i <= t.cuts.size() && a < e; i++) {
        u128 stop = i < t.cuts.size() && t.cuts[i] < e ? t.cuts[i] : e;
        if (stop <= a) continue;
        q.start_lo = (uint64_t)a;
        q.start_hi = (uint64_t)(a >> 64);
        q.count = (uint64_t)(stop - a);
        q.fin = stop == e ? p.fin : FieldFinish{nullptr, nullptr, 0, 0};  // finish with the last launch
        hipError_t err = fd2::launch_segment(q, t.combos[i], num_cus, s);
        if (err != hipSuccess) return err;
        a = stop;
    }
    return hipSuccess;
}

}  // namespace nice

#include NICE_PROBE_INC("fd2_detailed_probe_exports.inc")
