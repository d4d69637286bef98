// host_math.hpp -- host-side number theory for the field-processing path.
//
// Product code (not the oracle): base ranges, near-miss cutoff, residue / LSD
// / stride tables and the MSD-prefix filter that feeds the niceonly kernel.
// Each function restates the cited reference function; tests/ check them
// against oracle/ and the reference's golden vectors.
#pragma once

#include <mutex>

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <utility>
#include <vector>

namespace nice {

typedef unsigned __int128 u128;

// ---------------------------------------------------------------------------
// Small arbitrary-precision naturals (u32 limbs, little endian) -- only what
// base_range needs: b^e and x^p comparisons.
// ---------------------------------------------------------------------------
struct Nat {
    std::vector<uint32_t> l;
    void trim() {
        while (!l.empty() && l.back() == 0) l.pop_back();
    }
    static Nat pow(uint32_t b, uint32_t e) {
        Nat r;
        r.l.push_back(1);
        for (uint32_t i = 0; i < e; i++) r.mul_small(b);
        return r;
    }
    static Nat from(u128 v) {
        Nat r;
        for (int i = 0; i < 4; i++) r.l.push_back((uint32_t)(v >> (32 * i)));
        r.trim();
        return r;
    }
    void mul_small(uint32_t m) {
        uint64_t c = 0;
        for (auto &x : l) {
            uint64_t t = (uint64_t)x * m + c;
            x = (uint32_t)t;
            c = t >> 32;
        }
        if (c) l.push_back((uint32_t)c);
    }
    Nat mul(const Nat &o) const {
        Nat r;
        r.l.assign(l.size() + o.l.size() + 1, 0);
        for (size_t i = 0; i < l.size(); i++) {
            uint64_t c = 0;
            for (size_t j = 0; j < o.l.size(); j++) {
                uint64_t t = (uint64_t)l[i] * o.l[j] + r.l[i + j] + c;
                r.l[i + j] = (uint32_t)t;
                c = t >> 32;
            }
            size_t k = i + o.l.size();
            while (c) {
                uint64_t t = (uint64_t)r.l[k] + c;
                r.l[k++] = (uint32_t)t;
                c = t >> 32;
            }
        }
        r.trim();
        return r;
    }
    int cmp(const Nat &o) const {
        if (l.size() != o.l.size()) return l.size() < o.l.size() ? -1 : 1;
        for (size_t i = l.size(); i-- > 0;)
            if (l[i] != o.l[i]) return l[i] < o.l[i] ? -1 : 1;
        return 0;
    }
    size_t bits() const { return l.empty() ? 0 : 32 * (l.size() - 1) + (32 - __builtin_clz(l.back())); }
    bool to_u128(u128 &out) const {
        if (l.size() > 4) return false;
        out = 0;
        for (size_t i = l.size(); i-- > 0;) out = (out << 32) | l[i];
        return true;
    }
};

// Smallest x with x^p >= v (malachite CeilingRoot); false if x >= 2^128.
inline bool ceil_root(const Nat &v, int p, u128 &out) {
    size_t rb = (v.bits() + p - 1) / p + 1;
    u128 lo = 0, hi = rb >= 128 ? ~(u128)0 : ((u128)1 << rb);
    auto powp = [&](u128 x) {
        Nat n = Nat::from(x);
        Nat r = n.mul(n);
        return p == 3 ? r.mul(n) : r;
    };
    while (lo < hi) {
        u128 mid = lo + (hi - lo) / 2;
        if (powp(mid).cmp(v) >= 0) hi = mid;
        else lo = mid + 1;
    }
    if (powp(lo).cmp(v) < 0) return false;
    out = lo;
    return true;
}

// common/src/base_range.rs:14-54.  1: range found, 0: none, -1: exceeds u128.
inline int base_range(uint32_t b, u128 &start, u128 &end) {
    uint32_t k = b / 5;
    bool ok = true;
    switch (b % 5) {
    case 0:
        if (k == 0) return 0;
        ok &= ceil_root(Nat::pow(b, 3 * k - 1), 3, start);
        ok &= Nat::pow(b, k).to_u128(end);
        break;
    case 1:
        return 0;
    case 2:
        ok &= Nat::pow(b, k).to_u128(start);
        ok &= ceil_root(Nat::pow(b, 3 * k + 1), 3, end);
        break;
    case 3:
        ok &= ceil_root(Nat::pow(b, 3 * k + 1), 3, start);
        ok &= ceil_root(Nat::pow(b, 2 * k + 1), 2, end);
        break;
    default:
        ok &= ceil_root(Nat::pow(b, 2 * k + 1), 2, start);
        ok &= ceil_root(Nat::pow(b, 3 * k + 2), 3, end);
        break;
    }
    if (!ok) return -1;
    return start < end ? 1 : 0;
}

// base_range, computed once per base (the bignum roots cost ~13 us, which is
// a third of a 1e6 field's wall time if paid per call).
inline int base_range_cached(uint32_t b, u128 &start, u128 &end) {
    struct Slot {
        std::once_flag once;
        int rc = 0;
        u128 s = 0, e = 0;
    };
    static Slot slots[129];
    if (b > 128) return base_range(b, start, end);
    Slot &sl = slots[b];
    std::call_once(sl.once, [&] { sl.rc = base_range(b, sl.s, sl.e); });
    start = sl.s;
    end = sl.e;
    return sl.rc;
}

// common/src/number_stats.rs:15-17 (f32 arithmetic, as the reference).
inline uint32_t near_miss_cutoff(uint32_t b) {
    volatile float f = (float)b * 0.9f;
    return (uint32_t)std::floor(f);
}

// common/src/residue_filter.rs:6-11
inline std::vector<uint32_t> residue_filter(uint32_t b) {
    std::vector<uint32_t> out;
    const uint32_t m = b - 1, target = b * (b - 1) / 2 % m;
    for (uint32_t r = 0; r < m; r++)
        if ((r * r + r * r * r) % m == target) out.push_back(r);
    return out;
}

// common/src/lsd_filter.rs:174-224 with extract_digits (:132-148), which stops
// once the remaining value is zero.
inline std::vector<uint8_t> lsd_bitmap(uint32_t b, uint32_t k) {
    uint64_t mod = 1;
    for (uint32_t i = 0; i < k; i++) mod *= b;
    std::vector<uint8_t> bm(mod);
    auto digit_set = [&](u128 v, uint64_t s[2]) {
        s[0] = s[1] = 0;
        for (uint32_t i = 0; i < k; i++) {
            uint32_t d = (uint32_t)(v % b);
            s[d >> 6] |= 1ull << (d & 63);
            v /= b;
            if (v == 0) break;
        }
    };
    for (uint64_t x = 0; x < mod; x++) {
        uint64_t a[2], c[2];
        digit_set(((u128)x * x) % mod, a);
        digit_set(((u128)x * x * x) % mod, c);
        bm[x] = ((a[0] & c[0]) | (a[1] & c[1])) == 0;
    }
    return bm;
}

// common/src/stride_filter.rs:40-87 (M = (b-1) * b^k, valid residues mod M).
struct StrideTable {
    uint64_t modulus = 0;
    std::vector<uint32_t> residues;

    StrideTable() {}
    StrideTable(uint32_t b, uint32_t k) {
        uint64_t bk = 1;
        for (uint32_t i = 0; i < k; i++) bk *= b;
        const uint64_t bm1 = b - 1;
        modulus = bm1 * bk;
        std::vector<uint8_t> rok(bm1, 0);
        for (uint32_t r : residue_filter(b)) rok[r] = 1;
        std::vector<uint8_t> lsd = lsd_bitmap(b, k);
        for (uint64_t r = 0; r < modulus; r++)
            if (rok[r % bm1] && lsd[r % bk]) residues.push_back((uint32_t)r);
    }
    // Global residue-sequence index of the first valid candidate >= x:
    // idx(x) = (x / M) * R + lower_bound(residues, x mod M).
    // stride_filter.rs:99-124 in index form.
    u128 index_of(u128 x) const {
        const uint64_t r = (uint64_t)(x % modulus);
        const u128 cyc = x / modulus;
        const uint64_t lb =
            std::lower_bound(residues.begin(), residues.end(), (uint32_t)r) - residues.begin();
        return cyc * residues.size() + lb;
    }
};

// ---------------------------------------------------------------------------
// MSD prefix filter, msd_prefix_filter.rs:382-674.
// ---------------------------------------------------------------------------

// Digits (least significant first) of a value held in u32 words, via chunks of
// D = b^E < 2^32.  BP supplies b, D, E: compile-time (CtBase, divisions become
// multiply-high sequences) or run-time (RtBase).
struct DigitBuf {
    uint8_t d[400];
    int n;
};

struct RtBase {
    uint32_t b, D, E;
    explicit RtBase(uint32_t base) : b(base), D(1), E(0) {
        while ((uint64_t)D * b < (1ull << 32)) {
            D *= b;
            E++;
        }
    }
};
template <uint32_t BASE>
struct CtBase {
    static constexpr uint32_t b = BASE;
    static constexpr uint32_t E = []() { uint32_t e = 0; uint64_t d = 1; while (d * BASE < (1ull << 32)) { d *= BASE; e++; } return e; }();
    static constexpr uint32_t D = []() { uint64_t d = 1; while (d * BASE < (1ull << 32)) d *= BASE; return (uint32_t)d; }();
};

template <class BP>
inline void digits_of(uint32_t *w, int nw, const BP &bp, DigitBuf &out) {
    out.n = 0;
    int top = nw - 1;
    while (top >= 0 && w[top] == 0) top--;
    while (top >= 0) {
        uint64_t rem = 0;
        for (int i = top; i >= 0; i--) {
            uint64_t cur = (rem << 32) | w[i];
            w[i] = (uint32_t)(cur / bp.D);
            rem = cur % bp.D;
        }
        while (top >= 0 && w[top] == 0) top--;
        uint32_t c = (uint32_t)rem;
        if (top >= 0) {
            for (uint32_t q = 0; q < bp.E; q++) {
                out.d[out.n++] = (uint8_t)(c % bp.b);
                c /= bp.b;
            }
        } else {
            while (c) {
                out.d[out.n++] = (uint8_t)(c % bp.b);
                c /= bp.b;
            }
        }
    }
}

template <class BP>
struct MsdFilterT {
    BP bp;
    explicit MsdFilterT(const BP &p) : bp(p) {}

    // n^2 and n^3 of x as u32 words (only the words that can be non-zero).
    static void powers(u128 x, uint32_t sq[8], uint32_t cu[12]) {
        uint32_t n[4] = {(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
        int nn = 4;
        while (nn > 1 && n[nn - 1] == 0) nn--;
        for (int i = 0; i < 8; i++) sq[i] = 0;
        for (int i = 0; i < nn; i++) {
            uint64_t c = 0;
            for (int j = 0; j < nn; j++) {
                uint64_t t = (uint64_t)n[i] * n[j] + sq[i + j] + c;
                sq[i + j] = (uint32_t)t;
                c = t >> 32;
            }
            sq[i + nn] = (uint32_t)c;
        }
        for (int i = 0; i < 12; i++) cu[i] = 0;
        for (int i = 0; i < 2 * nn; i++) {
            uint64_t c = 0;
            for (int j = 0; j < nn; j++) {
                uint64_t t = (uint64_t)sq[i] * n[j] + cu[i + j] + c;
                cu[i + j] = (uint32_t)t;
                c = t >> 32;
            }
            cu[i + nn] = (uint32_t)c;
        }
    }

    static bool dup(const uint8_t *d, int n) {
        uint64_t s[2] = {0, 0};
        for (int i = 0; i < n; i++) {
            uint64_t bit = 1ull << (d[i] & 63);
            if (s[d[i] >> 6] & bit) return true;
            s[d[i] >> 6] |= bit;
        }
        return false;
    }
    static bool overlap(const uint8_t *a, int na, const uint8_t *c, int nc) {
        uint64_t s[2] = {0, 0};
        for (int i = 0; i < na; i++) s[a[i] >> 6] |= 1ull << (a[i] & 63);
        for (int i = 0; i < nc; i++)
            if (s[c[i] >> 6] & (1ull << (c[i] & 63))) return true;
        return false;
    }
    static int common_msd(const DigitBuf &x, const DigitBuf &y) {
        int m = std::min(x.n, y.n), c = 0;
        for (int i = 0; i < m; i++) {
            if (x.d[x.n - 1 - i] != y.d[y.n - 1 - i]) break;
            c++;
        }
        return c;
    }

    // has_duplicate_msd_prefix on [s, e) (msd_prefix_filter.rs:382-563).
    bool skippable(u128 s, u128 e) const {
        if (e - s == 1) return false;
        const u128 first = s, last = e - 1;
        uint32_t fsq[8], fcu[12], lsq[8], lcu[12];
        powers(first, fsq, fcu);
        powers(last, lsq, lcu);
        DigitBuf ds, de, cs, ce;
        digits_of(fsq, 8, bp, ds);
        digits_of(lsq, 8, bp, de);
        if (ds.n != de.n) return false;
        const int sp = common_msd(ds, de);
        const uint8_t *sqp = ds.d + (ds.n - sp);
        if (dup(sqp, sp)) return true;
        digits_of(fcu, 12, bp, cs);
        digits_of(lcu, 12, bp, ce);
        if (cs.n != ce.n) return false;
        const int cp = common_msd(cs, ce);
        const uint8_t *cup = cs.d + (cs.n - cp);
        if (dup(cup, cp)) return true;
        if (overlap(sqp, sp, cup, cp)) return true;
        // Filter C (k = MSD_LSD_OVERLAP_K_VALUE = 2): uses *first*'s two LSDs.
        const uint64_t bk = (uint64_t)bp.b * bp.b;
        const bool one_class = (uint64_t)(last >> 64) == 0
                                   ? (uint64_t)first / bk == (uint64_t)last / bk
                                   : first / bk == last / bk;
        if (one_class) {
            const int ls = std::min(ds.n, 2), lc = std::min(cs.n, 2);
            if (overlap(sqp, sp, ds.d, ls) || overlap(cup, cp, cs.d, lc) ||
                overlap(sqp, sp, cs.d, lc) || overlap(cup, cp, ds.d, ls) || dup(ds.d, ls) ||
                dup(cs.d, lc) || overlap(ds.d, ls, cs.d, lc))
                return true;
        }
        return false;
    }

    // get_valid_ranges_recursive (msd_prefix_filter.rs:583-658), depth <= 22,
    // subdivision factor 2.  Appends surviving [s, e) pairs.
    template <class F>
    void valid_ranges(u128 s, u128 e, uint32_t depth, u128 floor_size, F &&emit) const {
        if (depth >= 22 || e - s <= floor_size) {
            emit(s, e);
            return;
        }
        if (skippable(s, e)) return;
        if (e - s < floor_size * 2) {
            emit(s, e);
            return;
        }
        const u128 half = (e - s) / 2;
        valid_ranges(s, s + half, depth + 1, floor_size, emit);
        valid_ranges(s + half, e, depth + 1, floor_size, emit);
    }
};

// Runtime-dispatched MSD producer: compile-time bases for the benchmark /
// production bases, a runtime-divisor instance for everything else.
struct MsdRunner {
    virtual ~MsdRunner() {}
    virtual bool skippable(u128 s, u128 e) const = 0;
    virtual void ranges(u128 s, u128 e, u128 floor_size,
                        std::vector<std::pair<u128, u128>> &out) const = 0;
};
template <class BP>
struct MsdRunnerT : MsdRunner {
    MsdFilterT<BP> f;
    explicit MsdRunnerT(const BP &bp) : f(bp) {}
    bool skippable(u128 s, u128 e) const override { return f.skippable(s, e); }
    void ranges(u128 s, u128 e, u128 floor_size,
                std::vector<std::pair<u128, u128>> &out) const override {
        f.valid_ranges(s, e, 0, floor_size, [&](u128 a, u128 b) { out.emplace_back(a, b); });
    }
};
inline std::unique_ptr<MsdRunner> make_msd(uint32_t base) {
    switch (base) {
    case 40: return std::unique_ptr<MsdRunner>(new MsdRunnerT<CtBase<40>>(CtBase<40>{}));
    case 50: return std::unique_ptr<MsdRunner>(new MsdRunnerT<CtBase<50>>(CtBase<50>{}));
    case 80: return std::unique_ptr<MsdRunner>(new MsdRunnerT<CtBase<80>>(CtBase<80>{}));
    default: return std::unique_ptr<MsdRunner>(new MsdRunnerT<RtBase>(RtBase(base)));
    }
}

// Reference client chunking (client/src/main.rs:158-168):
// 1e6 * clamp(ceil(size / (1e6 * 1e5)), 1, 1000).
inline u128 client_chunk_size(u128 size) {
    const u128 def = 1000000, target = 100000;
    u128 mult = (size + def * target - 1) / (def * target);
    mult = std::max<u128>(1, std::min<u128>(mult, 1000));
    return def * mult;
}

}  // namespace nice
