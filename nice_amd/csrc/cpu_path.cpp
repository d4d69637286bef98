// cpu_path.cpp -- the reference's CPU API for the field-processing path
// (common/src/client_process.rs:150 process_range_detailed, :439
// process_range_niceonly) on the host cores: for callers of that API that
// have no GPU, and for the reference client's CPU mode.  Product code
// (independent of oracle/, which stays test-only); the GPU entry points
// never call it -- there is no silent fallback from the device.
//
// Detailed: every n's square and cube as u32 words (host_math.hpp powers),
// their base-b digits by chunked division (compile-time divisors for the
// benchmark and live bases), a digit-set popcount.  Niceonly: the MSD filter
// over the whole range (msd_prefix_filter.rs:665-674, floor 250), then the
// stride candidates of every surviving range (stride_filter.rs:139-155) with
// the early-exit niceness test (client_process.rs:222-253: the square's digits
// first, then the cube's).  `threads` splits the work into contiguous pieces
// whose results are concatenated in order, so lists stay ascending.
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nice_hip.h"
#include "host_math.hpp"

namespace {

using nice::u128;

int cpu_fail(int code, const char *msg);

inline u128 mk(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }

struct Bits {
    uint64_t w[2] = {0, 0};
    // false if the digit was already present
    bool add(uint8_t d) {
        const uint64_t b = 1ull << (d & 63);
        uint64_t &x = w[d >> 6];
        const bool fresh = (x & b) == 0;
        x |= b;
        return fresh;
    }
    uint32_t count() const { return (uint32_t)(__builtin_popcountll(w[0]) + __builtin_popcountll(w[1])); }
};

template <class BP>
uint32_t unique_digits(u128 n, const BP &bp) {
    uint32_t sq[8], cu[12];
    nice::MsdFilterT<BP>::powers(n, sq, cu);
    nice::DigitBuf d;
    Bits s;
    nice::digits_of(sq, 8, bp, d);
    for (int i = 0; i < d.n; i++) s.add(d.d[i]);
    nice::digits_of(cu, 12, bp, d);
    for (int i = 0; i < d.n; i++) s.add(d.d[i]);
    return s.count();
}

template <class BP>
bool is_nice(u128 n, const BP &bp) {
    uint32_t sq[8], cu[12];
    nice::MsdFilterT<BP>::powers(n, sq, cu);
    nice::DigitBuf d;
    Bits s;
    nice::digits_of(sq, 8, bp, d);
    for (int i = 0; i < d.n; i++)
        if (!s.add(d.d[i])) return false;
    nice::digits_of(cu, 12, bp, d);
    for (int i = 0; i < d.n; i++)
        if (!s.add(d.d[i])) return false;
    // No digit-count test: the reference's get_is_nice returns true once both
    // scans finish without a repeat (client_process.rs:258-290), so below a
    // base's valid range an n whose digits are merely distinct is listed.
    return true;
}

struct Piece {
    std::vector<uint64_t> hist;
    std::vector<std::pair<u128, uint32_t>> list;
};

template <class BP>
void detailed_piece(u128 s, u128 e, const BP &bp, uint32_t cutoff, Piece &out) {
    out.hist.assign(bp.b + 1, 0);
    for (u128 n = s; n < e; n++) {
        const uint32_t u = unique_digits(n, bp);
        out.hist[u]++;
        if (u > cutoff) out.list.emplace_back(n, u);
    }
}

// Candidates of [s, e) in the stride table's residue sequence, nice ones appended.
template <class BP>
void niceonly_range(u128 s, u128 e, const BP &bp, const nice::StrideTable &t,
                    std::vector<u128> &out) {
    const size_t R = t.residues.size();
    if (!R) return;
    const u128 M = t.modulus;
    const u128 i0 = t.index_of(s), i1 = t.index_of(e);
    u128 cyc = i0 / R;
    size_t r = (size_t)(i0 - cyc * R);
    for (u128 g = i0; g < i1; g++) {
        const u128 n = cyc * M + t.residues[r];
        if (is_nice(n, bp)) out.push_back(n);
        if (++r == R) {
            r = 0;
            cyc++;
        }
    }
}

int nthreads(int threads, u128 work) {
    int t = threads < 1 ? 1 : threads;
    if ((u128)t > work) t = work ? (int)work : 1;
    return t;
}

template <class BP>
int detailed_cpu(u128 s, u128 e, const BP &bp, int threads, uint64_t *hist, nice_number *out,
                 size_t cap, size_t *n_out) {
    const uint32_t cutoff = nice::near_miss_cutoff(bp.b);
    const u128 size = e - s;
    const int nt = nthreads(threads, size);
    std::vector<Piece> pieces(nt);
    std::vector<std::thread> ws;
    for (int i = 0; i < nt; i++) {
        const u128 a = s + size / nt * i + std::min<u128>(i, size % nt);
        const u128 b = s + size / nt * (i + 1) + std::min<u128>(i + 1, size % nt);
        if (i + 1 == nt) detailed_piece(a, b, bp, cutoff, pieces[i]);  // the caller's thread
        else ws.emplace_back([&, a, b, i] { detailed_piece(a, b, bp, cutoff, pieces[i]); });
    }
    for (auto &w : ws) w.join();
    size_t total = 0;
    for (uint32_t u = 0; u <= bp.b; u++) hist[u] = 0;
    for (auto &p : pieces) {
        for (uint32_t u = 0; u <= bp.b; u++) hist[u] += p.hist[u];
        total += p.list.size();
    }
    *n_out = total;
    if (total > cap) return cpu_fail(NICE_ERR_CAPACITY, "output capacity too small (n_out = required)");
    size_t k = 0;
    for (auto &p : pieces)
        for (auto &x : p.list)
            out[k++] = nice_number{(uint64_t)x.first, (uint64_t)(x.first >> 64), x.second, 0};
    return NICE_OK;
}

template <class BP>
int niceonly_cpu(u128 s, u128 e, const BP &bp, uint32_t k, int threads, nice_number *out,
                 size_t cap, size_t *n_out) {
    // get_valid_ranges over the whole range (msd_prefix_filter.rs:665-674)
    std::vector<std::pair<u128, u128>> ranges;
    nice::MsdFilterT<BP> f(bp);
    f.valid_ranges(s, e, 0, 250, [&](u128 a, u128 b) { ranges.emplace_back(a, b); });
    const nice::StrideTable table(bp.b, k);
    const int nt = nthreads(threads, ranges.size());
    std::vector<std::vector<u128>> found(nt);
    std::vector<std::thread> ws;
    const size_t nr = ranges.size();
    for (int i = 0; i < nt; i++) {
        const size_t a = nr / nt * i + std::min<size_t>(i, nr % nt);
        const size_t b = nr / nt * (i + 1) + std::min<size_t>(i + 1, nr % nt);
        auto run = [&, a, b, i] {
            for (size_t q = a; q < b; q++) niceonly_range(ranges[q].first, ranges[q].second, bp, table, found[i]);
        };
        if (i + 1 == nt) run();
        else ws.emplace_back(run);
    }
    for (auto &w : ws) w.join();
    size_t total = 0;
    for (auto &v : found) total += v.size();
    *n_out = total;
    if (total > cap) return cpu_fail(NICE_ERR_CAPACITY, "output capacity too small (n_out = required)");
    size_t q = 0;
    for (auto &v : found)
        for (u128 n : v) out[q++] = nice_number{(uint64_t)n, (uint64_t)(n >> 64), bp.b, 0};
    return NICE_OK;
}

// Compile-time divisors for the benchmark and live bases, run-time otherwise.
template <class F>
int with_base(uint32_t base, F &&f) {
    switch (base) {
    case 10: return f(nice::CtBase<10>{});
    case 40: return f(nice::CtBase<40>{});
    case 50: return f(nice::CtBase<50>{});
    case 52: return f(nice::CtBase<52>{});
    case 53: return f(nice::CtBase<53>{});
    case 54: return f(nice::CtBase<54>{});
    case 80: return f(nice::CtBase<80>{});
    default: return f(nice::RtBase(base));
    }
}

}  // namespace

namespace nice {
void set_last_error(const char *msg);  // nice_abi.cpp: nice_last_error()'s thread-local message
}

namespace {
int cpu_fail(int code, const char *msg) {
    nice::set_last_error(msg);
    return code;
}
}  // namespace

extern "C" int nice_cpu_process_range_detailed(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                                               uint64_t end_hi, uint32_t base, int32_t threads,
                                               uint64_t *hist, nice_number *out, size_t cap,
                                               size_t *n_out) {
    if (!hist || !n_out || (cap && !out)) return cpu_fail(NICE_ERR_INVALID, "null output pointer");
    if (base < 2 || base > 128) return cpu_fail(NICE_ERR_INVALID, "base must be in 2..128");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (e < s) return cpu_fail(NICE_ERR_INVALID, "range end before start");
    return with_base(base, [&](const auto &bp) { return detailed_cpu(s, e, bp, threads, hist, out, cap, n_out); });
}

extern "C" int nice_cpu_process_range_niceonly(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                                               uint64_t end_hi, uint32_t base, uint32_t stride_k,
                                               int32_t threads, nice_number *out, size_t cap,
                                               size_t *n_out) {
    if (!n_out || (cap && !out)) return cpu_fail(NICE_ERR_INVALID, "null output pointer");
    if (base < 2 || base > 128) return cpu_fail(NICE_ERR_INVALID, "base must be in 2..128");
    const uint32_t k = stride_k ? stride_k : 2;
    uint64_t bk = 1;
    for (uint32_t i = 0; i < k; i++) bk *= base;
    if (k > 4 || (base - 1) * bk > (1ull << 32)) return cpu_fail(NICE_ERR_INVALID, "stride table too large (k)");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (e < s) return cpu_fail(NICE_ERR_INVALID, "range end before start");
    *n_out = 0;
    if (s == e) return NICE_OK;
    return with_base(base, [&](const auto &bp) { return niceonly_cpu(s, e, bp, k, threads, out, cap, n_out); });
}
