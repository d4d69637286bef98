// radix_fast.hpp -- in-range fast paths for the niceonly kernels (b40/50/52/53/54/80).
//
// Inside a base's valid range n^2 and n^3 have exactly D2 and D3 base-b digits
// (base_range.rs:14-32), so both fit fixed radix-B = b^2 limb arrays sized at
// compile time.  Converting n to NX radix-B limbs and multiplying limb-wise
// (every column sum < 2^32, so u32 arithmetic throughout) replaces the generic
// path's chunked long division of 8- and 12-word numbers by b^E: the digit
// pairs fall out of the limbs, and the dependent chains are a few steps long
// instead of hundreds.  Used by
//   * is_nice_fast      == get_is_nice (client_process.rs:222-253): with
//                          exactly b digits in n^2 and n^3, "no digit
//                          repeats" is "the digit union has b members";
//   * msd_skippable_fast == has_duplicate_msd_prefix (msd_prefix_filter.rs:
//                          382-563) incl. Filter C, for [first, last] in range.
// Both agree bit-for-bit with the generic device functions (nice_device.hpp,
// niceonly.hip) on in-range input; the GPU parity tests compare the candidate
// sets and nice lists against the CPU path.  The same templates also compile
// for the host (plain integer C++), exported as test hooks so the CPU suite
// checks them against the oracle on random in-range inputs.
#pragma once

#include "nice_device.hpp"

namespace nice {

template <int BASE>
struct Radix {
    static constexpr u32 B = (u32)BASE * BASE;
    static constexpr int k = BASE / 5, r5 = BASE % 5;
    static constexpr int D2 = r5 == 0 ? 2 * k : (r5 == 4 ? 2 * k + 2 : 2 * k + 1);
    static constexpr int D3 = r5 == 0 ? 3 * k : (r5 == 2 ? 3 * k + 1 : 3 * k + 2);
    static constexpr int DN = r5 == 0 ? k : k + 1;
    static constexpr int NX = cdiv(DN, 2), NS = cdiv(D2, 2), NC = cdiv(D3, 2);
    static constexpr int MW = (BASE + 31) / 32;
    static constexpr bool FITS64 = []() {
        unsigned long long v = 1;
        for (int i = 0; i < NX; i++) {
            if (v > ~0ull / B) return false;
            v *= B;
        }
        return true;
    }();
    // column sums: NX * (B-1)^2 (square) and NX * (B-1)^2 (cube, S limbs < B)
    static_assert((unsigned long long)NX * (B - 1) * (B - 1) + B < (1ull << 32), "u32 columns");
};

template <int MW>
__host__ __device__ __forceinline__ u32 mset(u32 (&m)[MW], u32 d) {
    u32 dup = 0;
#pragma unroll
    for (int w = 0; w < MW; w++) {
        const u32 bit = (d >> 5) == (u32)w ? 1u << (d & 31) : 0u;
        dup |= m[w] & bit;
        m[w] |= bit;
    }
    return dup;
}
template <int MW>
__host__ __device__ __forceinline__ bool moverlap(const u32 (&a)[MW], const u32 (&b)[MW]) {
    u32 o = 0;
#pragma unroll
    for (int w = 0; w < MW; w++) o |= a[w] & b[w];
    return o != 0;
}

// B^e fits 32 bits (B^e <= 2^32).
constexpr bool pow_le32(unsigned long long b, int e) {
    unsigned long long v = 1;
    for (int i = 0; i < e; i++) {
        v *= b;
        if (v > (1ull << 32)) return false;
    }
    return true;
}

// n (in range, < B^NX) as NX radix-B limbs.
template <int BASE>
__host__ __device__ __forceinline__ void to_limbs(u64 lo, u64 hi, u32 (&X)[Radix<BASE>::NX]) {
    constexpr u32 B = Radix<BASE>::B;
    if constexpr (Radix<BASE>::FITS64) {  // n < B^NX < 2^64 (b40, b50)
        // two limbs per u64 division by B^2 (< 2^32), the pair split in 32
        // bits; once the rest fits 32 bits (B^(NX-j) <= 2^32) all in 32 bits
        (void)hi;
        constexpr u64 B2 = (u64)B * B;
        u64 v = lo;
#pragma unroll
        for (int j = 0; j < Radix<BASE>::NX; j += 2) {
            if (j + 1 == Radix<BASE>::NX) {  // the top limb: v < B
                X[j] = (u32)v;
            } else if (pow_le32(B, Radix<BASE>::NX - j)) {
                const u32 w = (u32)v, q = w / (u32)B2, r = w - q * (u32)B2;
                X[j] = r % B;
                X[j + 1] = r / B;
                v = q;
            } else {
                const u64 q = v / B2;
                const u32 r = (u32)(v - q * B2);
                X[j] = r % B;
                X[j + 1] = r / B;
                v = q;
            }
        }
    } else {
        u32 w[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
#pragma unroll
        for (int j = 0; j < Radix<BASE>::NX; j++) {
            u64 rem = 0;
#pragma unroll
            for (int q = 3; q >= 0; q--) {
                const u64 cur = (rem << 32) | w[q];
                w[q] = (u32)(cur / B);
                rem = cur - (u64)w[q] * B;
            }
            X[j] = (u32)rem;
        }
    }
}

// S = X^2 (NS limbs), C = S * X (NC limbs), normalised radix B.
template <int BASE>
__host__ __device__ __forceinline__ void square_limbs(const u32 (&X)[Radix<BASE>::NX], u32 (&S)[Radix<BASE>::NS]) {
    using R = Radix<BASE>;
    u32 acc[2 * R::NX];
#pragma unroll
    for (int t = 0; t < 2 * R::NX; t++) acc[t] = 0;
#pragma unroll
    for (int i = 0; i < R::NX; i++)
#pragma unroll
        for (int j = 0; j < R::NX; j++) acc[i + j] += X[i] * X[j];
    u32 cy = 0;
#pragma unroll
    for (int t = 0; t < R::NS; t++) {
        const u32 v = (t < 2 * R::NX ? acc[t] : 0u) + cy;
        cy = v / R::B;
        S[t] = v - cy * R::B;
    }
}
template <int BASE>
__host__ __device__ __forceinline__ void cube_limbs(const u32 (&S)[Radix<BASE>::NS], const u32 (&X)[Radix<BASE>::NX],
                                           u32 (&C)[Radix<BASE>::NC]) {
    using R = Radix<BASE>;
    u32 acc[R::NS + R::NX];
#pragma unroll
    for (int t = 0; t < R::NS + R::NX; t++) acc[t] = 0;
#pragma unroll
    for (int i = 0; i < R::NS; i++)
#pragma unroll
        for (int j = 0; j < R::NX; j++) acc[i + j] += S[i] * X[j];
    u32 cy = 0;
#pragma unroll
    for (int t = 0; t < R::NC; t++) {
        const u32 v = (t < R::NS + R::NX ? acc[t] : 0u) + cy;
        cy = v / R::B;
        C[t] = v - cy * R::B;
    }
}

__host__ __device__ __forceinline__ u32 popc32(u32 x) { return (u32)__builtin_popcount(x); }

// Digit bits of a radix-B limb v (two base-b digits, or one when `two` is
// false: the top limb of an odd digit count) OR-ed into m, by VALU: the high
// digit by one multiply-high, the low one by a multiply-subtract, each bit by
// a 64-bit shift (digits >= 64 go to word 2 at MW = 3).  No repeat test: the
// caller counts the union.
template <int BASE>
__host__ __device__ __forceinline__ void or_limb(u32 v, bool two, u32 (&m)[Radix<BASE>::MW]) {
    constexpr int MW = Radix<BASE>::MW;
    const u32 d1 = v / BASE, d0 = v - d1 * BASE;
    if constexpr (MW == 2) {
        const u64 bits = (1ull << d0) | (two ? 1ull << d1 : 0ull);
        m[0] |= (u32)bits;
        m[1] |= (u32)(bits >> 32);
    } else {
        static_assert(MW == 3, "in-range fast bases are 33..96");
        const u64 b0 = d0 < 64 ? 1ull << (d0 & 63) : 0ull, b1 = two && d1 < 64 ? 1ull << (d1 & 63) : 0ull;
        m[0] |= (u32)(b0 | b1);
        m[1] |= (u32)((b0 | b1) >> 32);
        m[2] |= (d0 >= 64 ? 1u << (d0 & 31) : 0u) | (two && d1 >= 64 ? 1u << (d1 & 31) : 0u);
    }
}

template <int BASE, int N>
__host__ __device__ __forceinline__ u32 limbs_popcount(const u32 (&A)[N], int D, u32 (&m)[Radix<BASE>::MW]) {
#pragma unroll
    for (int t = 0; t < N; t++) or_limb<BASE>(A[t], 2 * t + 1 < D, m);
    u32 c = 0;
#pragma unroll
    for (int w = 0; w < Radix<BASE>::MW; w++) c += popc32(m[w]);
    return c;
}

// Two-word bases: each limb's two digit bits from a pair-mask table in LDS
// (entry v marks v's digits v / b and v % b; one ds_read_b64 instead of ~7
// VALU).  A top limb holding one digit keeps the VALU path.
template <int BASE, int N>
__device__ __forceinline__ u32 limbs_popcount_tab(const u32 (&A)[N], int D, u32 (&m)[2], const uint2 *tab) {
#pragma unroll
    for (int t = 0; t < N; t++) {
        if (2 * t + 1 < D) {
            const uint2 e = tab[A[t]];
            m[0] |= e.x;
            m[1] |= e.y;
        } else {
            or_limb<BASE>(A[t], false, m);
        }
    }
    return popc32(m[0]) + popc32(m[1]);
}

// get_is_nice (client_process.rs:222-253) for in-range n.  Inside the valid
// range n^2 and n^3 have exactly D2 + D3 = b digits, so "no digit repeats"
// (the reference's early-exit scan, n^2 then n^3) is "the union of their
// digits has b members": no per-digit test or branch, one popcount after n^2
// (a repeat there ends it; the cube is multiplied out only for the ~1-2 % of
// stride candidates whose square is repeat-free) and one after n^3.
template <int BASE>
__host__ __device__ __forceinline__ bool is_nice_limbs(const u32 (&X)[Radix<BASE>::NX]) {
    using R = Radix<BASE>;
    u32 S[R::NS];
    square_limbs<BASE>(X, S);
    u32 m[R::MW];
#pragma unroll
    for (int w = 0; w < R::MW; w++) m[w] = 0;
    if (limbs_popcount<BASE>(S, R::D2, m) != (u32)R::D2) return false;
    u32 C[R::NC];
    cube_limbs<BASE>(S, X, C);
    return limbs_popcount<BASE>(C, R::D3, m) == (u32)BASE;
}

// First half of is_nice_limbs: n^2 repeat-free (the stride candidates that
// pass go on to the cube; niceonly_kernel batches them, see there).
template <int BASE>
__host__ __device__ __forceinline__ bool square_ok(u64 lo, u64 hi) {
    using R = Radix<BASE>;
    u32 X[R::NX], S[R::NS];
    to_limbs<BASE>(lo, hi, X);
    square_limbs<BASE>(X, S);
    u32 m[R::MW];
#pragma unroll
    for (int w = 0; w < R::MW; w++) m[w] = 0;
    return limbs_popcount<BASE>(S, R::D2, m) == (u32)R::D2;
}

template <int BASE>
__host__ __device__ __forceinline__ bool is_nice_fast(u64 lo, u64 hi) {
    u32 X[Radix<BASE>::NX];
    to_limbs<BASE>(lo, hi, X);
    return is_nice_limbs<BASE>(X);
}

// The same two tests with the LDS pair table (two-word bases, see above).
template <int BASE>
__device__ __forceinline__ bool square_ok_tab_limbs(const u32 (&X)[Radix<BASE>::NX], const uint2 *tab) {
    using R = Radix<BASE>;
    static_assert(R::MW == 2, "pair table: two-word bases");
    u32 S[R::NS];
    square_limbs<BASE>(X, S);
    u32 m[2] = {0, 0};
    return limbs_popcount_tab<BASE>(S, R::D2, m, tab) == (u32)R::D2;
}
template <int BASE>
__device__ __forceinline__ bool square_ok_tab(u64 lo, u64 hi, const uint2 *tab) {
    u32 X[Radix<BASE>::NX];
    to_limbs<BASE>(lo, hi, X);
    return square_ok_tab_limbs<BASE>(X, tab);
}
template <int BASE>
__device__ __forceinline__ bool is_nice_tab(u64 lo, u64 hi, const uint2 *tab) {
    using R = Radix<BASE>;
    static_assert(R::MW == 2, "pair table: two-word bases");
    u32 X[R::NX], S[R::NS], C[R::NC];
    to_limbs<BASE>(lo, hi, X);
    square_limbs<BASE>(X, S);
    u32 m[2] = {0, 0};
    if (limbs_popcount_tab<BASE>(S, R::D2, m, tab) != (u32)R::D2) return false;
    cube_limbs<BASE>(S, X, C);
    return limbs_popcount_tab<BASE>(C, R::D3, m, tab) == (u32)BASE;
}

// Unique-digit count of in-range n by the same limb path (test hook: checks
// every digit bit the niceness test relies on against the oracle).
template <int BASE>
__host__ __device__ __forceinline__ u32 unique_fast(u64 lo, u64 hi) {
    using R = Radix<BASE>;
    u32 X[R::NX], S[R::NS], C[R::NC];
    to_limbs<BASE>(lo, hi, X);
    square_limbs<BASE>(X, S);
    cube_limbs<BASE>(S, X, C);
    u32 m[R::MW];
#pragma unroll
    for (int w = 0; w < R::MW; w++) m[w] = 0;
    limbs_popcount<BASE>(S, R::D2, m);
    return limbs_popcount<BASE>(C, R::D3, m);
}

// Common most-significant prefix of two D-digit limb arrays: its digit mask
// and whether a digit repeats inside it.  Limbs are walked from the top (fully
// unrolled, static indices); the walk stops at the first differing digit.
template <int BASE, int N>
__host__ __device__ __forceinline__ void msd_prefix(const u32 (&F)[N], const u32 (&L)[N], int D,
                                           u32 (&m)[Radix<BASE>::MW], u32 &dup) {
#pragma unroll
    for (int w = 0; w < Radix<BASE>::MW; w++) m[w] = 0;
    dup = 0;
    bool live = true;
#pragma unroll
    for (int t = N - 1; t >= 0; t--) {
        if (live) {
            const u32 f = F[t], l = L[t];
            const u32 fh = f / BASE, lh = l / BASE;
            if (2 * t + 1 < D) {  // high digit of the limb (absent above the top digit)
                if (fh != lh) live = false;
                else dup |= mset(m, fh);
            }
            if (live) {
                if (f != l) live = false;  // high digits equal, so the low ones differ
                else dup |= mset(m, f - fh * BASE);
            }
        }
    }
}

// msd_prefix for two-word bases with the LDS pair-mask table: per limb one
// table read and a few selects instead of a test-and-set per digit; "a digit
// repeats in the prefix" is "the prefix mask has fewer bits than the prefix
// has digits".  The walk stops as soon as no lane of the wave is still inside
// its common prefix.
template <int BASE, int N>
__device__ __forceinline__ void msd_prefix_tab(const u32 (&F)[N], const u32 (&L)[N], int D, u32 (&m)[2], u32 &dup,
                                               const uint2 *tab) {
    m[0] = m[1] = 0;
    u32 nd = 0;
    bool live = true;
#pragma unroll
    for (int t = N - 1; t >= 0; t--) {
        if (!__builtin_amdgcn_ballot_w64(live)) break;  // wave-uniform
        const u32 f = F[t], l = L[t];
        const bool eq = live && f == l;
        if (2 * t + 1 < D) {
            const u32 fh = f / BASE, lh = l / BASE;
            const bool heq = live && !eq && fh == lh;  // only the high digit is common
            const uint2 e = tab[f];
            const u64 hb = 1ull << fh;
            m[0] |= eq ? e.x : (heq ? (u32)hb : 0u);
            m[1] |= eq ? e.y : (heq ? (u32)(hb >> 32) : 0u);
            nd += eq ? 2u : (heq ? 1u : 0u);
        } else {  // the top limb of an odd digit count: one digit
            const u64 b = 1ull << f;
            m[0] |= eq ? (u32)b : 0u;
            m[1] |= eq ? (u32)(b >> 32) : 0u;
            nd += eq ? 1u : 0u;
        }
        live = eq;
    }
    dup = popc32(m[0]) + popc32(m[1]) != nd ? 1u : 0u;
}

// has_duplicate_msd_prefix on [first, last], both in range (equal digit counts).
// TAB: two-word bases with the LDS pair table `tab` (device only).
template <int BASE, bool TAB = false>
__host__ __device__ __forceinline__ bool msd_skippable_fast(u64 f_lo, u64 f_hi, u64 l_lo, u64 l_hi,
                                                            const uint2 *tab = nullptr) {
    using R = Radix<BASE>;
    u32 Xf[R::NX], Xl[R::NX], Sf[R::NS], Sl[R::NS];
    to_limbs<BASE>(f_lo, f_hi, Xf);
    to_limbs<BASE>(l_lo, l_hi, Xl);
    square_limbs<BASE>(Xf, Sf);
    square_limbs<BASE>(Xl, Sl);
    u32 msq[R::MW], dsq;
    if constexpr (TAB) msd_prefix_tab<BASE>(Sf, Sl, R::D2, msq, dsq, tab);
    else msd_prefix<BASE>(Sf, Sl, R::D2, msq, dsq);
    if (dsq) return true;
    u32 Cf[R::NC], Cl[R::NC];
    cube_limbs<BASE>(Sf, Xf, Cf);
    cube_limbs<BASE>(Sl, Xl, Cl);
    u32 mcu[R::MW], dcu;
    if constexpr (TAB) msd_prefix_tab<BASE>(Cf, Cl, R::D3, mcu, dcu, tab);
    else msd_prefix<BASE>(Cf, Cl, R::D3, mcu, dcu);
    if (dcu) return true;
    if (moverlap(msq, mcu)) return true;
    // Filter C (msd_prefix_filter.rs:461-559): first / b^2 == last / b^2, with
    // first's two lowest digits of n^2 and n^3.
    u32 diff = 0;
#pragma unroll
    for (int j = 1; j < R::NX; j++) diff |= Xf[j] ^ Xl[j];
    if (diff == 0) {
        u32 ms[R::MW], mc[R::MW];
#pragma unroll
        for (int w = 0; w < R::MW; w++) ms[w] = mc[w] = 0;
        u32 ds = mset(ms, Sf[0] % BASE);
        ds |= mset(ms, Sf[0] / BASE);
        u32 dc = mset(mc, Cf[0] % BASE);
        dc |= mset(mc, Cf[0] / BASE);
        if (moverlap(msq, ms) || moverlap(mcu, mc) || moverlap(msq, mc) || moverlap(mcu, ms) || ds ||
            dc || moverlap(ms, mc))
            return true;
    }
    return false;
}

}  // namespace nice
