// nice_device.hpp -- gfx950 device code shared by the field-processing kernels.
//
// Everything here is integer VALU work (the path has no HBM stream and no
// contraction), written for 64-lane CDNA4 waves:
//   * compile-time base specialisation (template <int BASE>) so every division
//     by the base or a radix is a multiply-high sequence, AOT-built by hipcc;
//   * digit-presence masks in MW 32-bit registers (MW = ceil(base / 32));
//   * the digit loops follow the reference's semantics exactly: digits are
//     produced least-significant first until the value reaches zero
//     (common/src/client_process.rs:87-98), so no leading zeros are counted.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nice {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

// --------------------------------------------------------------------------
// Digit masks: MW words of 32 bits (base <= 32 -> 1, <= 64 -> 2, <= 128 -> 4).
// --------------------------------------------------------------------------
template <int MW>
struct Mask {
    u32 w[MW];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < MW; i++) w[i] = 0;
    }
    __device__ __forceinline__ void set(u32 d) {
#pragma unroll
        for (int i = 0; i < MW; i++) w[i] |= (d >> 5) == (u32)i ? (1u << (d & 31)) : 0u;
    }
    // Returns non-zero if d was already present; records it either way.
    __device__ __forceinline__ u32 test_set(u32 d) {
        u32 dup = 0;
#pragma unroll
        for (int i = 0; i < MW; i++) {
            u32 bit = (d >> 5) == (u32)i ? (1u << (d & 31)) : 0u;
            dup |= w[i] & bit;
            w[i] |= bit;
        }
        return dup;
    }
    __device__ __forceinline__ u32 popcount() const {
        u32 c = 0;
#pragma unroll
        for (int i = 0; i < MW; i++) c += __popc(w[i]);
        return c;
    }
};

// --------------------------------------------------------------------------
// u128 helpers ({lo, hi} u64 pairs, the reference GPU ABI's split).
// --------------------------------------------------------------------------
__host__ __device__ __forceinline__ void add_u128(u64 &lo, u64 &hi, u64 v) {
    u64 t = lo + v;
    hi += (t < lo) ? 1 : 0;
    lo = t;
}

// r[0..na+nb) = a * b over u32 limbs (schoolbook, u64 accumulation).
template <int NA, int NB>
__device__ __forceinline__ void mul_words(const u32 (&a)[NA], const u32 (&b)[NB],
                                          u32 (&r)[NA + NB]) {
#pragma unroll
    for (int i = 0; i < NA + NB; i++) r[i] = 0;
#pragma unroll
    for (int i = 0; i < NA; i++) {
        u64 carry = 0;
#pragma unroll
        for (int j = 0; j < NB; j++) {
            u64 cur = (u64)a[i] * b[j] + r[i + j] + carry;
            r[i + j] = (u32)cur;
            carry = cur >> 32;
        }
        r[i + NB] = (u32)carry;
    }
}

// Largest E with base^E <= 65535 (chunk divisor D = base^E fits 16 bits, so
// every long-division step is a u32 by u32 division).
struct GenericBase {
    u32 base, D, E;
};
// Compile-time flavour: same members, constexpr, so every division below is
// strength-reduced to multiply-high sequences.
template <int BASE>
struct ConstBase {
    static constexpr u32 base = BASE;
    static constexpr u32 E = []() { u32 e = 0; unsigned long long d = 1; while (d * BASE <= 65535u) { d *= BASE; e++; } return e; }();
    static constexpr u32 D = []() { u32 d = 1; while ((unsigned long long)d * BASE <= 65535u) d *= BASE; return d; }();
};

// Index of the highest non-zero word (-1 for zero), static indexing only (a
// data-dependent index would push the array to scratch memory).
template <int NW>
__device__ __forceinline__ int top_word(const u32 (&v)[NW]) {
    int t = -1;
#pragma unroll
    for (int i = 0; i < NW; i++) t = v[i] ? i : t;
    return t;
}

// In-place v /= D over 16-bit halves of u32 words [0, top]; returns v % D.
// D < 2^16, so the quotient loses at most one top word.
template <int NW>
__device__ __forceinline__ u32 div_chunk(u32 (&v)[NW], int &top, u32 D) {
    u32 rem = 0, vt = 0;
#pragma unroll
    for (int i = NW - 1; i >= 0; i--) {
        if (i > top) continue;
        u32 w = v[i];
        u32 cur = (rem << 16) | (w >> 16);
        u32 qh = cur / D;
        rem = cur - qh * D;
        cur = (rem << 16) | (w & 0xffffu);
        u32 ql = cur / D;
        rem = cur - ql * D;
        v[i] = (qh << 16) | ql;
        if (i == top) vt = v[i];
    }
    top -= (vt == 0) ? 1 : 0;
    return rem;
}

// Scan all digits of v (LSD first, until zero) into m.  STOP: early exit on a
// repeated digit (returns false).
template <int NW, bool STOP, class G>
__device__ __forceinline__ bool scan_generic(u32 (&v)[NW], const G &g, Mask<4> &m) {
    int top = top_word(v);
    while (top >= 0) {
        u32 chunk = div_chunk<NW>(v, top, g.D);
        u32 dup = 0;
        if (top >= 0) {
            for (u32 q = 0; q < g.E; q++) {
                u32 d = chunk % g.base;
                chunk /= g.base;
                dup |= m.test_set(d);
            }
        } else {
            while (chunk) {
                u32 d = chunk % g.base;
                chunk /= g.base;
                dup |= m.test_set(d);
            }
        }
        if (STOP && dup) return false;
    }
    return true;
}

template <class G>
__device__ __forceinline__ u32 unique_generic(u64 lo, u64 hi, const G &g) {
    u32 n[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
    u32 sq[8], cu[12];
    mul_words<4, 4>(n, n, sq);
    u32 sq8[8];
#pragma unroll
    for (int i = 0; i < 8; i++) sq8[i] = sq[i];
    // cu = sq * n (sq < 2^256 -> 8 words; result 12 words)
    mul_words<8, 4>(sq8, n, cu);
    Mask<4> m;
    m.clear();
    scan_generic<8, false>(sq, g, m);
    scan_generic<12, false>(cu, g, m);
    return m.popcount();
}

// Reference get_is_nice semantics (client_process.rs:222-253): scan n^2 then
// n^3, least significant digit first, stop at the first repeated digit.  True
// when no digit repeats (the cube is only multiplied out if n^2 survives).
template <class G>
__device__ __forceinline__ bool is_nice_dev(u64 lo, u64 hi, const G &g) {
    u32 n[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
    u32 sq[8];
    mul_words<4, 4>(n, n, sq);
    u32 sq_scan[8];
#pragma unroll
    for (int i = 0; i < 8; i++) sq_scan[i] = sq[i];
    Mask<4> m;
    m.clear();
    if (!scan_generic<8, true>(sq_scan, g, m)) return false;
    u32 cu[12];
    mul_words<8, 4>(sq, n, cu);
    return scan_generic<12, true>(cu, g, m);
}

static inline GenericBase make_generic(u32 base) {
    GenericBase g;
    g.base = base;
    g.D = 1;
    g.E = 0;
    while ((u64)g.D * base <= 65535u) {
        g.D *= base;
        g.E++;
    }
    return g;
}


// Last-workgroup detection without one hot counter.  Every workgroup, after
// draining its own atomics (vmcnt(0) + barrier by the caller), adds to the
// counter of its group (blockIdx.x % kDoneGroups) in done[1 + group]; the
// workgroup completing a group adds to done[0]; the one completing done[0]
// is last.  A single counter hit by every workgroup serialises in L2 at
// ~40 ns an add: ~500 workgroups ending together (a 1e6 field) cost ~20 us,
// the niceonly kernel's ~2000 mostly idle ones ~80 us.  Every add is an
// agent-scope RMW whose result the next one waits for, so the chain orders
// the hand-off like a single counter (MI355X_MICROARCH.md, inter-workgroup
// visibility).  done[] has kDoneWords words; the last workgroup re-zeroes
// them with done_reset().  Called by thread 0; returns true in the last one.
constexpr uint32_t kDoneGroups = 64, kDoneWords = kDoneGroups + 1;
__device__ __forceinline__ bool last_block_arrive(uint32_t *done) {
    const uint32_t g = blockIdx.x % kDoneGroups, n = gridDim.x;
    // small grids: one counter (saves an L2 round trip on the critical path;
    // one counter for every grid up to 4096 workgroups made b40 1e6 15.8 us
    // against 14.8, the 391 arrivals contending: small_arrive_one_level.log)
    if (n <= kDoneGroups) return atomicAdd(&done[0], 1u) == n - 1;
    const uint32_t expect = g < n ? (n - 1 - g) / kDoneGroups + 1 : 0;
    if (atomicAdd(&done[1 + g], 1u) != expect - 1) return false;
    const uint32_t groups = n < kDoneGroups ? n : kDoneGroups;
    return atomicAdd(&done[0], 1u) == groups - 1;
}
__device__ __forceinline__ void done_reset(uint32_t *done) {
    for (uint32_t w = threadIdx.x; w < kDoneWords; w += blockDim.x)
        __hip_atomic_store(&done[w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace nice
