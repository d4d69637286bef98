// detailed.hip -- gfx950 kernels for detailed field processing.
//
// Replaces the reference's detailed_kernel (common/src/cuda/nice_kernels.cu:
// 486-531) and the CPU loop it mirrors (common/src/client_process.rs:150-191):
// for every n in a segment, count the distinct base-b digits of n^2 and n^3,
// histogram the counts and list the near-misses (count > cutoff).
//
// Two kernels:
//
// detailed_fd_kernel<BASE>  (segments inside the base's valid range)
//   Each thread walks a contiguous run of n and never multiplies: n^2 and n^3
//   are kept directly in radix B = BASE^2 limbs and advanced by finite
//   differences,
//       S = n^2   += D1,  D1 = 2n+1        += 2
//       C = n^3   += E1,  E1 = 3n^2+3n+1   += E2,  E2 = 6n+6 += 6
//   so no digit is ever divided out: every limb IS two base-b digits, and its
//   digit mask comes from one LDS table lookup (B entries).  Limb additions
//   use the 32-bit carry chain (v_add_co/v_addc_co): one operand is stored
//   biased by 2^32 - B so the hardware carry-out is exactly the radix-B carry.
//   Only the low limbs change every step; the high limbs of S and C change on
//   a carry out of the low part (probability ~D1/B^SL per step), so their
//   masks are cached in registers and recomputed on that rare branch.
//   Histograms are per-thread LDS counters ([bin][thread], conflict-free),
//   reduced per workgroup with wave shuffles and flushed with one global
//   atomic per bin per workgroup.
//
// detailed_generic_kernel  (any base 2..128, any n < 2^128)
//   Per-n multiply + chunked radix extraction with a runtime base.  Used for
//   segments outside the valid range (e.g. the reference's b10 @ 1e6 GPU
//   test, client_process_gpu.rs:1485) and for bases without an FD instance.
#include "kernels.h"
#include "nice_device.hpp"

namespace nice {

// ---------------------------------------------------------------------------
// Compile-time layout of the finite-difference state for a base.
// Digit counts inside the valid range (base_range.rs:14-32): with k = b / 5,
//   b%5==0: n^2 2k digits, n^3 3k, n <= k digits
//   b%5==2: 2k+1, 3k+1, n <= k+1      b%5==3: 2k+1, 3k+2      b%5==4: 2k+2, 3k+2
// ---------------------------------------------------------------------------
constexpr int log2ceil(unsigned v) { int t = 0; while ((1u << t) < v) t++; return t; }

template <int BASE_>
struct FdTraits {
    static constexpr int BASE = BASE_;
    static constexpr int k = BASE / 5, r5 = BASE % 5;
    static constexpr int D2 = r5 == 0 ? 2 * k : (r5 == 4 ? 2 * k + 2 : 2 * k + 1);
    static constexpr int D3 = r5 == 0 ? 3 * k : (r5 == 2 ? 3 * k + 1 : 3 * k + 2);
    static constexpr int DN = r5 == 0 ? k : k + 1;
    static constexpr int K = 2;  // digits per limb
    static constexpr u32 B = (u32)BASE * BASE;
    static constexpr int T = log2ceil(B);          // carry bit of a biased limb sum
    static constexpr u32 BT = (1u << T) - B;       // limb bias: x + BT >= 2^T  <=>  x >= B
    static constexpr int NS = cdiv(D2, K), NC = cdiv(D3, K), NX = cdiv(DN, K);
    static constexpr int ND = cdiv(DN + 1, K);   // limbs of D1 = 2n+1
    static constexpr int NE = cdiv(D2 + 1, K);   // limbs of E1 = 3n^2+3n+1
    static constexpr int NE2 = cdiv(DN + 1, K);  // limbs of E2 = 6n+6
    static constexpr int SL = ND, CL = NE + 1, EL = NE2 + 1;  // per-step (low) limbs
    static constexpr int SH = NS - SL, CH = NC - CL, EH = NE - EL;
    static constexpr int S_TOPD = D2 - K * (NS - 1), C_TOPD = D3 - K * (NC - 1);
    static constexpr int MW = (BASE + 31) / 32;
    static constexpr int ES = MW == 1 ? 4 : (MW == 2 ? 8 : 16);  // LDS bytes per table entry
    static constexpr bool PER_THREAD_HIST = BASE <= 64;
    static constexpr int WG = PER_THREAD_HIST ? 256 : 1024;
    static constexpr int NBINS = BASE + 1;
    static constexpr int HIST_BYTES = PER_THREAD_HIST ? NBINS * WG * 4 : (WG / 64) * NBINS * 4;
    // Table after the histogram, at an offset >= BT*ES so a biased limb's
    // address (limb*ES + TB - BT*ES) keeps a non-negative constant offset.
    static constexpr int TB0 = HIST_BYTES > (int)BT * ES ? HIST_BYTES : (int)BT * ES;
    static constexpr int TB = (TB0 + 15) / 16 * 16;
    static constexpr int LDS_BYTES = TB + (int)B * ES;
    static_assert(SH >= 1 && CH >= 1 && EH >= 0, "FD layout needs cached high limbs");
    static_assert(S_TOPD >= 1 && S_TOPD <= K && C_TOPD >= 1 && C_TOPD <= K, "top limb");
    static_assert(BASE <= 96, "mask layout");
    static_assert(2 * B <= (1u << (T + 1)), "carry bit");
};

// OR the table mask of one limb into m.  BIAS: the limb's storage bias.
template <class P, u32 BIAS>
__device__ __forceinline__ void lds_mask(const unsigned char *smem, u32 limb, Mask<P::MW> &m) {
    const unsigned char *p = smem + (P::TB - (int)BIAS * P::ES) + limb * P::ES;
    if constexpr (P::MW == 1) {
        m.w[0] |= *(const u32 *)p;
    } else if constexpr (P::MW == 2) {
        uint2 v = *(const uint2 *)p;
        m.w[0] |= v.x;
        m.w[1] |= v.y;
    } else {
        uint4 v = *(const uint4 *)p;
        m.w[0] |= v.x;
        m.w[1] |= v.y;
        m.w[2] |= v.z;
    }
}

// Mask of the top limb holding `d` significant digits (d == 1: a single digit).
template <class P>
__device__ __forceinline__ void top_mask(const unsigned char *smem, u32 limb, int d,
                                         Mask<P::MW> &m) {
    if (d == P::K) lds_mask<P, 0>(smem, limb, m);
    else m.set(limb);
}

// State of one thread's walk.  Low limbs of S and C are stored biased by BT
// (the per-step carry chains); everything else is plain radix-B.
template <class P>
struct FdState {
    u32 S[P::NS];   // n^2
    u32 C[P::NC];   // n^3
    u32 D1[P::ND];  // 2n+1
    u32 E1[P::NE];  // 3n^2+3n+1
    u32 E2[P::NE2]; // 6n+6
    Mask<P::MW> hiS, hiC;  // cached masks of the high limbs
};

// Radix-B conversion of an arbitrary-width accumulator (u64 columns).
template <class P, int N, int M>
__device__ __forceinline__ void normalize(const u64 (&acc)[N], u32 (&out)[M]) {
    u64 cy = 0;
#pragma unroll
    for (int t = 0; t < M; t++) {
        u64 v = (t < N ? acc[t] : 0) + cy;
        out[t] = (u32)(v % P::B);
        cy = v / P::B;
    }
}

template <class P>
__device__ __forceinline__ void recompute_high(FdState<P> &st, const unsigned char *smem) {
    st.hiS.clear();
#pragma unroll
    for (int i = P::SL; i < P::NS - 1; i++) lds_mask<P, 0>(smem, st.S[i], st.hiS);
    top_mask<P>(smem, st.S[P::NS - 1], P::S_TOPD, st.hiS);
    st.hiC.clear();
#pragma unroll
    for (int i = P::CL; i < P::NC - 1; i++) lds_mask<P, 0>(smem, st.C[i], st.hiC);
    top_mask<P>(smem, st.C[P::NC - 1], P::C_TOPD, st.hiC);
}

template <class P>
__device__ __forceinline__ void fd_init(FdState<P> &st, u64 n_lo, u64 n_hi,
                                        const unsigned char *smem) {
    constexpr u32 B = P::B;
    // n in radix B
    u32 w[4] = {(u32)n_lo, (u32)(n_lo >> 32), (u32)n_hi, (u32)(n_hi >> 32)};
    u32 X[P::NX];
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
    {  // S = X^2
        u64 acc[2 * P::NX];
#pragma unroll
        for (int t = 0; t < 2 * P::NX; t++) acc[t] = 0;
#pragma unroll
        for (int i = 0; i < P::NX; i++)
#pragma unroll
            for (int j = 0; j < P::NX; j++) acc[i + j] += (u64)X[i] * X[j];
        normalize<P>(acc, st.S);
    }
    {  // C = S * X
        u64 acc[P::NS + P::NX];
#pragma unroll
        for (int t = 0; t < P::NS + P::NX; t++) acc[t] = 0;
#pragma unroll
        for (int i = 0; i < P::NS; i++)
#pragma unroll
            for (int j = 0; j < P::NX; j++) acc[i + j] += (u64)st.S[i] * X[j];
        normalize<P>(acc, st.C);
    }
    {
        u64 acc[P::ND];
#pragma unroll
        for (int t = 0; t < P::ND; t++) acc[t] = (t < P::NX ? 2ull * X[t] : 0) + (t == 0);
        normalize<P>(acc, st.D1);
    }
    {
        u64 acc[P::NE];
#pragma unroll
        for (int t = 0; t < P::NE; t++)
            acc[t] = (t < P::NS ? 3ull * st.S[t] : 0) + (t < P::NX ? 3ull * X[t] : 0) + (t == 0);
        normalize<P>(acc, st.E1);
    }
    {
        u64 acc[P::NE2];
#pragma unroll
        for (int t = 0; t < P::NE2; t++) acc[t] = (t < P::NX ? 6ull * X[t] : 0) + 6 * (t == 0);
        normalize<P>(acc, st.E2);
    }
    recompute_high<P>(st, smem);
#pragma unroll
    for (int i = 0; i < P::SL; i++) st.S[i] += P::BT;
#pragma unroll
    for (int i = 0; i < P::CL; i++) st.C[i] += P::BT;
}

// Propagate a +1 carry into limbs [from, N) (branch-free and fully unrolled so
// the limbs stay in registers).
template <int N>
__device__ __forceinline__ void carry_into(u32 (&x)[N], int from, u32 B) {
    u32 c = 1;
#pragma unroll
    for (int i = 0; i < N; i++) {
        if (i < from) continue;
        u32 v = x[i] + c;
        u32 wrap = v == B;
        x[i] = wrap ? 0u : v;
        c = wrap;
    }
}

// Biased accumulate: acc (bias BT) += add (plain) + c.  Carry = bit T.
template <class P>
__device__ __forceinline__ u32 acc_biased(u32 &acc, u32 add, u32 c) {
    u32 t = acc + add + c;               // v_add3_u32
    u32 co = t >> P::T;                  // v_lshrrev_b32
    acc = t - co * P::B;                 // v_mad_i32_i24
    return co;
}
// Plain accumulate: acc += add + c, both plain radix-B.
template <class P>
__device__ __forceinline__ u32 acc_plain(u32 &acc, u32 add, u32 c) {
    u32 t = acc + add + c;
    u32 co = (t + P::BT) >> P::T;
    acc = t - co * P::B;
    return co;
}

// One step n -> n+1.  Carries leaving a low part are rare; they are folded
// into the high limbs (and the cached masks refreshed) on a divergent branch.
template <class P>
__device__ __forceinline__ void fd_step(FdState<P> &st, const unsigned char *smem) {
    u32 cS = 0, cC = 0, cE = 0, cD, cE2;
#pragma unroll
    for (int i = 0; i < P::SL; i++) cS = acc_biased<P>(st.S[i], i < P::ND ? st.D1[i] : 0u, cS);
#pragma unroll
    for (int i = 0; i < P::CL; i++) cC = acc_biased<P>(st.C[i], i < P::NE ? st.E1[i] : 0u, cC);
#pragma unroll
    for (int i = 0; i < P::EL; i++) cE = acc_plain<P>(st.E1[i], i < P::NE2 ? st.E2[i] : 0u, cE);
    cD = acc_plain<P>(st.D1[0], 2u, 0u);
    cD = acc_plain<P>(st.D1[1], 0u, cD);
    cE2 = acc_plain<P>(st.E2[0], 6u, 0u);
    cE2 = acc_plain<P>(st.E2[1], 0u, cE2);
    if (cS | cC | cE | cD | cE2) {
        if (cD) carry_into(st.D1, 2, P::B);
        if (cE2) carry_into(st.E2, 2, P::B);
        if (cE) carry_into(st.E1, P::EL, P::B);
        if (cS) carry_into(st.S, P::SL, P::B);
        if (cC) carry_into(st.C, P::CL, P::B);
        if (cS | cC) recompute_high<P>(st, smem);
    }
}

template <int BASE>
__global__ void __launch_bounds__(FdTraits<BASE>::WG, FdTraits<BASE>::WG == 256 ? 2 : 4)
detailed_fd_kernel(u64 start_lo, u64 start_hi, u64 count, u64 chunk, u32 cutoff,
                   u64 *__restrict__ hist_out, NumOut out) {
    using P = FdTraits<BASE>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u32 *hist = (u32 *)smem;
    const u32 tid = threadIdx.x;

    // Digit-pair mask table: entry e = d1*BASE + d0 marks digits d0 and d1.
    for (u32 e = tid; e < P::B; e += P::WG) {
        u32 d0 = e % BASE, d1 = e / BASE;
        u32 v[4] = {0, 0, 0, 0};
        v[d0 >> 5] |= 1u << (d0 & 31);
        v[d1 >> 5] |= 1u << (d1 & 31);
        unsigned char *p = smem + P::TB + e * P::ES;
        if constexpr (P::ES == 4) *(u32 *)p = v[0];
        else if constexpr (P::ES == 8) *(uint2 *)p = make_uint2(v[0], v[1]);
        else *(uint4 *)p = make_uint4(v[0], v[1], v[2], v[3]);
    }
    for (u32 i = tid; i < (u32)P::HIST_BYTES / 4; i += P::WG) hist[i] = 0;
    __syncthreads();

    const u32 slot = P::PER_THREAD_HIST ? tid : (tid >> 6) * P::NBINS;
    const u32 stride = P::PER_THREAD_HIST ? P::WG : 1;
    const u64 nchunks = (count + chunk - 1) / chunk;
    for (u64 c = (u64)blockIdx.x * P::WG + tid; c < nchunks; c += (u64)gridDim.x * P::WG) {
        const u64 off = c * chunk;
        const u32 len = (u32)((count - off) < chunk ? (count - off) : chunk);
        u64 n0_lo = start_lo, n0_hi = start_hi;
        add_u128(n0_lo, n0_hi, off);
        FdState<P> st;
        fd_init<P>(st, n0_lo, n0_hi, smem);
        for (u32 i = 0;;) {
            // Issue this n's lookups, then advance the state while they land.
            Mask<P::MW> m;
#pragma unroll
            for (int q = 0; q < P::MW; q++) m.w[q] = st.hiS.w[q] | st.hiC.w[q];
#pragma unroll
            for (int q = 0; q < P::SL; q++) lds_mask<P, P::BT>(smem, st.S[q], m);
#pragma unroll
            for (int q = 0; q < P::CL; q++) lds_mask<P, P::BT>(smem, st.C[q], m);
            const bool more = ++i < len;
            if (more) fd_step<P>(st, smem);
            const u32 u = m.popcount();
            atomicAdd(&hist[u * stride + slot], 1u);  // ds_add_u32; per-thread slots
            if (u > cutoff) {
                u64 lo = n0_lo, hi = n0_hi;
                add_u128(lo, hi, i - 1);
                u32 pos = atomicAdd(out.count, 1u);
                if (pos < out.cap) {
                    out.n[2 * (u64)pos] = lo;
                    out.n[2 * (u64)pos + 1] = hi;
                    out.u[pos] = u;
                }
            }
            if (!more) break;
        }
    }
    __syncthreads();
    // Flush: one global atomic per (workgroup, non-empty bin).
    const u32 wave = tid >> 6, lane = tid & 63;
    for (u32 bin = wave; bin < (u32)P::NBINS; bin += P::WG / 64) {
        u32 s = 0;
        if constexpr (P::PER_THREAD_HIST) {
#pragma unroll
            for (int q = 0; q < P::WG / 64; q++) s += hist[bin * P::WG + lane + 64 * q];
        } else {
            if (lane < P::WG / 64) s = hist[lane * P::NBINS + bin];
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0 && s) atomicAdd((unsigned long long *)&hist_out[bin], (unsigned long long)s);
    }
}

// ---------------------------------------------------------------------------
// Generic per-n kernel (runtime base).
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256)
detailed_generic_kernel(u64 start_lo, u64 start_hi, u64 count, GenericBase g, u32 cutoff,
                        u64 *__restrict__ hist_out, NumOut out) {
    __shared__ u32 hist[4][129];
    const u32 tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (u32 i = tid; i < 4 * 129; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    for (u64 idx = (u64)blockIdx.x * 256 + tid; idx < count; idx += (u64)gridDim.x * 256) {
        u64 lo = start_lo, hi = start_hi;
        add_u128(lo, hi, idx);
        u32 u = unique_generic(lo, hi, g);
        atomicAdd(&hist[wave][u], 1u);
        if (u > cutoff) {
            u32 pos = atomicAdd(out.count, 1u);
            if (pos < out.cap) {
                out.n[2 * (u64)pos] = lo;
                out.n[2 * (u64)pos + 1] = hi;
                out.u[pos] = u;
            }
        }
    }
    __syncthreads();
    for (u32 b = tid; b <= g.base; b += 256) {
        u32 s = hist[0][b] + hist[1][b] + hist[2][b] + hist[3][b];
        if (s) atomicAdd((unsigned long long *)&hist_out[b], (unsigned long long)s);
    }
    (void)lane;
}

// Diagnostics: per-n unique counts / nice flags through the device functions.
__global__ void unique_counts_kernel(const u64 *n_pairs, u32 count, GenericBase g, u32 *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = unique_generic(n_pairs[2 * i], n_pairs[2 * i + 1], g);
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
template <int BASE>
static hipError_t launch_fd(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    using P = FdTraits<BASE>;
    static bool configured = false;
    if (!configured) {
        hipError_t e = hipFuncSetAttribute((const void *)detailed_fd_kernel<BASE>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           P::LDS_BYTES);
        if (e != hipSuccess) return e;
        configured = true;
    }
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, (const void *)detailed_fd_kernel<BASE>, P::WG, P::LDS_BYTES);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const u64 resident_threads = (u64)num_cus * per_cu * P::WG;
    // Aim for ~4 chunks per resident thread (balances tails against init cost).
    u64 chunk = (p.count + 4 * resident_threads - 1) / (4 * resident_threads);
    if (chunk < 64) chunk = 64;
    if (chunk > (1u << 20)) chunk = 1u << 20;
    const u64 nchunks = (p.count + chunk - 1) / chunk;
    u64 grid = (nchunks + P::WG - 1) / P::WG;
    const u64 max_grid = (u64)num_cus * per_cu;
    if (grid > max_grid) grid = max_grid;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(detailed_fd_kernel<BASE>, dim3((u32)grid), dim3(P::WG), P::LDS_BYTES, s,
                       p.start_lo, p.start_hi, p.count, chunk, p.cutoff, p.hist, p.out);
    return hipGetLastError();
}

#define NICE_FD_BASES(X) X(40) X(50) X(80)

bool fd_supported(uint32_t base) {
    switch (base) {
#define X(b) case b: return true;
        NICE_FD_BASES(X)
#undef X
    default: return false;
    }
}

hipError_t launch_detailed_fd(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    switch (p.base) {
#define X(b) case b: return launch_fd<b>(p, num_cus, s);
        NICE_FD_BASES(X)
#undef X
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_detailed_generic(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    GenericBase g = make_generic(p.base);
    u64 grid = (p.count + 255) / 256;
    u64 cap = (u64)num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(detailed_generic_kernel, dim3((u32)grid), dim3(256), 0, s, p.start_lo,
                       p.start_hi, p.count, g, p.cutoff, p.hist, p.out);
    return hipGetLastError();
}

hipError_t launch_unique_counts(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                                uint32_t *out, hipStream_t s) {
    GenericBase g = make_generic(base);
    hipLaunchKernelGGL(unique_counts_kernel, dim3((count + 255) / 256), dim3(256), 0, s, n_pairs,
                       count, g, out);
    return hipGetLastError();
}

}  // namespace nice
