// fd_detailed.hip -- finite-difference detailed kernel for in-range segments.
//
// Replaces the reference's detailed_kernel (common/src/cuda/nice_kernels.cu:
// 486-531) for fields inside a base's valid range, computing exactly what
// process_range_detailed does (common/src/client_process.rs:150-191).
//
// Each lane walks an arithmetic progression n, n+H, n+2H, ... and never
// multiplies: n^2 and n^3 live in radix B = BASE^2 limbs and advance by
// finite differences with step H,
//     S = n^2   += D1,  D1 = 2Hn + H^2               += 2H^2
//     C = n^3   += E1,  E1 = 3Hn^2 + 3H^2 n + H^3     += E2
//                       E2 = 6H^2 n + 6H^3            += 6H^3
// so no digit is divided out: each limb IS two base-b digits, and its digit
// mask comes from one LDS table lookup (B entries) -- or, for a tunable number
// of limbs, from two multiply-high digit peels, to balance LDS against VALU.
//
// Carry handling.  Low limbs of S and C are stored biased by BT = 2^T - B, so
// acc + addend + carry >= 2^T exactly when the radix-B sum overflows: the
// carry is bit T (v_add3 + v_lshrrev + v_mad_i24, pure VGPR data flow).  Only
// the low limbs change every step; a carry out of a low part (probability
// ~addend / B^L) is handled on a divergent branch that also refreshes the
// cached masks of the high limbs.
//
// Lane mapping.  H = 1: each lane owns a contiguous chunk.  H = 64: the 64
// lanes of a wave own consecutive n (lane l: n0 + l + 64 i), so the
// slow-moving upper limbs of the low part, and the n mod B index of the
// low-digit table, are consecutive or equal across the wave (bank-conflict
// free / broadcast LDS reads), which random per-lane chunks never are.
//
// LSD table.  n^2 mod B and n^3 mod B depend only on n mod B, so the masks of
// limb 0 of S and of C come from one lookup T_lsd[n mod B].
#include "kernels.h"
#include "nice_device.hpp"

namespace nice {

constexpr int log2ceil(unsigned v) { int t = 0; while ((1u << t) < v) t++; return t; }
constexpr int ndigits(unsigned long long v, unsigned b) { int d = 0; while (v) { v /= b; d++; } return d; }
constexpr unsigned long long ipow(unsigned long long b, int e) { unsigned long long r = 1; while (e-- > 0) r *= b; return r; }

// Variant knobs (benchmarked): lane stride H, low-digit table,
// number of arithmetic (non-LDS) limbs in the low parts of S and C.
template <int H_, bool LSD_, int AS_, int AC_, bool H16_ = false>
struct FdVariant {
    static constexpr int H = H_;
    static constexpr bool LSD = LSD_;
    static constexpr int AS = AS_, AC = AC_;
    static constexpr bool H16 = H16_;  // 16-bit per-thread histogram counters
};

template <int BASE_, class V>
struct FdTraits {
    static constexpr int BASE = BASE_;
    static constexpr int H = V::H;
    static constexpr int k = BASE / 5, r5 = BASE % 5;
    // Digit counts inside the valid range (base_range.rs:14-32).
    static constexpr int D2 = r5 == 0 ? 2 * k : (r5 == 4 ? 2 * k + 2 : 2 * k + 1);
    static constexpr int D3 = r5 == 0 ? 3 * k : (r5 == 2 ? 3 * k + 1 : 3 * k + 2);
    static constexpr int DN = r5 == 0 ? k : k + 1;
    static constexpr int K = 2;
    static constexpr u32 B = (u32)BASE * BASE;
    static constexpr int T = log2ceil(B);
    static constexpr u32 BT = (1u << T) - B;
    static constexpr int NS = cdiv(D2, K), NC = cdiv(D3, K), NX = cdiv(DN, K);
    // Upper bounds of the difference terms (n < b^DN):
    //   D1 < (2H+1) b^DN, E1 < (3H+1) b^(2DN), E2 < (6H^2+1) b^DN
    static constexpr int ND = cdiv(DN + ndigits(2ull * H + 1, BASE), K);
    static constexpr int NE = cdiv(2 * DN + ndigits(3ull * H + 1, BASE), K);
    static constexpr int NE2 = cdiv(DN + ndigits(6ull * H * H + 1, BASE), K);
    static constexpr int SL = ND + 1, CL = NE + 1, EL = NE2 + 1;  // per-step (low) limbs
    static constexpr int SH = NS - SL, CH = NC - CL, EH = NE - EL;
    static constexpr int S_TOPD = D2 - K * (NS - 1), C_TOPD = D3 - K * (NC - 1);
    // Constant increments of D1 and E2 in radix B.
    static constexpr unsigned long long DD1 = 2ull * H * H, DE2 = 6ull * H * H * H;
    static constexpr int NDD1 = cdiv(ndigits(DD1, BASE), K), NDE2 = cdiv(ndigits(DE2, BASE), K);
    static constexpr int MW = (BASE + 31) / 32;
    static constexpr int ES = MW == 1 ? 4 : (MW == 2 ? 8 : 16);
    static constexpr bool PER_THREAD_HIST = BASE <= 64;
    static constexpr int WG = PER_THREAD_HIST ? 256 : 512;
    static constexpr int NBINS = BASE + 1;
    // Per-thread counters are u32, or u16 pairs packed in a u32 (HIST16: half the
    // LDS, so twice the resident waves; the host caps a launch at 65535 numbers
    // per lane so a counter cannot wrap).
    static constexpr bool HIST16 = PER_THREAD_HIST && V::H16;
    static constexpr int HROWS = HIST16 ? (NBINS + 1) / 2 : NBINS;
    static constexpr int HIST_BYTES = PER_THREAD_HIST ? HROWS * WG * 4 : (WG / 64) * NBINS * 4;
    static constexpr int TB0 = HIST_BYTES > (int)BT * ES ? HIST_BYTES : (int)BT * ES;
    static constexpr int TB = (TB0 + 15) / 16 * 16;           // digit-pair table
    static constexpr int TL = TB + (int)B * ES;               // low-digit (n mod B) table
    // The low-digit table is dropped where it would not fit in LDS (b80).
    static constexpr bool LSD = V::LSD && TL + (int)B * ES <= 160 * 1024;
    static constexpr int LDS_BYTES = TL + (LSD ? (int)B * ES : 0);
    static constexpr int LO = LSD ? 1 : 0;                    // first low limb looked up
    static constexpr bool ARITH_OK = MW <= 2;
    static_assert(SH >= 1 && CH >= 1 && EH >= 0, "FD layout needs cached high limbs");
    static_assert(S_TOPD >= 1 && S_TOPD <= K && C_TOPD >= 1 && C_TOPD <= K, "top limb");
    static_assert(BASE <= 96, "mask layout");
    static_assert(H < (int)B && NDD1 <= 2 && NDE2 <= 3, "increments");
    static_assert(V::AS + LO <= SL && V::AC + LO <= CL, "arith limbs");
    static_assert(ARITH_OK || (V::AS == 0 && V::AC == 0), "arith needs <= 64-bit masks");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

template <class P, u32 BIAS>
__device__ __forceinline__ void tab_or(const unsigned char *smem, int tbase, u32 limb,
                                       Mask<P::MW> &m) {
    const unsigned char *p = smem + (tbase - (int)BIAS * P::ES) + limb * P::ES;
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

// Two digits of a biased limb by multiply-high peeling (no LDS).
template <class P>
__device__ __forceinline__ void arith_or(u32 limb_biased, Mask<P::MW> &m) {
    // floor(x / BASE) = (x * MAGIC) >> 16 for x < B (error term checked below)
    constexpr u32 MAGIC = (u32)((1ull << 16) / P::BASE + 1);
    static_assert(!P::ARITH_OK ||
                      (unsigned long long)MAGIC * P::BASE - (1ull << 16) < (1ull << 16) / P::B,
                  "peel magic not exact over [0, B)");
    if constexpr (!P::ARITH_OK) return;
    const u32 x = limb_biased - P::BT;
    const u32 d1 = (x * MAGIC) >> 16;
    const u32 d0 = x - d1 * P::BASE;
    if constexpr (P::MW == 1) {
        m.w[0] |= (1u << d0) | (1u << d1);
    } else if constexpr (P::MW == 2) {
        unsigned long long b = (1ull << d0) | (1ull << d1);
        m.w[0] |= (u32)b;
        m.w[1] |= (u32)(b >> 32);
    }
}

template <class P>
__device__ __forceinline__ void top_or(const unsigned char *smem, u32 limb, int d, Mask<P::MW> &m) {
    if (d == P::K) tab_or<P, 0>(smem, P::TB, limb, m);
    else m.set(limb);
}

template <class P>
struct FdState {
    u32 S[P::NS];   // n^2 (low SL limbs biased by BT)
    u32 C[P::NC];   // n^3 (low CL limbs biased)
    u32 D1[P::ND];
    u32 E1[P::NE];
    u32 E2[P::NE2];
    u32 r;          // n mod B (low-digit table index)
    Mask<P::MW> hiS, hiC;
};

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
    for (int i = P::SL; i < P::NS - 1; i++) tab_or<P, 0>(smem, P::TB, st.S[i], st.hiS);
    top_or<P>(smem, st.S[P::NS - 1], P::S_TOPD, st.hiS);
    st.hiC.clear();
#pragma unroll
    for (int i = P::CL; i < P::NC - 1; i++) tab_or<P, 0>(smem, P::TB, st.C[i], st.hiC);
    top_or<P>(smem, st.C[P::NC - 1], P::C_TOPD, st.hiC);
}

template <class P>
__device__ __forceinline__ void fd_init(FdState<P> &st, u64 n_lo, u64 n_hi,
                                        const unsigned char *smem) {
    constexpr u32 B = P::B;
    constexpr u64 H = P::H;
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
    st.r = X[0];
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
    {  // D1 = 2H n + H^2
        u64 acc[P::ND];
#pragma unroll
        for (int t = 0; t < P::ND; t++) acc[t] = (t < P::NX ? 2 * H * X[t] : 0) + (t == 0 ? H * H : 0);
        normalize<P>(acc, st.D1);
    }
    {  // E1 = 3H n^2 + 3H^2 n + H^3
        u64 acc[P::NE];
#pragma unroll
        for (int t = 0; t < P::NE; t++)
            acc[t] = (t < P::NS ? 3 * H * st.S[t] : 0) + (t < P::NX ? 3 * H * H * X[t] : 0) +
                     (t == 0 ? H * H * H : 0);
        normalize<P>(acc, st.E1);
    }
    {  // E2 = 6H^2 n + 6H^3
        u64 acc[P::NE2];
#pragma unroll
        for (int t = 0; t < P::NE2; t++)
            acc[t] = (t < P::NX ? 6 * H * H * X[t] : 0) + (t == 0 ? 6 * H * H * H : 0);
        normalize<P>(acc, st.E2);
    }
    recompute_high<P>(st, smem);
#pragma unroll
    for (int i = 0; i < P::SL; i++) st.S[i] += P::BT;
#pragma unroll
    for (int i = 0; i < P::CL; i++) st.C[i] += P::BT;
}

// +1 carry into limbs [from, N) (branch-free, unrolled: limbs stay in VGPRs).
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

template <class P>
__device__ __forceinline__ u32 acc_biased(u32 &acc, u32 add, u32 c) {
    u32 t = acc + add + c;   // v_add3_u32
    u32 co = t >> P::T;      // v_lshrrev_b32
    acc = t - co * P::B;     // v_mad_i32_i24
    return co;
}
template <class P>
__device__ __forceinline__ u32 acc_plain(u32 &acc, u32 add, u32 c) {
    u32 t = acc + add + c;
    u32 co = (t + P::BT) >> P::T;
    acc = t - co * P::B;
    return co;
}
// X += constant V (radix-B digits, NV limbs) with carry into limb NV; returns
// the carry out of limb NV (rare).
template <class P, unsigned long long V, int NV, int N>
__device__ __forceinline__ u32 add_const(u32 (&x)[N]) {
    u32 c = 0;
#pragma unroll
    for (int i = 0; i < NV; i++) c = acc_plain<P>(x[i], (u32)((V / ipow(P::B, i)) % P::B), c);
    if constexpr (NV < N) c = acc_plain<P>(x[NV], 0u, c);
    return c;
}

template <class P>
__device__ __forceinline__ void fd_step(FdState<P> &st, const unsigned char *smem) {
    u32 cS = 0, cC = 0, cE = 0;
#pragma unroll
    for (int i = 0; i < P::SL; i++) cS = acc_biased<P>(st.S[i], i < P::ND ? st.D1[i] : 0u, cS);
#pragma unroll
    for (int i = 0; i < P::CL; i++) cC = acc_biased<P>(st.C[i], i < P::NE ? st.E1[i] : 0u, cC);
#pragma unroll
    for (int i = 0; i < P::EL; i++) cE = acc_plain<P>(st.E1[i], i < P::NE2 ? st.E2[i] : 0u, cE);
    const u32 cD = add_const<P, P::DD1, P::NDD1>(st.D1);
    const u32 cE2 = add_const<P, P::DE2, P::NDE2>(st.E2);
    if constexpr (P::H > 0) {
        u32 r = st.r + P::H;
        st.r = r >= P::B ? r - P::B : r;
    }
    if (cS | cC | cE | cD | cE2) {
        if (cD) carry_into(st.D1, P::NDD1 + 1, P::B);
        if (cE2) carry_into(st.E2, P::NDE2 + 1, P::B);
        if (cE) carry_into(st.E1, P::EL, P::B);
        if (cS) carry_into(st.S, P::SL, P::B);
        if (cC) carry_into(st.C, P::CL, P::B);
        if (cS | cC) recompute_high<P>(st, smem);
    }
}

template <int BASE, class V>
__global__ void __launch_bounds__((FdTraits<BASE, V>::WG), (FdTraits<BASE, V>::HIST16 ? 4 : 2))
detailed_fd_kernel(u64 start_lo, u64 start_hi, u64 count, u64 chunk, u32 cutoff,
                   u64 *__restrict__ hist_out, NumOut out) {
    using P = FdTraits<BASE, V>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u32 *hist = (u32 *)smem;
    const u32 tid = threadIdx.x;

    // Digit-pair table: entry e = d1*BASE + d0 marks digits d0 and d1.
    // Low-digit table: entry r marks the two low digits of r^2 and of r^3.
    for (u32 e = tid; e < P::B; e += P::WG) {
        u32 v[4] = {0, 0, 0, 0};
        auto mark = [&](u32 x) {
            u32 d0 = x % BASE, d1 = x / BASE;
            v[d0 >> 5] |= 1u << (d0 & 31);
            v[d1 >> 5] |= 1u << (d1 & 31);
        };
        auto put = [&](int base_off) {
            unsigned char *p = smem + base_off + e * P::ES;
            if constexpr (P::ES == 4) *(u32 *)p = v[0];
            else if constexpr (P::ES == 8) *(uint2 *)p = make_uint2(v[0], v[1]);
            else *(uint4 *)p = make_uint4(v[0], v[1], v[2], v[3]);
        };
        mark(e);
        put(P::TB);
        if constexpr (P::LSD) {
            v[0] = v[1] = v[2] = v[3] = 0;
            const u64 sq = (u64)e * e % P::B;
            mark((u32)sq);
            mark((u32)(sq * e % P::B));
            put(P::TL);
        }
    }
    for (u32 i = tid; i < (u32)P::HIST_BYTES / 4; i += P::WG) hist[i] = 0;
    __syncthreads();

    const u32 slot = P::PER_THREAD_HIST ? tid : (tid >> 6) * P::NBINS;
    const u32 hstride = P::PER_THREAD_HIST ? P::WG : 1;
    // Work units: H == 1 -> one chunk per lane; H == 64 -> one block of
    // 64*chunk consecutive n per wave.
    const u64 unit = P::H == 1 ? chunk : 64 * chunk;
    const u64 nunits = (count + unit - 1) / unit;
    const u64 first = P::H == 1 ? (u64)blockIdx.x * P::WG + tid : ((u64)blockIdx.x * P::WG + tid) >> 6;
    const u64 ustride = P::H == 1 ? (u64)gridDim.x * P::WG : ((u64)gridDim.x * P::WG) >> 6;
    const u32 lane = tid & 63;
    for (u64 c = first; c < nunits; c += ustride) {
        u64 off = c * unit + (P::H == 1 ? 0 : lane);
        u32 len;
        if (off >= count) len = 0;
        else len = (u32)min((u64)chunk, (count - off + P::H - 1) / P::H);
        if (P::H == 1 && len == 0) continue;
        u64 n0_lo = start_lo, n0_hi = start_hi;
        add_u128(n0_lo, n0_hi, off < count ? off : 0);
        FdState<P> st;
        fd_init<P>(st, n0_lo, n0_hi, smem);
        for (u32 i = 0; i < (u32)chunk; i++) {
            if (P::H != 1 && i >= len) break;  // partial last block
            Mask<P::MW> m;
#pragma unroll
            for (int q = 0; q < P::MW; q++) m.w[q] = st.hiS.w[q] | st.hiC.w[q];
            if constexpr (P::LSD) tab_or<P, 0>(smem, P::TL, st.r, m);
#pragma unroll
            for (int q = P::LO; q < P::SL; q++) {
                if (q < P::LO + V::AS) arith_or<P>(st.S[q], m);
                else tab_or<P, P::BT>(smem, P::TB, st.S[q], m);
            }
#pragma unroll
            for (int q = P::LO; q < P::CL; q++) {
                if (q < P::LO + V::AC) arith_or<P>(st.C[q], m);
                else tab_or<P, P::BT>(smem, P::TB, st.C[q], m);
            }
            const bool more = i + 1 < len;
            if (more) fd_step<P>(st, smem);
            const u32 u = m.popcount();
            if constexpr (P::HIST16) atomicAdd(&hist[(u >> 1) * hstride + slot], 1u << ((u & 1) << 4));
            else atomicAdd(&hist[u * hstride + slot], 1u);
            if (u > cutoff) {
                u64 lo = n0_lo, hi = n0_hi;
                add_u128(lo, hi, (u64)i * P::H);
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
    const u32 wave = tid >> 6;
    hist_out += (blockIdx.x % kHistCopies) * 129;
    for (u32 bin = wave; bin < (u32)P::NBINS; bin += P::WG / 64) {
        u32 s = 0;
        if constexpr (P::HIST16) {
#pragma unroll
            for (int q = 0; q < P::WG / 64; q++)
                s += (hist[(bin >> 1) * P::WG + lane + 64 * q] >> ((bin & 1) << 4)) & 0xffffu;
        } else if constexpr (P::PER_THREAD_HIST) {
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

template <int BASE, class V>
static hipError_t launch_fd_variant(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    using P = FdTraits<BASE, V>;
    auto kern = detailed_fd_kernel<BASE, V>;
    static bool configured = false;
    if (!configured) {
        hipError_t e = hipFuncSetAttribute((const void *)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, P::LDS_BYTES);
        if (e != hipSuccess) return e;
        configured = true;
    }
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kern, P::WG,
                                                                P::LDS_BYTES);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const u64 lanes = (u64)num_cus * per_cu * P::WG;
    if (P::HIST16 && p.count > lanes * 65535ull) {
        // Split so no lane counts more than 65535 numbers (u16 counters).
        DetailedLaunch q = p;
        u64 left = p.count;
        while (left) {
            q.count = left < lanes * 65535ull ? left : lanes * 65535ull;
            hipError_t e2 = launch_fd_variant<BASE, V>(q, num_cus, s);
            if (e2 != hipSuccess) return e2;
            add_u128(q.start_lo, q.start_hi, q.count);
            left -= q.count;
        }
        return hipSuccess;
    }
    // ~4 work units per resident lane: balances tails against init cost.
    u64 chunk = (p.count + 4 * lanes - 1) / (4 * lanes);
    if (chunk < 64) chunk = 64;
    if (chunk > (1u << 20)) chunk = 1u << 20;
    const u64 unit = P::H == 1 ? chunk : 64 * chunk;
    const u64 nunits = (p.count + unit - 1) / unit;
    const u64 per_wg = P::H == 1 ? P::WG : P::WG / 64;
    u64 grid = (nunits + per_wg - 1) / per_wg;
    const u64 max_grid = (u64)num_cus * per_cu;
    if (grid > max_grid) grid = max_grid;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(kern, dim3((u32)grid), dim3(P::WG), P::LDS_BYTES, s, p.start_lo, p.start_hi,
                       p.count, chunk, p.cutoff, p.hist, p.out);
    return hipGetLastError();
}

// Variant table.  Index 0 is the production choice per base; the rest exist
// for the variant sweep (scripts/fd_sweep.py, NICE_FD_VARIANT).
using V_contig = FdVariant<1, false, 0, 0>;
using V_il = FdVariant<64, false, 0, 0>;
using V_il_lsd = FdVariant<64, true, 0, 0>;
using V_il_lsd_a2 = FdVariant<64, true, 1, 1>;
using V_il_lsd_a4 = FdVariant<64, true, 2, 2>;
using V_il_lsd_a6 = FdVariant<64, true, 3, 3>;
using V_il_lsd_a8 = FdVariant<64, true, 3, 5>;
using V_contig16 = FdVariant<1, false, 0, 0, true>;
using V_il_lsd16 = FdVariant<64, true, 0, 0, true>;
using V_il_lsd_a2_16 = FdVariant<64, true, 1, 1, true>;
using V_contig16_a2 = FdVariant<1, false, 1, 1, true>;

template <int BASE>
static hipError_t launch_fd_base(const DetailedLaunch &p, int num_cus, hipStream_t s, int var) {
    constexpr bool arith = FdTraits<BASE, V_contig>::ARITH_OK;
    switch (var) {
    case 1: return launch_fd_variant<BASE, V_contig>(p, num_cus, s);
    case 2: return launch_fd_variant<BASE, V_il>(p, num_cus, s);
    case 3: return launch_fd_variant<BASE, V_il_lsd>(p, num_cus, s);
    case 4: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd_a2>(p, num_cus, s); break;
    case 5: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd_a4>(p, num_cus, s); break;
    case 6: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd_a6>(p, num_cus, s); break;
    case 7: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd_a8>(p, num_cus, s); break;
    case 8: return launch_fd_variant<BASE, V_contig16>(p, num_cus, s);
    case 9: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd16>(p, num_cus, s); break;
    case 10: if constexpr (arith) return launch_fd_variant<BASE, V_il_lsd_a2_16>(p, num_cus, s); break;
    case 11: if constexpr (arith) return launch_fd_variant<BASE, V_contig16_a2>(p, num_cus, s); break;
    default: break;
    }
    // Production choice (scripts/fd_sweep.py, profiles/): bases with 64-bit
    // masks use the interleaved walk; b80's larger state stays contiguous
    // (the interleaved layout spills at 256 VGPRs).
    // Production choice, from the variant sweep on MI355X (profiles/r01/):
    // b40: contiguous walk + u16 histograms (4 waves/SIMD) 3.80 ms / 1e9;
    // b50: contiguous, u32 histograms (its 150-VGPR state spills at 4 waves);
    // b80: interleaved walk (2.95 vs 3.09 ms / 2e8).
    if constexpr (BASE == 40) return launch_fd_variant<BASE, V_contig16>(p, num_cus, s);
    else if constexpr (BASE == 80) return launch_fd_variant<BASE, V_il>(p, num_cus, s);
    else return launch_fd_variant<BASE, V_contig>(p, num_cus, s);
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

hipError_t launch_detailed_fd(const DetailedLaunch &p, int num_cus, hipStream_t s, int variant) {
    switch (p.base) {
#define X(b) case b: return launch_fd_base<b>(p, num_cus, s, variant);
        NICE_FD_BASES(X)
#undef X
    default: return hipErrorInvalidValue;
    }
}

}  // namespace nice
