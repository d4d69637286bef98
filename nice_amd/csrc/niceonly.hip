// niceonly.hip -- gfx950 kernels for niceonly field processing.
//
// Replaces niceonly_ranges_kernel (common/src/cuda/nice_kernels.cu:420-470),
// the CPU stride walk it mirrors (common/src/stride_filter.rs:139-155) and,
// optionally, the host MSD recursion in front of it
// (common/src/msd_prefix_filter.rs:382-674).
//
// niceonly_kernel: wave-level load balancing.  A wave takes 8 leaves (lanes
// 0..7), scans their candidate counts across the wave, and then walks the
// packed candidate space 64 at a time: lane k finds its leaf by a binary
// search over the wave's exclusive prefix (cross-lane reads), rebuilds n = b0
// + ((g0 + j) / R) * M + residues[(g0 + j) % R] and tests it: in range, the
// digit union of n^2 (pair-mask table in LDS) and, for the few repeat-free
// squares queued per wave, of n^3 has b members (client_process.rs:222-253).
// A leaf holds ~20 candidates at the CPU path's MSD floor of 250 (b40), so
// one-wave-per-range would leave two thirds of a 64-lane wave idle.
//
// msd_fused_kernel: a chunk's whole MSD recursion in one workgroup (chunks up
// to 16384 floors, e.g. the client's 1e6 chunks).
// msd_level_kernel: the MSD recursion as a level-synchronous BFS.  Every node
// of level d is one lane: leaf -> stride-index descriptor appended to the leaf
// list; skippable -> dropped; else two children appended to level d+1.
// msd_wave_kernel: larger chunks -- the level BFS stops at a root level and
// each wave recurses below it with its own work stack, testing the leaves it
// finds in the same launch (see there).
#include "kernels.h"
#include "nice_device.hpp"
#include "probe.hpp"
#include "radix_fast.hpp"

namespace nice {

template <class G>
struct IsConst {
    static constexpr bool value = false;
    static constexpr int base = 0;
};
template <int B>
struct IsConst<ConstBase<B>> {
    static constexpr bool value = true;
    static constexpr int base = B;
};

// ---------------------------------------------------------------------------
// Candidate check kernel
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32 lane_rank(u64 mask) {
    return __builtin_amdgcn_mbcnt_hi((u32)(mask >> 32), __builtin_amdgcn_mbcnt_lo((u32)mask, 0u));
}

// LDS (and, with the workgroup-scope fence, global) accesses of one wave
// ordered across its lanes: a wave runs in lockstep, so no barrier is needed.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void wave_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void emit_nice(const NiceonlyLaunch &p, u64 n_lo, u64 n_hi) {
    const u32 pos = atomicAdd(p.out.count, 1u);
    if (pos < p.out.cap) {
        p.out.n[2 * (u64)pos] = n_lo;
        p.out.n[2 * (u64)pos + 1] = n_hi;
    }
}

// Square-survivor ring per wave (entries; a power of two >= 128: a round adds
// at most 64 to fewer than 64 queued).
constexpr u32 kCubeQ = 128;

// LDS pair-mask table of the in-range test (two-word fast bases): entries
// per base, 1 (unused) otherwise.
template <class G>
struct PairTab {
    static constexpr bool on = IsConst<G>::value && IsConst<G>::base > 32 && IsConst<G>::base <= 64;
    static constexpr u32 N = on ? (u32)IsConst<G>::base * IsConst<G>::base : 1u;
};
// Every thread of the workgroup calls it (ends with a barrier).
template <class G>
__device__ __forceinline__ void pair_tab_fill(uint2 *tab) {
    if constexpr (PairTab<G>::on) {
        constexpr u32 b = IsConst<G>::base;
        for (u32 e = threadIdx.x; e < PairTab<G>::N; e += blockDim.x) {
            const u64 bits = (1ull << (e % b)) | (1ull << (e / b));
            tab[e] = make_uint2((u32)bits, (u32)(bits >> 32));
        }
    }
    __syncthreads();
}

// The full niceness test on `cnt` <= 64 queued candidates, one per lane.  At
// the MSD floor about one stride candidate in ~20 has a repeat-free square
// (the MSD filter already vetted the leading digits), yet nearly every round of
// 64 holds one: testing the cube in place ran the 220-instruction cube for
// almost every wave and round.  Queued, it runs once per 64 survivors.
template <int B>
__device__ __forceinline__ void cube_pass(const NiceonlyLaunch &p, const ulonglong2 *q, u32 head, u32 cnt,
                                          u32 lane, const uint2 *tab) {
    wave_sync_lds();  // the queue was written by other lanes of this wave
    if (lane < cnt) {
        const ulonglong2 e = q[(head + lane) & (kCubeQ - 1)];
        bool nice;
        if constexpr (B > 32 && B <= 64) nice = is_nice_tab<B>(e.x, e.y, tab);
        else nice = is_nice_fast<B>(e.x, e.y);
        if (nice) emit_nice(p, e.x, e.y);
    }
    wave_sync_lds();
}

// Per-wave candidate state: the exact gi / R of the stride walk and the
// square-survivor ring (head / tail wave-uniform).
struct CandWave {
    u64 r_magic;
    u32 r_shift;
    ulonglong2 *cq;
    const uint2 *tab;  // LDS pair-mask table (PairTab), or unused
    u32 q_head, q_tail;
};
__device__ __forceinline__ CandWave cand_wave(const NiceonlyLaunch &p, ulonglong2 *cq, const uint2 *tab) {
    // gi / R by one 32x32->64 multiply and a shift: gi = g0 + j < R + 2^28 <
    // 2^29 and m = floor(2^s / R) + 1 with s = 30 + ceil(log2 R) keep the error
    // below 2^-(L+1) <= 1/(2R), so the quotient is exact (m < 2^31 + 1).
    const u32 r_log = 32 - __clz(p.R - 1);
    return CandWave{(1ull << (30 + r_log)) / p.R + 1, 30 + r_log, cq, tab, 0, 0};
}

// The stride candidates of LPW leaves (lane l < LPW holds leaf l, the others
// count 0), 64 per round: lane k finds its leaf by a uniform binary search over
// the wave's exclusive prefix (cross-lane reads), rebuilds n = b0 + ((g0 + j) /
// R) * M + residues[(g0 + j) % R] and tests it (client_process.rs:222-253).
template <class G, u32 LPW>
__device__ __forceinline__ void check_leaf_group(const NiceonlyLaunch &p, const G &g, const Leaf &lf, u32 lane,
                                                 CandWave &cw) {
    u32 incl = lf.count;
#pragma unroll
    for (int o = 1; o < (int)LPW; o <<= 1) {
        u32 v = __shfl_up(incl, o);
        if (lane >= (u32)o) incl += v;
    }
    const u32 excl = incl - lf.count;
    const u32 total = __shfl(incl, LPW - 1);
    for (u32 r0 = 0; r0 < total; r0 += 64) {
        const u32 k = r0 + lane;
        // largest l < LPW with excl_l <= k (uniform search, all lanes active)
        u32 lo = 0;
#pragma unroll
        for (u32 step = LPW / 2; step >= 1; step >>= 1) {
            const u32 e = __shfl(excl, lo + step);
            if (lo + step < LPW && e <= k) lo += step;
        }
        const u32 j = k - __shfl(excl, lo);
        const u32 g0 = __shfl(lf.g0, lo);
        const u64 b0lo = __shfl(lf.b0_lo, lo), b0hi = __shfl(lf.b0_hi, lo);
        u64 n_lo = 0, n_hi = 0;
        if (k < total) {
            const u32 gi = g0 + j;
            const u32 cyc = (u32)(((u64)gi * cw.r_magic) >> cw.r_shift);
            const u32 idx = gi - cyc * p.R;
            n_lo = b0lo;
            n_hi = b0hi;
            add_u128(n_lo, n_hi, (u64)cyc * p.M + p.residues[idx]);
        }
        if constexpr (IsConst<G>::value) {
            if (p.in_range) {  // wave-uniform
                // n^2 first; the few survivors queue for a full-wave cube pass
                bool sq = false;
                if (k < total) {
                    if constexpr (PairTab<G>::on) sq = square_ok_tab<IsConst<G>::base>(n_lo, n_hi, cw.tab);
                    else sq = square_ok<IsConst<G>::base>(n_lo, n_hi);
                }
                const u64 bal = __ballot(sq);
                if (bal) {
                    if (sq) cw.cq[(cw.q_tail + lane_rank(bal)) & (kCubeQ - 1)] = make_ulonglong2(n_lo, n_hi);
                    cw.q_tail += (u32)__popcll(bal);
                    if (cw.q_tail - cw.q_head >= 64) {
                        cube_pass<IsConst<G>::base>(p, cw.cq, cw.q_head, 64, lane, cw.tab);
                        cw.q_head += 64;
                    }
                }
                continue;
            }
        }
        if (k < total && is_nice_dev(n_lo, n_hi, g)) emit_nice(p, n_lo, n_hi);
    }
}

template <class G>
__device__ __forceinline__ void cand_flush(const NiceonlyLaunch &p, CandWave &cw, u32 lane) {
    if constexpr (IsConst<G>::value) {
        if (cw.q_tail != cw.q_head)
            cube_pass<IsConst<G>::base>(p, cw.cq, cw.q_head, cw.q_tail - cw.q_head, lane, cw.tab);
        cw.q_head = cw.q_tail;
    }
}

// This workgroup's square survivors (every wave's cube-queue total) into the
// field's partial counts (counters[32 + b % 64]): one LDS add per wave, one
// global add per workgroup.  Every thread calls it (a barrier inside).
__device__ __forceinline__ void square_ok_flush(u32 *ctr, u32 *wg_sum, u32 waves_total, u32 lane) {
    if (lane == 0 && waves_total) atomicAdd(wg_sum, waves_total);
    __syncthreads();
    if (threadIdx.x == 0 && ctr && *wg_sum) atomicAdd(&ctr[32 + blockIdx.x % 64], *wg_sum);
}

// End of a niceonly launch (every thread of the workgroup calls it): the last
// workgroup to retire copies the field's results to mapped host memory (the
// count is agent-atomic, so: own atomics drained, barrier, one agent add per
// workgroup -- no L2 write-back fence, see fd2's field_finish).  Field end
// (count_mapped set): the MSD counters and the nice count out, then re-zeroed
// for the slot's next field.  Batch end: only the per-batch leaf-record count
// is re-zeroed, for the next batch.
__device__ __forceinline__ void nice_launch_finish(const NiceFinish &fin, u32 *count) {
    __shared__ u32 last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) last = last_block_arrive(fin.done);
    __syncthreads();
    if (!last) return;
    u32 *ctr = fin.msd_counters;
    const u32 w = threadIdx.x;
    if (fin.count_mapped) {
        if (ctr && w < 64) {  // wave 0
            // the square-survivor partials summed into word 27, then re-zeroed
            u32 part = __hip_atomic_load(&ctr[32 + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctr[32 + w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
            if (w < 32) {
                const u32 v = __hip_atomic_load(&ctr[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                fin.msd_mapped[w] = w == 27 ? part : v;
                if (w >= 24) __hip_atomic_store(&ctr[w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (w == 0) {
            *fin.count_mapped = __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (ctr && w == 24) {
        __hip_atomic_store(&ctr[24], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    done_reset(fin.done);
}

template <class G>
__global__ void __launch_bounds__(256)
niceonly_kernel(NiceonlyLaunch p, G g) {
    const u32 lane = threadIdx.x & 63;
    const u32 gwave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const u32 nwaves = (gridDim.x * blockDim.x) >> 6;
    const u32 n_leaves = p.n_leaves_dev ? min(*p.n_leaves_dev, p.n_leaves) : p.n_leaves;
    __shared__ ulonglong2 cq[4][IsConst<G>::value ? kCubeQ : 1];
    __shared__ uint2 tab[PairTab<G>::N];
    __shared__ u32 sq_sum;
    if (threadIdx.x == 0) sq_sum = 0;
    pair_tab_fill<G>(tab);  // (ends with a barrier)
    CandWave cw = cand_wave(p, cq[threadIdx.x >> 6], tab);
    // LPW leaves per wave (lanes >= LPW carry count 0): at the CPU path's
    // floor a leaf holds ~40 candidates, so 8 leaves keep a wave ~5 rounds
    // deep and spread a 35k-leaf field over ~4400 waves instead of ~550.
    constexpr u32 LPW = 8;
    for (u32 base = gwave * LPW; base < n_leaves; base += nwaves * LPW) {
        const u32 li = base + lane;
        Leaf lf{0, 0, 0, 0};
        if (lane < LPW && li < n_leaves) lf = p.leaves[li];
        check_leaf_group<G, LPW>(p, g, lf, lane, cw);
    }
    cand_flush<G>(p, cw, lane);
    square_ok_flush(p.fin.msd_counters, &sq_sum, cw.q_tail, lane);
    if (p.fin.done) nice_launch_finish(p.fin, p.out.count);
}

__global__ void is_nice_kernel(const u64 *n_pairs, u32 count, GenericBase g, u32 *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = is_nice_dev(n_pairs[2 * i], n_pairs[2 * i + 1], g) ? 1u : 0u;
}

// ---------------------------------------------------------------------------
// Device MSD filter
// ---------------------------------------------------------------------------

// u128 {lo, hi} divided by a u32 (q written back), returns the remainder.
__device__ __forceinline__ u32 divmod_u128(u64 &lo, u64 &hi, u32 d) {
    u32 w[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
    u64 rem = 0;
#pragma unroll
    for (int i = 3; i >= 0; i--) {
        u64 cur = (rem << 32) | w[i];
        w[i] = (u32)(cur / d);
        rem = cur - (u64)w[i] * d;
    }
    lo = ((u64)w[1] << 32) | w[0];
    hi = ((u64)w[3] << 32) | w[2];
    return (u32)rem;
}

__device__ __forceinline__ bool overlaps(const Mask<4> &a, const Mask<4> &b) {
    return ((a.w[0] & b.w[0]) | (a.w[1] & b.w[1]) | (a.w[2] & b.w[2]) | (a.w[3] & b.w[3])) != 0;
}

// Common most-significant-digit prefix of x and y (both consumed), in one
// least-significant-first pass over both, without storing digits: the running
// mask holds the digits seen since the last position where x and y differed,
// and is snapshotted at every non-zero digit of x, so after the pass the
// snapshot is the mask of the common prefix of the two numbers.  Returns false
// if the digit counts differ; lsd0/lsd1 are x's two lowest digits.
struct PrefixScan {
    Mask<4> mask;
    u32 dup;
    u32 lsd0, lsd1;
    int len;
};
template <int NW, class G>
__device__ __forceinline__ bool common_prefix(u32 (&x)[NW], u32 (&y)[NW], const G &g,
                                              PrefixScan &r) {
    int tx = top_word(x), ty = top_word(y);
    Mask<4> cur;
    cur.clear();
    r.mask.clear();
    u32 dup = 0;
    r.dup = 0;
    r.lsd0 = r.lsd1 = 0;
    int pos = 0, lx = 0, ly = 0;
    while (tx >= 0 || ty >= 0) {
        u32 cx = tx >= 0 ? div_chunk<NW>(x, tx, g.D) : 0u;
        u32 cy = ty >= 0 ? div_chunk<NW>(y, ty, g.D) : 0u;
        for (u32 q = 0; q < g.E; q++, pos++) {
            const u32 dx = cx % g.base, dy = cy % g.base;
            cx /= g.base;
            cy /= g.base;
            if (pos == 0) r.lsd0 = dx;
            if (pos == 1) r.lsd1 = dx;
            if (dx != dy) {
                cur.clear();
                dup = 0;
            } else {
                dup |= cur.test_set(dx);
            }
            if (dx) {
                lx = pos + 1;
                r.mask = cur;
                r.dup = dup;
            }
            if (dy) ly = pos + 1;
        }
    }
    r.len = lx;
    return lx == ly;
}

// has_duplicate_msd_prefix (msd_prefix_filter.rs:382-563) on [first, last].
template <class G>
__device__ bool msd_skippable(u64 f_lo, u64 f_hi, u64 l_lo, u64 l_hi, const G &g) {
    u32 fn[4] = {(u32)f_lo, (u32)(f_lo >> 32), (u32)f_hi, (u32)(f_hi >> 32)};
    u32 ln[4] = {(u32)l_lo, (u32)(l_lo >> 32), (u32)l_hi, (u32)(l_hi >> 32)};
    u32 fsq[8], lsq[8];
    mul_words<4, 4>(fn, fn, fsq);
    mul_words<4, 4>(ln, ln, lsq);
    u32 fcu[12], lcu[12];
    mul_words<8, 4>(fsq, fn, fcu);
    mul_words<8, 4>(lsq, ln, lcu);
    PrefixScan sq, cu;
    if (!common_prefix<8>(fsq, lsq, g, sq)) return false;  // digit counts differ
    if (sq.dup) return true;
    if (!common_prefix<12>(fcu, lcu, g, cu)) return false;
    if (cu.dup) return true;
    if (overlaps(sq.mask, cu.mask)) return true;
    // Filter C (MSD_LSD_OVERLAP_K_VALUE = 2): first / b^2 == last / b^2, with
    // *first*'s two lowest digits of n^2 and n^3 (msd_prefix_filter.rs:461-559).
    u64 a_lo = f_lo, a_hi = f_hi, b_lo = l_lo, b_hi = l_hi;
    divmod_u128(a_lo, a_hi, g.base * g.base);
    divmod_u128(b_lo, b_hi, g.base * g.base);
    if (a_lo == b_lo && a_hi == b_hi) {
        Mask<4> ms, mc;
        ms.clear();
        mc.clear();
        u32 ds = 0, dc = 0;
        if (sq.len > 0) ds |= ms.test_set(sq.lsd0);
        if (sq.len > 1) ds |= ms.test_set(sq.lsd1);
        if (cu.len > 0) dc |= mc.test_set(cu.lsd0);
        if (cu.len > 1) dc |= mc.test_set(cu.lsd1);
        if (overlaps(sq.mask, ms) || overlaps(cu.mask, mc) || overlaps(sq.mask, mc) ||
            overlaps(cu.mask, ms) || ds || dc || overlaps(ms, mc))
            return true;
    }
    return false;
}

// Stride-index descriptor of [a, a + size): cycle base b0 = a - a mod M,
// first residue index g0 and candidate count (stride_filter.rs:99-155).
struct LeafDesc {
    u64 b0_lo, b0_hi, count;
    u32 g0;
};
template <u32 MC>
__device__ __forceinline__ LeafDesc leaf_desc(u64 a_lo, u64 a_hi, u64 size, const MsdLaunch &p) {
    if constexpr (MC != 0) {
        // In-range b40 / b50 (n < 2^64) with the k = 2 stride modulus as a
        // compile-time constant: u64 divisions by a constant.
        const u64 a = a_lo, e = a_lo + size;
        const u64 qa = a / MC, qe = e / MC;
        const u32 ra = (u32)(a - qa * MC), re = (u32)(e - qe * MC);
        const u32 g0 = p.ranks[ra], g1 = p.ranks[re];
        return LeafDesc{a - ra, 0, (qe - qa) * p.R + g1 - g0, g0};
    }
    u64 q_lo = a_lo, q_hi = a_hi;
    const u32 ra = divmod_u128(q_lo, q_hi, p.M);
    u64 e_lo = a_lo, e_hi = a_hi;
    add_u128(e_lo, e_hi, size);
    u64 qe_lo = e_lo, qe_hi = e_hi;
    const u32 re = divmod_u128(qe_lo, qe_hi, p.M);
    const u32 g0 = p.ranks[ra], g1 = p.ranks[re];
    // cycles between the two ends (< 2^64 / M for any batch)
    const u64 count = (qe_lo - q_lo) * p.R + g1 - g0;
    u64 b0_lo = a_lo, b0_hi = a_hi;
    b0_hi -= (b0_lo < ra) ? 1 : 0;  // b0 = a - ra (u128 minus u32)
    b0_lo -= ra;
    return LeafDesc{b0_lo, b0_hi, count, g0};
}

// Wave-level helpers (every lane of the wave calls them together).
__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// Reserve `mine` slots per lane in counter *ctr with ONE atomic per wave;
// returns this lane's first slot.
__device__ __forceinline__ u32 wave_reserve(u32 *ctr, u32 mine) {
    u32 incl = mine;
    const u32 lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 v = __shfl_up(incl, o);
        if (lane >= (u32)o) incl += v;
    }
    const u32 total = __shfl(incl, 63);
    u32 base = 0;
    if (lane == 0 && total) base = atomicAdd(ctr, total);
    return __shfl(base, 0) + incl - mine;
}

// Level 0: this batch's chunks of the field (dealt: every deal_stride-th
// chunk from deal_offset), each clipped to the field's end.
__global__ void msd_init_kernel(MsdLaunch p) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < p.nchunks;
         i += (u64)gridDim.x * blockDim.x) {
        const u64 c = p.deal_offset + (p.first + i) * p.deal_stride;
        u64 lo = p.start_lo, hi = p.start_hi;
        // c * chunk < field size < 2^64 (checked by the host)
        add_u128(lo, hi, c * p.chunk);
        // numbers left in the field from this chunk's start: end - lo (u128)
        const u64 rem_lo = p.end_lo - lo;
        const u64 rem_hi = p.end_hi - hi - (p.end_lo < lo ? 1 : 0);
        const u64 size = rem_hi || rem_lo > p.chunk ? p.chunk : rem_lo;
        p.q[0][i] = MsdNode{c * p.chunk, size};
    }
    // counters: [0] level-0 size, [1..24] per batch, [25..31] sticky over the
    // field (zeroed with the first batch, as is the field's nice count)
    if (blockIdx.x == 0 && threadIdx.x < 32) {
        const u32 w = threadIdx.x;
        if (w == 0) p.counters[0] = (u32)p.nchunks;
        else if (w < 25 || p.first_batch) p.counters[w] = 0;
        if (w == 0 && p.first_batch) *p.nice_count = 0;
    }
}

// Reserve `mine` slots per thread of a 256-thread workgroup with ONE atomic
// per workgroup (same-address atomics from every wave of the chip serialise in
// L2: ~1000 per level cost ~40 us).  All threads must call it; `slots` is 4
// words of LDS.  Returns this thread's first slot.
__device__ __forceinline__ u32 block_reserve(u32 *ctr, u32 mine, u32 *slots) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 v = __shfl_up(incl, o);
        if (lane >= (u32)o) incl += v;
    }
    if (lane == 63) slots[wave] = incl;
    __syncthreads();
    u32 before = 0, total = 0;
#pragma unroll
    for (u32 w = 0; w < 4; w++) {
        const u32 t = slots[w];
        before += w < wave ? t : 0u;
        total += t;
    }
    __syncthreads();
    if (threadIdx.x == 0) slots[0] = total ? atomicAdd(ctr, total) : 0u;
    __syncthreads();
    const u32 base = slots[0];
    __syncthreads();
    return base + before + incl - mine;
}

// The recursion's rule for one node (msd_prefix_filter.rs:583-658):
// 0 = dropped (has_duplicate_msd_prefix), 1 = leaf, 2 = split in two.
template <class G, bool TAB = false>
__device__ __forceinline__ u32 classify_node(const MsdLaunch &p, u32 level, u64 lo, u64 hi, u64 size,
                                             const G &g, const uint2 *tab = nullptr) {
    bool leaf = level >= 22 || size <= p.floor_size;
    if (leaf) return 1;
    u64 l_lo = lo, l_hi = hi;
    add_u128(l_lo, l_hi, size - 1);
    const bool no_skip_test = kProbes && (p.probe & 1);
    bool skip = false;
    if (size != 1 && !no_skip_test) {
        if constexpr (IsConst<G>::value) {
            skip = p.in_range ? msd_skippable_fast<IsConst<G>::base, TAB>(lo, hi, l_lo, l_hi, tab)
                              : msd_skippable<G>(lo, hi, l_lo, l_hi, g);
        } else {
            skip = msd_skippable<G>(lo, hi, l_lo, l_hi, g);
        }
    }
    if (skip) return 0;
    return size < 2 * p.floor_size ? 1u : 2u;
}

// A leaf's stride-index records (one per kLeafPiece candidates; a range
// without candidates still counts as an MSD-surviving range, none stored),
// appended with one atomic per workgroup; statistics accumulated per lane.
// Every thread of the workgroup calls it (act == 1: this lane has a leaf).
template <u32 MC>
__device__ __forceinline__ void append_leaf(const MsdLaunch &p, u32 act, u64 lo, u64 hi, u64 size,
                                            u32 *slots, u64 &n_st, u64 &c_st, u64 &s_st) {
    LeafDesc ld{0, 0, 0, 0};
    if (kProbes && act == 1 && (p.probe & 2)) {
        ld = LeafDesc{lo, hi, size, 0};
    } else
    if (act == 1) {
        ld = leaf_desc<MC>(lo, hi, size, p);
    }
    const u64 pieces64 = act == 1 ? (ld.count + kLeafPiece - 1) / kLeafPiece : 0;
    const u32 pieces = pieces64 > 0xffffu ? 0xffffu : (u32)pieces64;
    const u32 pos = block_reserve(&p.counters[24], pieces, slots);
    if (act != 1) return;
    if (pieces64 > 0xffffu || (u64)pos + pieces > p.leaf_cap) {
        atomicOr(&p.counters[25], 1u);
    } else {
        u64 b0_lo = ld.b0_lo, b0_hi = ld.b0_hi;
        u64 gi = ld.g0;  // residue-sequence index relative to b0
        for (u32 q = 0; q < pieces; q++) {
            if (gi >= p.R) {  // re-base: g0 < R keeps the kernel's index 32-bit
                const u64 cyc = gi / p.R;
                add_u128(b0_lo, b0_hi, cyc * p.M);
                gi -= cyc * p.R;
            }
            const u64 left = ld.count - (u64)q * kLeafPiece;
            const u32 cnt = left < kLeafPiece ? (u32)left : kLeafPiece;
            p.leaves[pos + q] = Leaf{b0_lo, b0_hi, (u32)gi, cnt};
            gi += cnt;
        }
    }
    n_st++;
    c_st += ld.count;
    s_st += size;
}

// Workgroup statistics -> the sticky counters, one atomic each.
__device__ __forceinline__ void flush_stats(const MsdLaunch &p, u64 n_st, u64 c_st, u64 s_st,
                                            unsigned long long *stat) {
    const u32 lane = threadIdx.x & 63;
    n_st = wave_sum(n_st);
    c_st = wave_sum(c_st);
    s_st = wave_sum(s_st);
    __syncthreads();
    if (lane == 0 && n_st) {
        atomicAdd(&stat[0], (unsigned long long)n_st);
        atomicAdd(&stat[1], (unsigned long long)c_st);
        atomicAdd(&stat[2], (unsigned long long)s_st);
    }
    __syncthreads();
    if (threadIdx.x == 0 && stat[0]) {
        atomicAdd(&p.counters[26], (u32)stat[0]);
        atomicAdd((unsigned long long *)(p.counters + 28), stat[1]);
        atomicAdd((unsigned long long *)(p.counters + 30), stat[2]);
    }
}

template <class G, u32 MC>
__global__ void __launch_bounds__(256)
msd_level_kernel(MsdLaunch p, u32 level, G g) {
    __shared__ u32 slots[4];
    __shared__ unsigned long long stat[3];
    if (threadIdx.x < 3) stat[threadIdx.x] = 0;
    const MsdNode *qin = p.q[level & 1];
    MsdNode *qout = p.q[(level + 1) & 1];
    // (an overflowed level leaves its count above the queue: flagged, and
    // never read past)
    const u32 n_in = min(p.counters[level], p.q_cap);
    // Workgroup-uniform loop: leaves and children are appended with one atomic
    // per workgroup, statistics summed in LDS and added once at the end.
    const u32 stride = gridDim.x * blockDim.x;
    u64 n_st = 0, c_st = 0, s_st = 0;
    for (u32 b0 = blockIdx.x * blockDim.x; b0 < n_in; b0 += stride) {
        const u32 i = b0 + threadIdx.x;
        u32 act = 0;  // 0 drop / idle, 1 leaf, 2 split
        MsdNode nd{0, 0};
        u64 lo = p.start_lo, hi = p.start_hi;
        if (i < n_in) {
            nd = qin[i];
            add_u128(lo, hi, nd.off);
            act = classify_node(p, level, lo, hi, nd.size, g);
        }
        append_leaf<MC>(p, act, lo, hi, nd.size, slots, n_st, c_st, s_st);
        // children
        const u32 cpos = block_reserve(&p.counters[level + 1], act == 2 ? 2u : 0u, slots);
        if (act == 2) {
            if (cpos + 1 >= p.q_cap) {
                atomicOr(&p.counters[25], 1u);
            } else {
                const u64 half = nd.size / 2;
                qout[cpos] = MsdNode{nd.off, half};
                qout[cpos + 1] = MsdNode{nd.off + half, nd.size - half};
            }
        }
    }
    flush_stats(p, n_st, c_st, s_st, stat);
}

// The whole recursion of a chunk in ONE workgroup, level by level with
// workgroup barriers, for chunks whose levels fit `cap` nodes (at most
// chunk / floor: a node splits only if it holds >= 2 floor numbers).  A
// batch is then ONE launch instead of init + up to 23 level launches --
// each of those waited for free CUs behind the detailed kernel that runs
// beside it, and their grids were sized for the unpruned tree.  Nodes are
// (offset in the chunk, size) pairs in a per-workgroup ping-pong queue in
// global memory (`scratch`: gridDim.x x 2 x cap).
template <class G, u32 MC>
__global__ void __launch_bounds__(256)
msd_fused_kernel(MsdLaunch p, ChunkNode *scratch, u32 cap, G g) {
    __shared__ u32 slots[4];
    __shared__ u32 cnt[2];
    __shared__ unsigned long long stat[3];
    if (threadIdx.x < 3) stat[threadIdx.x] = 0;
    ChunkNode *qa = scratch + (u64)blockIdx.x * 2 * cap, *qb = qa + cap;
    u64 n_st = 0, c_st = 0, s_st = 0;
    for (u64 ci = blockIdx.x; ci < p.nchunks; ci += gridDim.x) {
        const u64 c = p.deal_offset + (p.first + ci) * p.deal_stride;
        u64 clo = p.start_lo, chi = p.start_hi;
        add_u128(clo, chi, c * p.chunk);
        const u64 rem_lo = p.end_lo - clo;
        const u64 rem_hi = p.end_hi - chi - (p.end_lo < clo ? 1 : 0);
        const u32 csize = (u32)(rem_hi || rem_lo > p.chunk ? p.chunk : rem_lo);
        if (threadIdx.x == 0) {
            qa[0] = ChunkNode{0u, csize};
            cnt[0] = 1;
            cnt[1] = 0;
        }
        __syncthreads();
        ChunkNode *qin = qa, *qout = qb;
        for (u32 level = 0; level <= 22; level++) {
            const u32 n_in = cnt[0];
            if (n_in == 0) break;
            for (u32 b0 = 0; b0 < n_in; b0 += 256) {
                const u32 i = b0 + threadIdx.x;
                u32 act = 0;
                ChunkNode nd{0u, 0u};
                u64 lo = clo, hi = chi;
                if (i < n_in) {
                    nd = qin[i];
                    add_u128(lo, hi, nd.off);
                    act = classify_node(p, level, lo, hi, nd.size, g);
                }
                append_leaf<MC>(p, act, lo, hi, nd.size, slots, n_st, c_st, s_st);
                if (act == 2) {
                    const u32 cp = atomicAdd(&cnt[1], 2u);
                    if (cp + 2 > cap) {
                        atomicOr(&p.counters[25], 1u);
                    } else {
                        const u32 half = nd.size / 2;
                        qout[cp] = ChunkNode{nd.off, half};
                        qout[cp + 1] = ChunkNode{nd.off + half, nd.size - half};
                    }
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                cnt[0] = cnt[1] > cap ? cap : cnt[1];
                cnt[1] = 0;
            }
            __syncthreads();
            ChunkNode *t = qin;
            qin = qout;
            qout = t;
        }
        __syncthreads();  // the queues are reused by the next chunk
    }
    flush_stats(p, n_st, c_st, s_st, stat);
}

// MSD recursion and candidate test fused, one wave per subtree stream, for
// chunks too large for msd_fused_kernel (the massive field's 1e8 chunks).
// The level BFS above it runs only the first few levels (until a batch has
// tens of thousands of nodes of <= 2^26 numbers); each wave then takes those
// roots grid-strided and recurses with a wave-private work stack in global
// memory: pop up to 64 nodes (one per lane), classify (the reference's node
// rule), push the split nodes' halves.  The stack is topped up with fresh
// roots whenever it holds fewer than 64 nodes, so lanes stay busy across
// small subtrees.  Leaves never leave the wave: their stride descriptors queue
// in LDS and are tested 64 at a time by the candidate code above (square
// first, cube on a full wave of survivors).  No leaf list, no level launches
// below the roots, and no same-address atomic per level iteration: the level
// BFS spent most of its 85 ms on the massive field in launches and in the
// L2-serialised queue and statistics atomics of ~10^4 small launches.
struct StackNode {
    u64 off;    // from the field start
    u32 size;   // <= 2^26 (the host picks the root level for it)
    u32 depth;  // recursion level (the reference's depth, <= 22)
};
// Work stack per wave: a pop takes <= 64 nodes off the top and pushes <= 128
// one level deeper, so at most ~64 nodes per level stay behind (23 levels) plus
// one refill of 64 roots; overflow sets the MSD overflow flag (an error).
constexpr u32 kStackCap = 2048;
// Leaf-descriptor queue per wave: tested 64 at a time, in groups of 16.
constexpr u32 kLeafQ = 128, kLeafGroup = 16;
// 512-thread workgroups: the pair table (<= 23 KB) is shared by 8 waves, two
// workgroups per CU at 4 waves per SIMD.
constexpr u32 kWaveWG = 512;

// Lane walk (two-word in-range bases whose n fit 64 bits: the wave kernel's
// const-modulus instantiations).  Each lane takes one leaf from the wave's
// queue and tests one of its candidates per round, stepping the residue index
// (no division, no search) and taking the next queued leaf when its own runs
// out.  The packed walk of check_leaf_group spends ~10 cross-lane reads per
// round locating each lane's leaf (a binary search over the group's prefix,
// then the leaf's fields).  Queue entries are 16 bytes; the queue is walked
// once it holds kWalkAt leaves (>= 3 per lane, so lanes rarely idle at the
// end).  Massive field: 0.0688 -> 0.0652 s.  (Loading the next round's
// residue ahead of the current test gained nothing, and stepping the limbs by
// the residue gaps instead of converting n lost 7 %: 0.0696 s.)
struct LeafW {
    u64 b0;
    u32 g0, count;
};
constexpr u32 kWalkQ = 256, kWalkAt = 192;

template <int B>
__device__ __forceinline__ void walk_leaves(const NiceonlyLaunch &c, const LeafW *q, u32 head, u32 n, u32 lane,
                                            CandWave &cw) {
    wave_sync_lds();  // queue entries written by other lanes
    u32 taken = 0;    // wave-uniform
    bool have = false;
    u64 cb = 0;  // the candidate's cycle base b0 + k M
    u32 idx = 0, left = 0;
    for (;;) {
        const u64 need = __ballot(!have);
        if (need && taken < n) {  // lanes without a leaf take the next ones
            const u32 r = lane_rank(need);
            if (!have && taken + r < n) {
                const LeafW e = q[(head + taken + r) & (kWalkQ - 1)];
                cb = e.b0;
                idx = e.g0;
                left = e.count;
                if (idx >= c.R) {  // g0 == R: the first candidate is in the next cycle
                    idx -= c.R;
                    cb += c.M;
                }
                have = left != 0;
            }
            const u32 np = (u32)__popcll(need);
            taken = n - taken > np ? taken + np : n;
        }
        if (!__ballot(have)) {
            if (taken >= n) break;
            continue;
        }
        u64 nv = 0;
        bool sq = false;
        if (have) {
            nv = cb + c.residues[idx];
            sq = square_ok_tab<B>(nv, 0, cw.tab);
            if (++idx == c.R) {
                idx = 0;
                cb += c.M;
            }
            have = --left != 0;
        }
        const u64 nv_sq = nv;
        const u64 bal = __ballot(sq);
        if (bal) {
            if (sq) cw.cq[(cw.q_tail + lane_rank(bal)) & (kCubeQ - 1)] = make_ulonglong2(nv_sq, 0ull);
            cw.q_tail += (u32)__popcll(bal);
            if (cw.q_tail - cw.q_head >= 64) {
                cube_pass<B>(c, cw.cq, cw.q_head, 64, lane, cw.tab);
                cw.q_head += 64;
            }
        }
    }
    wave_sync_lds();
}

// 4 waves per SIMD (<= 128 VGPRs) where the base's limb arrays allow it
// without spilling; the three-word b80 path needs ~220.
template <class G>
constexpr int wave_occupancy() { return IsConst<G>::value && IsConst<G>::base > 64 ? 2 : 4; }

template <class G, u32 MC>
__global__ void __launch_bounds__(kWaveWG) __attribute__((amdgpu_waves_per_eu(wave_occupancy<G>())))
msd_wave_kernel(MsdLaunch p, NiceonlyLaunch c, u32 level0, StackNode *scratch, G g) {
    constexpr u32 W = kWaveWG / 64;
    constexpr bool WALK = PairTab<G>::on && MC != 0;  // lane walk (see walk_leaves)
    __shared__ ulonglong2 cq[W][IsConst<G>::value ? kCubeQ : 1];
    __shared__ Leaf lq[W][WALK ? 1 : kLeafQ];
    __shared__ LeafW lw[W][WALK ? kWalkQ : 1];
    __shared__ uint2 tab[PairTab<G>::N];
    __shared__ unsigned long long stat[3];
    __shared__ u32 sq_sum;
    if (threadIdx.x < 3) stat[threadIdx.x] = 0;
    if (threadIdx.x == 0) sq_sum = 0;
    pair_tab_fill<G>(tab);  // (ends with a barrier)
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u64 gwave = (u64)blockIdx.x * W + wv, nwaves = (u64)gridDim.x * W;
    StackNode *st = scratch + gwave * kStackCap;
    Leaf *q = lq[wv];
    LeafW *qw = lw[wv];
    CandWave cw = cand_wave(c, cq[wv], tab);
    u64 n_st = 0, c_st = 0, s_st = 0;

    // Leaves the BFS levels above produced (clipped or depth-limited nodes):
    // already stride descriptors in the batch's leaf list.
    const u32 n_list = min(p.counters[24], p.leaf_cap);
    for (u64 b = gwave * kLeafGroup; b < n_list; b += nwaves * kLeafGroup) {
        Leaf lf{0, 0, 0, 0};
        if (lane < kLeafGroup && b + lane < n_list) lf = p.leaves[b + lane];
        check_leaf_group<G, kLeafGroup>(c, g, lf, lane, cw);
    }

    const MsdNode *roots = p.q[level0 & 1];
    const u64 n_roots = min(p.counters[level0], p.q_cap);
    u64 next = gwave;    // next root of this wave (grid-strided)
    u32 sp = 0;          // stack depth (wave-uniform)
    u32 lq_head = 0, lq_tail = 0;
    for (;;) {
        if (sp < 64 && next < n_roots) {  // top up with roots
            const u64 ri = next + (u64)lane * nwaves;
            const bool ok = lane < 64 - sp && ri < n_roots;
            if (ok) {
                const MsdNode r = roots[ri];
                st[sp + lane] = StackNode{r.off, (u32)r.size, level0};
            }
            const u32 got = (u32)__popcll(__ballot(ok));
            next += (u64)got * nwaves;
            sp += got;
            wave_sync_global();
        }
        if (sp == 0) break;
        const u32 cnt = sp < 64 ? sp : 64;
        sp -= cnt;
        StackNode nd{0, 0, 0};
        if (lane < cnt) nd = st[sp + lane];
        wave_sync_global();  // popped before the pushes below reuse the slots
        u64 lo = p.start_lo, hi = p.start_hi;
        add_u128(lo, hi, nd.off);
        const u32 act = lane < cnt ? classify_node<G, PairTab<G>::on>(p, nd.depth, lo, hi, nd.size, g, tab) : 0u;
        // a leaf: its stride descriptor to the queue (statistics as the
        // reference counts them: every MSD-surviving range)
        LeafDesc ld{0, 0, 0, 0};
        if (act == 1) {
            ld = leaf_desc<MC>(lo, hi, nd.size, p);
            n_st++;
            c_st += ld.count;
            s_st += nd.size;
        }
        const bool put = act == 1 && ld.count != 0 && !(kProbes && (p.probe & 4));  // probe 4: MSD only
        const u64 bl = __ballot(put);
        if (put) {
            if constexpr (WALK) qw[(lq_tail + lane_rank(bl)) & (kWalkQ - 1)] = LeafW{ld.b0_lo, ld.g0, (u32)ld.count};
            else q[(lq_tail + lane_rank(bl)) & (kLeafQ - 1)] = Leaf{ld.b0_lo, ld.b0_hi, ld.g0, (u32)ld.count};
        }
        lq_tail += (u32)__popcll(bl);
        // a split: both halves on the stack, one level deeper
        const u64 bs = __ballot(act == 2);
        const u32 nsplit = (u32)__popcll(bs);
        if (sp + 2 * nsplit > kStackCap) {
            if (lane == 0) atomicOr(&p.counters[25], 1u);  // reported as an error by the host
        } else {
            if (act == 2) {
                const u32 r = sp + 2 * lane_rank(bs), half = nd.size / 2;
                st[r] = StackNode{nd.off, half, nd.depth + 1};
                st[r + 1] = StackNode{nd.off + half, nd.size - half, nd.depth + 1};
            }
            sp += 2 * nsplit;
        }
        wave_sync_global();
        // test queued leaves: the lane walk once kWalkAt are queued, else 64
        // at a time in packed groups
        if constexpr (WALK) {
            if (lq_tail - lq_head >= kWalkAt) {
                walk_leaves<IsConst<G>::base>(c, qw, lq_head, lq_tail - lq_head, lane, cw);
                lq_head = lq_tail;
            }
        } else if (lq_tail - lq_head >= 64) {
            wave_sync_lds();
            for (u32 gq = 0; gq < 64; gq += kLeafGroup) {
                Leaf lf{0, 0, 0, 0};
                if (lane < kLeafGroup) lf = q[(lq_head + gq + lane) & (kLeafQ - 1)];
                check_leaf_group<G, kLeafGroup>(c, g, lf, lane, cw);
            }
            lq_head += 64;
        }
    }
    wave_sync_lds();
    if constexpr (WALK) {
        if (lq_head != lq_tail) walk_leaves<IsConst<G>::base>(c, qw, lq_head, lq_tail - lq_head, lane, cw);
        lq_head = lq_tail;
    }
    while (lq_head != lq_tail) {
        const u32 n = lq_tail - lq_head < kLeafGroup ? lq_tail - lq_head : kLeafGroup;
        Leaf lf{0, 0, 0, 0};
        if (lane < n) lf = q[(lq_head + lane) & (kLeafQ - 1)];
        check_leaf_group<G, kLeafGroup>(c, g, lf, lane, cw);
        lq_head += n;
    }
    cand_flush<G>(c, cw, lane);
    square_ok_flush(c.fin.msd_counters, &sq_sum, cw.q_tail, lane);
    flush_stats(p, n_st, c_st, s_st, stat);
    if (c.fin.done) nice_launch_finish(c.fin, c.out.count);
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
template <class G>
static hipError_t launch_nice(const NiceonlyLaunch &p, const G &g, int num_cus, hipStream_t s) {
    u64 waves = p.n_leaves_dev ? (u64)num_cus * 32 : ((u64)p.n_leaves + 7) / 8;
    u64 grid = (waves + 3) / 4;
    // (probe NICE_NICE_GRID: caps of 128..2048 workgroups tie on the bench
    // step, 1.25e8 and 1e9; profiles/r06/niceonly/nice_grid.log)
    const u64 cap = probe_knob("NICE_NICE_GRID", (u64)num_cus * 8);
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(niceonly_kernel<G>, dim3((u32)grid), dim3(256), 0, s, p, g);
    return hipGetLastError();
}

// Bases with compile-time niceonly kernels (ConstBase: constant divisors in
// the generic paths, radix_fast.hpp's in-range fast paths): the benchmark
// bases and the live production bases (CHANGELOG.md:21).
#define NICE_NICEONLY_BASES(X) X(40) X(50) X(52) X(53) X(54) X(80)

// The k = 2 stride modulus M = (b - 1) b^2 as a compile-time constant, for
// in-range fields whose n fit 64 bits (leaf_desc's u64 path), else 0.
template <int B>
constexpr u32 const_modulus() {
    return Radix<B>::DN <= 11 && B <= 54 ? (u32)((B - 1) * B * B) : 0u;
}

bool niceonly_specialised(uint32_t base) {
    switch (base) {
#define X(b) case b: return true;
        NICE_NICEONLY_BASES(X)
#undef X
    default: return false;
    }
}

hipError_t launch_niceonly(const NiceonlyLaunch &p, int num_cus, hipStream_t s) {
    if (!p.n_leaves_dev && p.n_leaves == 0 && !p.fin.done) return hipSuccess;
    switch (p.base) {
#define X(b) case b: return launch_nice(p, ConstBase<b>{}, num_cus, s);
        NICE_NICEONLY_BASES(X)
#undef X
    default: return launch_nice(p, make_generic(p.base), num_cus, s);
    }
}

template <class G, u32 MC = 0>
static hipError_t launch_msd(const MsdLaunch &p, const G &g, int num_cus, hipStream_t s) {
    hipLaunchKernelGGL(msd_init_kernel, dim3(256), dim3(256), 0, s, p);
    const u64 nchunks = p.nchunks;
    // A node of level d has at most ceil(chunk / 2^d) numbers and splits only
    // if it holds >= 2 * floor, so levels past the first d with
    // ceil(chunk / 2^d) < 2 * floor are empty: launch only levels 0..last
    // (b40 1e9 field, chunk 1e6, floor 250: 12 launches instead of 23).
    u32 last = 0;
    while (last < 22 && ((p.chunk + (1ull << last) - 1) >> last) >= 2 * p.floor_size) last++;
    // Level d holds <= nchunks * 2^d nodes: size its grid to that (the first
    // levels are a few thousand lanes), capped at 8 workgroups per CU.
    for (u32 level = 0; level <= last; level++) {
        const u64 nodes = level < 40 ? nchunks << level : ~0ull;
        u64 grid = (nodes + 255) / 256;
        const u64 cap = (u64)num_cus * 2;
        if (grid > cap || nodes >> level != nchunks) grid = cap;
        hipLaunchKernelGGL((msd_level_kernel<G, MC>), dim3((u32)grid), dim3(256), 0, s, p, level, g);
    }
    return hipGetLastError();
}

// (Measured and not kept, round 6: one wave per chunk instead of four.  On
// the bench field's first 1.25e8 numbers, which have no survivors, the
// pipelined step was 1.3 % faster; on the whole 1e9 field 0.7 % slower (the
// niceonly chain 0.061 against 0.040 ms) and on the 8-way dealt shares, the
// N = 8 load, 0.7-0.9 % slower; profiles/r06/niceonly/msd_wg.log, sp_wg.log.)
template <class G, u32 MC = 0>
static hipError_t launch_fused(const MsdLaunch &p, const G &g, ChunkNode *scratch, u32 cap, u32 grid,
                               hipStream_t s) {
    hipLaunchKernelGGL((msd_fused_kernel<G, MC>), dim3(grid), dim3(256), 0, s, p, scratch, cap, g);
    return hipGetLastError();
}

template <class G, u32 MC = 0>
static hipError_t launch_wave(const MsdLaunch &p, const NiceonlyLaunch &c, u32 level0, StackNode *scratch,
                              u32 grid, const G &g, int num_cus, hipStream_t s) {
    hipLaunchKernelGGL(msd_init_kernel, dim3(256), dim3(256), 0, s, p);
    for (u32 level = 0; level < level0; level++) {
        const u64 nodes = p.nchunks << level;
        u64 lgrid = (nodes + 255) / 256;
        const u64 cap = (u64)num_cus * 2;
        if (lgrid > cap) lgrid = cap;
        hipLaunchKernelGGL((msd_level_kernel<G, MC>), dim3((u32)lgrid), dim3(256), 0, s, p, level, g);
    }
    hipLaunchKernelGGL((msd_wave_kernel<G, MC>), dim3(grid), dim3(kWaveWG), 0, s, p, c, level0, scratch, g);
    return hipGetLastError();
}

hipError_t launch_msd_wave(const MsdLaunch &p, const NiceonlyLaunch &c, uint32_t level0, void *scratch,
                           uint32_t grid, int num_cus, hipStream_t s) {
    if (level0 > 22 || (p.nchunks << level0) >> level0 != p.nchunks) return hipErrorInvalidValue;
    StackNode *st = (StackNode *)scratch;
    switch (p.base) {
#define X(b)                                                                                        \
    case b:                                                                                          \
        if (const_modulus<b>() && p.in_range && p.M == const_modulus<b>())                         \
            return launch_wave<ConstBase<b>, const_modulus<b>()>(p, c, level0, st, grid, ConstBase<b>{}, num_cus, s); \
        return launch_wave(p, c, level0, st, grid, ConstBase<b>{}, num_cus, s);
        NICE_NICEONLY_BASES(X)
#undef X
    default: return launch_wave(p, c, level0, st, grid, make_generic(p.base), num_cus, s);
    }
}

size_t msd_wave_scratch_bytes(uint32_t grid) { return (size_t)grid * (kWaveWG / 64) * kStackCap * sizeof(StackNode); }
uint32_t msd_wave_waves_per_group() { return kWaveWG / 64; }

u32 msd_fused_cap(u64 chunk, u64 floor_size) {
    if (chunk > 0xffffffffull || floor_size == 0) return 0;
    const u64 need = chunk / floor_size + 2;
    if (need > kFusedMaxCap) return 0;
    u32 cap = 64;
    while (cap < need) cap <<= 1;
    return cap;
}

hipError_t launch_msd_device(const MsdLaunch &p, int num_cus, hipStream_t s, ChunkNode *scratch,
                             u32 cap, u32 grid) {
    if (scratch) {  // one workgroup per chunk, all levels in-kernel
        if (p.nchunks > 0xffffffffull) return hipErrorInvalidValue;
        switch (p.base) {
#define X(b)                                                                                      \
    case b:                                                                                        \
        if (const_modulus<b>() && p.in_range && p.M == const_modulus<b>())                       \
            return launch_fused<ConstBase<b>, const_modulus<b>()>(p, ConstBase<b>{}, scratch, cap, grid, s); \
        return launch_fused(p, ConstBase<b>{}, scratch, cap, grid, s);
            NICE_NICEONLY_BASES(X)
#undef X
        default: return launch_fused(p, make_generic(p.base), scratch, cap, grid, s);
        }
    }
    switch (p.base) {
#define X(b)                                                                          \
    case b:                                                                            \
        if (const_modulus<b>() && p.in_range && p.M == const_modulus<b>())           \
            return launch_msd<ConstBase<b>, const_modulus<b>()>(p, ConstBase<b>{}, num_cus, s); \
        return launch_msd(p, ConstBase<b>{}, num_cus, s);
        NICE_NICEONLY_BASES(X)
#undef X
    default: return launch_msd(p, make_generic(p.base), num_cus, s);
    }
}

// Diagnostics: the in-range fast path's unique-digit count (the popcount that
// niceonly_kernel's in-range test compares with the base), per n.
template <int B>
__global__ void unique_fast_kernel(const u64 *n_pairs, u32 count, u32 *out) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = unique_fast<B>(n_pairs[2 * i], n_pairs[2 * i + 1]);
}

hipError_t launch_unique_fast(const uint64_t *n_pairs, uint32_t count, uint32_t base, uint32_t *out,
                              hipStream_t s) {
    switch (base) {
#define X(b)                                                                                     \
    case b:                                                                                       \
        hipLaunchKernelGGL(unique_fast_kernel<b>, dim3((count + 255) / 256), dim3(256), 0, s, n_pairs, \
                           count, out);                                                           \
        return hipGetLastError();
        NICE_NICEONLY_BASES(X)
#undef X
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_is_nice(const uint64_t *n_pairs, uint32_t count, uint32_t base, uint32_t *out,
                          hipStream_t s) {
    hipLaunchKernelGGL(is_nice_kernel, dim3((count + 255) / 256), dim3(256), 0, s, n_pairs, count,
                       make_generic(base), out);
    return hipGetLastError();
}

}  // namespace nice
