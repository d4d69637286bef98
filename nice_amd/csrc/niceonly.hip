// niceonly.hip -- gfx950 kernel for niceonly field processing.
//
// Replaces niceonly_ranges_kernel (common/src/cuda/nice_kernels.cu:420-470)
// and the CPU stride walk it mirrors (common/src/stride_filter.rs:139-155).
//
// The host MSD-prefix filter (msd_prefix_filter.rs:583-674) emits surviving
// sub-ranges; the host turns each into a descriptor {B0, g0, prefix}:
//   B0     = range_start - range_start mod M       (u128, M = (b-1) b^k)
//   g0     = index of the first valid residue >= range_start mod M
//   prefix = exclusive prefix sum of the per-range candidate counts.
// Candidates are flattened across ranges (load-balanced: one lane per
// candidate, however short the ranges are -- at the CPU path's MSD floor of
// 250 a range holds ~20 candidates, a third of a 64-lane wave).  Lane c finds
// its range by binary search over `prefix`, reconstructs
//   n = B0 + (g / R) * M + residues[g % R],  g = g0 + (c - prefix[r]),
// and runs the reference's early-exit check (client_process.rs:222-253).
#include "kernels.h"
#include "nice_device.hpp"

namespace nice {

template <class G>
__global__ void __launch_bounds__(256)
niceonly_kernel(NiceonlyLaunch p, G g) {
    for (u64 c = (u64)blockIdx.x * 256 + threadIdx.x; c < p.total; c += (u64)gridDim.x * 256) {
        // largest r with prefix[r] <= c (that range is non-empty)
        u32 lo = 0, hi = p.n_ranges;
        while (hi - lo > 1) {
            u32 mid = (lo + hi) >> 1;
            if (p.prefix[mid] <= c) lo = mid;
            else hi = mid;
        }
        const u32 gi = p.g0[lo] + (u32)(c - p.prefix[lo]);
        const u32 cyc = gi / p.R;
        const u32 j = gi - cyc * p.R;
        u64 n_lo = p.b0[2 * lo], n_hi = p.b0[2 * lo + 1];
        add_u128(n_lo, n_hi, (u64)cyc * p.M + p.residues[j]);
        if (is_nice_dev(n_lo, n_hi, g)) {
            u32 pos = atomicAdd(p.out.count, 1u);
            if (pos < p.out.cap) {
                p.out.n[2 * (u64)pos] = n_lo;
                p.out.n[2 * (u64)pos + 1] = n_hi;
            }
        }
    }
}

__global__ void is_nice_kernel(const u64 *n_pairs, u32 count, GenericBase g, u32 *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = is_nice_dev(n_pairs[2 * i], n_pairs[2 * i + 1], g) ? 1u : 0u;
}

template <class G>
static hipError_t launch_nice(const NiceonlyLaunch &p, const G &g, int num_cus, hipStream_t s) {
    u64 grid = (p.total + 255) / 256;
    const u64 cap = (u64)num_cus * 16;
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(niceonly_kernel<G>, dim3((u32)grid), dim3(256), 0, s, p, g);
    return hipGetLastError();
}

#define NICE_NICEONLY_BASES(X) X(40) X(50) X(80)

bool niceonly_specialised(uint32_t base) {
    switch (base) {
#define X(b) case b: return true;
        NICE_NICEONLY_BASES(X)
#undef X
    default: return false;
    }
}

hipError_t launch_niceonly(const NiceonlyLaunch &p, int num_cus, hipStream_t s) {
    if (p.total == 0) return hipSuccess;
    switch (p.base) {
#define X(b) case b: return launch_nice(p, ConstBase<b>{}, num_cus, s);
        NICE_NICEONLY_BASES(X)
#undef X
    default: return launch_nice(p, make_generic(p.base), num_cus, s);
    }
}

hipError_t launch_is_nice(const uint64_t *n_pairs, uint32_t count, uint32_t base, uint32_t *out,
                          hipStream_t s) {
    hipLaunchKernelGGL(is_nice_kernel, dim3((count + 255) / 256), dim3(256), 0, s, n_pairs, count,
                       make_generic(base), out);
    return hipGetLastError();
}

}  // namespace nice
