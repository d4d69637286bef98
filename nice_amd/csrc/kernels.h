// kernels.h -- host-side launch entry points for the gfx950 kernels
// (implemented in detailed.hip / niceonly.hip, used by nice_abi.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nice {

// Near-miss / nice-number output buffer on the device.
struct NumOut {
    uint64_t *n;     // (lo, hi) pairs
    uint32_t *u;     // num_uniques per entry (may be null for niceonly)
    uint32_t *count; // atomically incremented; may exceed cap (overflow detection)
    uint32_t cap;
};

struct DetailedLaunch {
    uint64_t start_lo, start_hi; // first n of the segment
    uint64_t count;              // numbers in the segment
    uint32_t base;
    uint32_t cutoff;             // near-miss cutoff (number_stats.rs:15-17)
    uint64_t *hist;              // base+1 u64 bins, accumulated
    NumOut out;
};

// Bases with a finite-difference kernel (valid only for n inside the base's
// range, where n^2 and n^3 have fixed digit counts).
bool fd_supported(uint32_t base);
// Launch the FD kernel over an in-range segment.  grid_cap: max workgroups.
hipError_t launch_detailed_fd(const DetailedLaunch &p, int num_cus, hipStream_t s, int variant = 0);
// Generic per-n kernel: any base 2..128, any n < 2^128.
hipError_t launch_detailed_generic(const DetailedLaunch &p, int num_cus, hipStream_t s);

// Niceonly: candidates are enumerated on the device from range descriptors.
struct NiceonlyLaunch {
    const uint64_t *b0;       // per range: u128 cycle base (lo, hi pairs) = start - start % M
    const uint32_t *g0;       // per range: residue-sequence index of the first candidate
    const uint64_t *prefix;   // per range: exclusive prefix sum of candidate counts (n_ranges+1)
    uint32_t n_ranges;
    uint64_t total;           // total candidates = prefix[n_ranges]
    const uint32_t *residues; // R valid residues mod M, ascending
    uint32_t R, M;
    uint32_t base;
    NumOut out;
};
bool niceonly_specialised(uint32_t base);
hipError_t launch_niceonly(const NiceonlyLaunch &p, int num_cus, hipStream_t s);

// Diagnostics used by the parity tests: per-n unique counts / nice flags
// computed by the same device functions the production kernels use.
hipError_t launch_unique_counts(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                                uint32_t *out, hipStream_t s);
hipError_t launch_is_nice(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                          uint32_t *out, hipStream_t s);

}  // namespace nice
