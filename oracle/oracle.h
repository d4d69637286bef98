/*
 * oracle.h -- CPU restatement of wasabipesto/nice's field-processing algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under nice_amd/ links, loads or calls this
 * code.  It exists so tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg can check (and time) the HIP product against an
 * independent restatement of the reference's CPU path.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to the reference repository root).  The restatement is pinned against the
 * reference's own golden vectors and against fixtures generated with the
 * reference's Python mirror (scripts/inspect_number.py); see
 * tests/golden/ and tests/test_oracle_golden.py.
 *
 * Integers up to u128 travel as {lo, hi} u64 pairs (the split the reference
 * GPU ABI already uses, common/src/client_process_gpu.rs:492-499).
 */
#ifndef NICE_ORACLE_H
#define NICE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* common/src/base_range.rs:14-54. Returns 1 and fills [start, end) when the
 * base has a valid u128 range, 0 when it has none (b % 5 == 1, or start >= end),
 * -1 when the bounds do not fit in u128. */
int oracle_base_range(uint32_t base, uint64_t *start_lo, uint64_t *start_hi,
                      uint64_t *end_lo, uint64_t *end_hi);

/* common/src/number_stats.rs:15-17: floor(base as f32 * 0.9f32). */
uint32_t oracle_near_miss_cutoff(uint32_t base);

/* common/src/client_process.rs:47-143 (all dispatch arms agree). */
uint32_t oracle_num_unique_digits(uint64_t n_lo, uint64_t n_hi, uint32_t base);

/* common/src/client_process.rs:222-413: early exit on the first repeated
 * digit, scanning n^2 (LSD first) then n^3.  Note: returns 1 for any n whose
 * digits never repeat, even if fewer than `base` digits exist (the reference
 * CPU semantics; only in-range n are guaranteed to have exactly `base`). */
int oracle_is_nice(uint64_t n_lo, uint64_t n_hi, uint32_t base);

/* Number of digits examined (in the reference's scan order, n^2 LSD-first
 * then n^3 LSD-first) up to and including the first repeated digit; equals
 * the total digit count when no digit repeats.  Diagnostic for the device
 * early-exit path. */
uint32_t oracle_scan_depth(uint64_t n_lo, uint64_t n_hi, uint32_t base);

/* common/src/client_process.rs:150-191.  hist has base+1 entries (index =
 * num_uniques; bin 0 always 0).  Near-misses (num_uniques > cutoff) are
 * written ascending as (lo, hi) pairs into miss_n and their counts into
 * miss_u, up to cap entries; *n_miss receives the true count.
 * Returns 0, or 1 if the list overflowed cap. */
int oracle_process_range_detailed(uint64_t start_lo, uint64_t start_hi,
                                  uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                  uint64_t *hist, uint64_t *miss_n, uint32_t *miss_u,
                                  size_t cap, size_t *n_miss);

/* client/src/main.rs:120-254 for SearchMode::Detailed: chunk the field as the
 * reference client does (1e6 * clamp(ceil(size/1e11), 1, 1000)), process the
 * chunks on `threads` POSIX threads, merge the histograms and concatenate the
 * near-miss lists in chunk order.  Same outputs as above. */
int oracle_process_field_detailed_mt(uint64_t start_lo, uint64_t start_hi,
                                     uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                     int threads, uint64_t *hist, uint64_t *miss_n,
                                     uint32_t *miss_u, size_t cap, size_t *n_miss);

/* common/src/residue_filter.rs:6-11.  Writes the valid residues mod (b-1)
 * ascending into out (capacity base), returns their count. */
uint32_t oracle_residue_filter(uint32_t base, uint32_t *out);

/* common/src/lsd_filter.rs:132-148 + 174-224 (extract_digits stops at zero).
 * bitmap has base^k bytes.  Returns the number of valid suffixes, or -1 if
 * base^k overflows u32. */
int64_t oracle_lsd_bitmap(uint32_t base, uint32_t k, uint8_t *bitmap);

/* common/src/stride_filter.rs:40-87.  Writes M = (b-1)*b^k to *modulus and the
 * valid residues mod M ascending into residues (capacity cap); returns their
 * count (may exceed cap, in which case only cap are written). */
uint64_t oracle_stride_residues(uint32_t base, uint32_t k, uint64_t *modulus,
                                uint64_t *residues, uint64_t cap);

/* common/src/msd_prefix_filter.rs:382-563 (has_duplicate_msd_prefix), on the
 * half-open range [start, end). */
/* Study switch (scripts/filter_c_share.py): 0 turns Filter C off (default 1). */
void oracle_set_filter_c(int on);
int oracle_has_duplicate_msd_prefix(uint64_t start_lo, uint64_t start_hi,
                                    uint64_t end_lo, uint64_t end_hi, uint32_t base);

/* common/src/msd_prefix_filter.rs:583-658 with max_depth 22, subdivision factor
 * 2 and the given floor (min_range_size; the reference CPU default is 250,
 * :281-287).  Writes surviving sub-ranges as (start_lo, start_hi, end_lo,
 * end_hi) quadruples, up to cap ranges; returns the true count. */
uint64_t oracle_valid_ranges(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                             uint64_t end_hi, uint32_t base, uint64_t floor_size,
                             uint64_t *out, uint64_t cap);

/* common/src/client_process.rs:439-465 with StrideTable::new(base, k)
 * (stride_filter.rs:99-155).  Nice numbers ascending as (lo, hi) pairs;
 * returns the true count.  *n_candidates receives the number of stride
 * candidates tested (diagnostic). */
uint64_t oracle_process_range_niceonly(uint64_t start_lo, uint64_t start_hi,
                                       uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                       uint32_t k, uint64_t floor_size, uint64_t *out,
                                       uint64_t cap, uint64_t *n_candidates);

/* client/src/main.rs:120-254 for SearchMode::Niceonly (chunking as above,
 * stride k = DEFAULT_LSD_K_VALUE = 2, main.rs:19), on `threads` threads. */
uint64_t oracle_process_field_niceonly_mt(uint64_t start_lo, uint64_t start_hi,
                                          uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                          int threads, uint64_t *out, uint64_t cap,
                                          uint64_t *n_candidates);
/* The same with an explicit MSD chunk size (0 -> client rule) and floor (0 ->
 * 250); *n_ranges receives the number of MSD-surviving ranges. */
uint64_t oracle_process_field_niceonly_ex(uint64_t start_lo, uint64_t start_hi,
                                          uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                          int threads, uint64_t chunk, uint64_t floor_size,
                                          uint64_t *out, uint64_t cap, uint64_t *n_candidates,
                                          uint64_t *n_ranges);
/* _ex plus *n_sq: candidates whose square alone has no repeated digit (test
 * statistic pinning the GPU's square-survivor count). */
uint64_t oracle_process_field_niceonly_sq(uint64_t start_lo, uint64_t start_hi,
                                          uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                          int threads, uint64_t chunk, uint64_t floor_size,
                                          uint64_t *out, uint64_t cap, uint64_t *n_candidates,
                                          uint64_t *n_ranges, uint64_t *n_sq);

#ifdef __cplusplus
}
#endif
#endif
