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

// Detailed histograms live in kHistCopies copies of 129 u64 bins (summed by
// the host); a workgroup flushes into copy blockIdx.x % kHistCopies.
constexpr uint32_t kHistCopies = 64;

// In-kernel end of a field (fd2 kernels): the launch's last workgroup sums
// the histogram copies into out_mapped[0..128] (mapped host memory), writes
// the near-miss count to out_mapped[129] and re-zeroes copies, count and
// *done; then, after a system-scope release, seq to out_mapped[130], which the
// host polls instead of waiting for the kernel's completion signal.
// out_mapped == nullptr: the caller runs launch_detailed_finish.
struct FieldFinish {
    uint64_t *out_mapped;
    uint32_t *done;  // kDoneWords arrival counters (nice_device.hpp), re-zeroed by the finish
    uint64_t seq;    // the field's sequence number (nonzero)
    // Nonzero (fields of < 2^31 numbers): every result word is published as
    // tag << 32 | value -- bins 0..base and the near-miss count [129] -- with
    // no ordering among them and no sequence word; the host takes the field
    // as finished once every word carries the tag (one fewer round trip to
    // host memory than stores, wait, release store of the sequence word).
    uint32_t tag;
};

struct DetailedLaunch {
    uint64_t start_lo, start_hi; // first n of the segment
    uint64_t count;              // numbers in the segment
    uint32_t base;
    uint32_t cutoff;             // near-miss cutoff (number_stats.rs:15-17)
    uint64_t *hist;              // kHistCopies x 129 u64 bins, accumulated
    uint32_t hist_copies;        // fd2: copies the field's launches use (set by launch_detailed_fd2)
    NumOut out;
    FieldFinish fin;             // fd2 only; see FieldFinish
    uint32_t *launches;          // if set, incremented per kernel launch enqueued
    uint32_t *sib;               // fd2, if set: [0] sibling lanes M of the field's last sibling-lane
                                 // launch (0: none ran), [1] its lane stride L
    uint32_t overlapped;         // fd2: another field of the device was still running when this one
                                 // was enqueued (the pipelined case), so launches are shaped for
                                 // throughput, not for the latency of a lone field
};

// Production FD kernel (fd2_detailed.hip): bases 40, 50, 80, in-range segments.
bool fd2_supported(uint32_t base);
hipError_t launch_detailed_fd2(const DetailedLaunch &p, int num_cus, hipStream_t s);
// The n where fd2's per-segment limb layout changes (ascending).
size_t fd2_cuts(uint32_t base, unsigned __int128 *out, size_t cap);
// Test hook: every later sibling-lane launch of the process uses lane stride
// L (odd; 0 restores the production pick, fd2_kernel.hpp launch_sib).
void fd2_force_sib_stride(uint32_t L);
// Field epilogue on the launch stream: out_mapped[0..128] = the summed
// histogram copies, out_mapped[129] = *count; copies and counter are zeroed.
hipError_t launch_detailed_finish(uint64_t *hist, uint32_t *count, uint64_t *out_mapped, hipStream_t s);
// Generic per-n kernel: any base 2..128, any n < 2^128.
hipError_t launch_detailed_generic(const DetailedLaunch &p, int num_cus, hipStream_t s);

// Niceonly.  A "leaf" is one MSD-surviving sub-range in stride-index form:
// its candidates are n = b0 + ((g0 + j) / R) * M + residues[(g0 + j) % R],
// j < count (stride_filter.rs:99-155).  Leaves come from the host MSD producer
// or from the device MSD filter below.
struct Leaf {
    uint64_t b0_lo, b0_hi;  // cycle base: range_start - range_start mod M
    uint32_t g0;            // lower_bound(residues, range_start mod M), in [0, R]
    uint32_t count;         // candidates in the range
};

// In-kernel end of a niceonly field (its last candidate launch): the last
// workgroup copies the MSD counters (device MSD) and the nice count into
// mapped host memory, so a field needs no copy launches.
// Every candidate launch ends with its last workgroup re-zeroing the device
// MSD's per-batch leaf-record count (counters[24]) for the next batch; the
// field's last launch instead copies the counters and the nice count out and
// re-zeroes them for the slot's next field (no memset or copy launches).
struct NiceFinish {
    uint32_t *msd_mapped;          // 32 words (device MSD field end) or null
    uint32_t *count_mapped;        // nice count (field end) or null
    uint32_t *msd_counters;        // device MSD counters, or null (host MSD)
    uint32_t *done;                // kDoneWords arrival counters (nice_device.hpp), re-zeroed;
                                   // null: no epilogue
};

struct NiceonlyLaunch {
    const Leaf *leaves;
    const uint32_t *n_leaves_dev;  // leaf count on the device (or null: use n_leaves)
    uint32_t n_leaves;
    const uint32_t *residues;      // R valid residues mod M, ascending
    uint32_t R, M;
    uint32_t base;
    uint32_t in_range;             // every candidate inside the base's valid range
    NumOut out;
    NiceFinish fin;
};
bool niceonly_specialised(uint32_t base);
hipError_t launch_niceonly(const NiceonlyLaunch &p, int num_cus, hipStream_t s);

// Device MSD filter (msd_prefix_filter.rs:583-658 as a level-synchronous BFS):
// one lane per node; leaves (already in stride-index form) are appended to
// `leaves`.  Nodes: {start lo, hi, size, depth}.
// A level-queue node: numbers [start + off, start + off + size) of the field
// (off < field size < 2^63; the level is the queue's).
struct MsdNode {
    uint64_t off, size;
};
struct MsdLaunch {
    // The batch's level-0 nodes are the field's chunks c_j = deal_offset +
    // (first + j) * deal_stride, j < nchunks: [start + c_j chunk, min(end,
    // start + (c_j + 1) chunk)).  deal_stride 1 / offset 0 is a contiguous run
    // of chunks; a rank of an N-way niceonly job is dealt every N-th chunk.
    uint64_t start_lo, start_hi;  // field start (chunk grid origin)
    uint64_t end_lo, end_hi;      // field end
    uint64_t first;               // first dealt chunk of this batch (index among this caller's chunks)
    uint64_t nchunks;             // chunks in this batch
    uint64_t deal_stride, deal_offset;
    uint64_t chunk;               // MSD chunk size (client rule)
    uint64_t floor_size;          // recursion floor (250)
    MsdNode *q[2];                // ping-pong level queues
    uint32_t *counters;           // [0..23] level sizes, [24] leaf records (batch), [25]
                                  // overflow flag, [26] MSD-surviving ranges (sticky),
                                  // [27] square survivors (written at the field's end),
                                  // [28..29] u64 candidates, [30..31] u64 numbers inside
                                  // the ranges (sticky); [32..95] square-survivor partial
                                  // counts (workgroup b adds to 32 + b % 64, sticky)
    uint32_t q_cap;
    Leaf *leaves;
    uint32_t leaf_cap;
    const uint32_t *residues;
    const uint32_t *ranks;        // ranks[r] = lower_bound(residues, r), r in [0, M]
    uint32_t R, M;
    uint32_t base;
    uint32_t in_range;            // the batch lies inside the base's valid range
    uint32_t first_batch;         // init zeroes the field's sticky counters and *nice_count
    uint32_t *nice_count;
    uint32_t probe;               // probe build only (NICE_MSD_PROBE): 1 no skip test, 2 no leaf stride math,
                                  // 4 wave kernel: no candidate test
};
constexpr uint32_t kMsdCounterWords = 96;
// A leaf's candidate count is capped at kLeafPiece: longer runs are stored as
// several leaves, so niceonly_kernel's per-wave sums of 8 leaves fit 32 bits.
constexpr uint32_t kLeafPiece = 1u << 28;
// Node of a chunk's fused recursion: offset from the chunk start, size.
struct ChunkNode {
    uint32_t off, size;
};
constexpr uint32_t kFusedMaxCap = 1u << 14;
// Nodes per level of a fused chunk recursion (a power of two), or 0 when the
// chunk needs the level-launch BFS (chunk / floor too large, or chunk >= 2^32).
uint32_t msd_fused_cap(uint64_t chunk, uint64_t floor_size);
// Enqueue a batch's MSD recursion (no host sync): with `scratch` (grid x 2 x
// cap ChunkNodes) ONE fused launch, one workgroup per chunk; otherwise the
// init + level kernels.
hipError_t launch_msd_device(const MsdLaunch &p, int num_cus, hipStream_t s, ChunkNode *scratch = nullptr,
                             uint32_t cap = 0, uint32_t grid = 0);

// Large chunks: init + the level BFS down to `level0` (nodes <= 2^26 numbers,
// enough roots to fill the chip), then msd_wave_kernel: the recursion below
// level0 AND the candidate test of every leaf in one launch (`c` holds the
// residues, output and finish; its leaf fields are unused), `grid` workgroups
// of msd_wave_waves_per_group() waves, each wave with a kStackCap-node stack
// in `scratch` (msd_wave_scratch_bytes(grid)).  Leaves of the BFS levels go
// to p.leaves and are tested by the same launch.
hipError_t launch_msd_wave(const MsdLaunch &p, const NiceonlyLaunch &c, uint32_t level0, void *scratch,
                           uint32_t grid, int num_cus, hipStream_t s);
size_t msd_wave_scratch_bytes(uint32_t grid);
uint32_t msd_wave_waves_per_group();

// Diagnostics used by the parity tests: per-n unique counts / nice flags
// computed by the same device functions the production kernels use.
hipError_t launch_unique_counts(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                                uint32_t *out, hipStream_t s);
hipError_t launch_is_nice(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                          uint32_t *out, hipStream_t s);
// In-range n of a niceonly fast base (40/50/52/53/54/80): the unique-digit
// count by niceonly_kernel's limb path (radix_fast.hpp unique_fast).
hipError_t launch_unique_fast(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                              uint32_t *out, hipStream_t s);

}  // namespace nice
