/*
 * nice_hip.h -- C ABI of libnice_hip.so, the MI355X (gfx950) field-processing
 * path of wasabipesto/nice.
 *
 * This is the drop-in boundary: plain pointers, sizes and u64 pairs, no torch
 * or HIP types, so a cgo / Rust FFI / ctypes binding can call it directly
 * (INTEGRATION.md shows the Rust `extern "C"` shim the reference would add).
 * Every entry point cites the reference interface it replaces
 * (paths relative to the reference repository root).
 *
 * Conventions
 *  - u128 values are passed as (lo, hi) u64 pairs, the split the reference
 *    GPU path already uses (common/src/client_process_gpu.rs:492-499).
 *  - Ranges are half-open [start, end) like FieldSize (common/src/lib.rs:84-153).
 *  - Every call returns NICE_OK (0) or an error code; nice_last_error() gives
 *    a thread-local message (the reference returns anyhow::Result,
 *    client_process_gpu.rs:777-782, 860-862).
 *  - Output lists are caller-allocated with a capacity; *n_out always receives
 *    the true length.  If it exceeds the capacity the call returns
 *    NICE_ERR_CAPACITY (never a silent truncation) and the caller may retry
 *    with a larger buffer.
 */
#ifndef NICE_HIP_H
#define NICE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NICE_OK 0
#define NICE_ERR_INVALID 1     /* bad argument (empty range, base out of 2..128, ...) */
#define NICE_ERR_HIP 2         /* HIP runtime / kernel failure */
#define NICE_ERR_CAPACITY 3    /* caller's output list too small; *n_out = needed */
#define NICE_ERR_NO_DEVICE 4   /* no usable GPU */
#define NICE_ERR_MSD_OVERFLOW 5 /* device MSD work queues overflowed (msd_floor too small for
                                   chunk_size); not retryable with a larger list */
#define NICE_ERR_BUSY 6         /* *_submit: every slot of the context holds a field in flight;
                                   collect one and submit again (the synchronous calls wait
                                   for a slot instead, see nice_process_range_detailed) */

/* NiceNumberSimple (common/src/lib.rs:182-186). */
typedef struct {
    uint64_t number_lo;
    uint64_t number_hi;
    uint32_t num_uniques;
    uint32_t reserved;
} nice_number;

typedef struct nice_ctx nice_ctx;

/* GpuContext::new(device_ordinal) (client_process_gpu.rs:215-244), extended to a
 * list of devices: a field is sharded into contiguous n-ranges, one per device.
 * No JIT happens here or later: kernels are AOT-built for gfx950. */
int nice_ctx_create(const int *devices, int n_devices, nice_ctx **out);
void nice_ctx_destroy(nice_ctx *ctx);
/* Wait until every stream of the context is idle (the fields in flight have
 * finished on the device; their results still wait for *_collect).  The
 * reference's one-stream context synchronises inside each call
 * (client_process_gpu.rs:858-866); callers timing a pipeline bracket it with this. */
int nice_ctx_synchronize(nice_ctx *ctx);
int nice_device_count(int *out);
const char *nice_last_error(void);

/* process_range_detailed_gpu(&GpuContext, &FieldSize, base) -> FieldResults
 * (client_process_gpu.rs:812-897; CPU semantics client_process.rs:150-191).
 * hist receives base+1 u64 counts indexed by num_uniques (bin 0 is always 0;
 * FieldResults.distribution is bins 1..=base).  out receives the near-misses
 * (num_uniques > floor(base * 0.9f)) in ascending order of number.
 * Thread-safe on a shared context (the reference shares its GpuContext across
 * the client's tasks behind a Mutex, client/src/main.rs:622,
 * client_process_gpu.rs:199-200): when every slot holds a field in flight the
 * call blocks until another thread's collect frees one.  It returns
 * NICE_ERR_BUSY instead only when no other thread could free a slot, which
 * would otherwise deadlock: no field in flight is being collected, and each
 * was submitted by the calling thread or by a thread that is itself blocked
 * in such a call (two threads holding tickets and waiting for each other's
 * slots: the second to call gets NICE_ERR_BUSY). */
int nice_process_range_detailed(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                uint64_t *hist, nice_number *out, size_t cap, size_t *n_out);

/* Niceonly tuning (all zero = reference CPU-path semantics, which make the
 * candidate set identical to process_range_niceonly's):
 *   msd_floor  MSD recursion floor; 0 -> NICE_GPU_MSD_FLOOR from the
 *              environment when set to a number >= 1 (the reference's pin,
 *              client_process_gpu.rs:161-172), else 250 (msd_prefix_filter.rs:282);
 *              NICE_MSD_FLOOR_ADAPTIVE -> the reference GPU path's adaptive
 *              floor (AdaptiveFloor, client_process_gpu.rs:96-184, 551-568):
 *              process-wide, pinned by NICE_GPU_MSD_FLOOR, else seeded at
 *              512 000 / logical cores in [250, 256 000]; after 3 warmup
 *              fields every host-MSD field moves it by msd / gpu-tail time
 *              (nice_adaptive_floor_step).  Device-MSD fields use it without
 *              updating it: their recursion is not a host phase to balance.
 *              A floor above 250 checks a superset of the candidates; the
 *              nice list is unchanged.
 *   chunk_size MSD chunking of the field; 0 -> reference client rule
 *              1e6 * clamp(ceil(size / 1e11), 1, 1000) (client/src/main.rs:158-168)
 *   threads    host MSD worker threads; 0 -> available parallelism (the
 *              affinity mask capped by the cgroup cpu.max quota, as Rust's
 *              std::thread::available_parallelism, client_process_gpu.rs:598;
 *              nice_host_threads)
 *   stride_k   LSD digits in the stride table; 0 -> 2 (client/src/main.rs:19)
 *   msd_where  where the MSD recursion runs: 0 auto (device for stride_k 2),
 *              1 host worker threads, 2 device (level-synchronous kernels)
 *   deal_stride, deal_offset
 *              process only the field's chunks c with c % deal_stride ==
 *              deal_offset (0 / 0 -> every chunk).  Rank r of an N-way job
 *              passes (N, r) with the whole field's bounds: the chunk grid and
 *              hence every chunk's MSD ranges are those of the single-process
 *              run, and survival skew along the field is spread over ranks (the
 *              reference deals descriptors from a shared channel,
 *              client_process_gpu.rs:589-709).
 * Both MSD placements produce the same candidate set. */
#define NICE_MSD_FLOOR_ADAPTIVE UINT64_MAX
#define NICE_MSD_AUTO 0
#define NICE_MSD_HOST 1
#define NICE_MSD_DEVICE 2
typedef struct {
    uint64_t msd_floor;
    uint64_t chunk_size;
    int32_t threads;
    uint32_t stride_k;
    int32_t msd_where;
    uint32_t deal_stride;
    uint32_t deal_offset;
    uint32_t reserved;
} nice_niceonly_opts;

typedef struct {
    uint64_t ranges;        /* MSD-surviving sub-ranges (get_valid_ranges output) */
    uint64_t range_numbers; /* numbers inside them */
    uint64_t candidates;    /* stride candidates checked on the GPU */
    uint32_t launches;
    uint32_t square_ok;     /* device MSD, in-range fast bases: candidates whose square alone
                               has no repeated digit (get_is_nice reached the cube scan),
                               mod 2^32; 0 where not counted (host MSD, other bases) */
    double msd_seconds;     /* until the last MSD worker finished (a field re-run after a
                               list overflow: its last run) */
    double total_seconds;
    uint64_t msd_floor;     /* the MSD recursion floor this field used */
    uint32_t msd_threads;   /* host MSD worker threads the field ran (0: device MSD) */
    uint32_t reruns;        /* times the field re-ran with grown device lists */
} nice_niceonly_stats;

/* AdaptiveFloor::update's step (client_process_gpu.rs:130-157): the floor
 * after a field whose MSD took msd_seconds of total_seconds -- ratio
 * msd / (total - msd), 1.5 when the GPU tail is under 2 ms, 1/1.5 when the
 * MSD is, clamped to [1/1.5, 1.5], the floor to [250, 256 000].  Pure. */
double nice_adaptive_floor_step(double floor, double msd_seconds, double total_seconds);
/* The process-wide adaptive floor now, and the warmup fields left
 * (0xffffffff: pinned by NICE_GPU_MSD_FLOOR). */
int nice_adaptive_floor(double *floor, uint32_t *warmup);

/* process_range_niceonly_gpu(&GpuContext, &FieldSize, base) -> FieldResults
 * (client_process_gpu.rs:515-557; CPU semantics client_process.rs:439-465).
 * Nice numbers (num_uniques = base) ascending.  Residue-empty bases return an
 * empty list (client_process_gpu.rs:525-531). */
int nice_process_range_niceonly(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                nice_number *out, size_t cap, size_t *n_out);
int nice_process_range_niceonly_ex(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                   uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                   const nice_niceonly_opts *opts, nice_number *out,
                                   size_t cap, size_t *n_out, nice_niceonly_stats *stats);

/* The coordination server's submit checks for a detailed result
 * (api/src/main.rs:309-359), which nice_process_range_detailed also applies to
 * its own output before returning (plus the server's recompute of every listed
 * number, on the device): the histogram (base+1 bins) sums to the field size
 * (size_lo, size_hi); every listed number lies above the near-miss cutoff; for
 * each bin above the cutoff the count equals the number of listed entries with
 * that num_uniques; the list length equals the sum of those bins.
 * NICE_OK or NICE_ERR_INVALID with the failed check in nice_last_error(). */
int nice_validate_detailed(uint32_t base, uint64_t size_lo, uint64_t size_hi, const uint64_t *hist,
                           const nice_number *list, size_t n);

/* The reference's CPU API on the host cores, for callers without a GPU and
 * the reference client's CPU mode (cpu_path.cpp).  No device is touched, and
 * the GPU entry points above never fall back to these.
 *
 * process_range_detailed (common/src/client_process.rs:150-191): the
 * histogram of unique-digit counts (base+1 bins) and the numbers above the
 * near-miss cutoff, ascending -- same outputs as nice_process_range_detailed.
 *
 * process_range_niceonly (client_process.rs:439-465): get_valid_ranges over
 * the whole range (msd_prefix_filter.rs:665-674, floor 250), then every
 * candidate of the (b-1) * b^k stride table (stride_filter.rs:139-155; k =
 * stride_k, 0 -> 2) tested with get_is_nice; the nice numbers, ascending.
 *
 * threads: host threads (< 1 -> 1, the reference's single-threaded call);
 * the range (detailed) or the surviving MSD ranges (niceonly) are split
 * into contiguous pieces.  Errors: NICE_ERR_INVALID (base outside 2..128,
 * end < start), NICE_ERR_CAPACITY (*n_out = the required capacity). */
int nice_cpu_process_range_detailed(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                                    uint64_t end_hi, uint32_t base, int32_t threads,
                                    uint64_t *hist, nice_number *out, size_t cap, size_t *n_out);
int nice_cpu_process_range_niceonly(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                                    uint64_t end_hi, uint32_t base, uint32_t stride_k,
                                    int32_t threads, nice_number *out, size_t cap, size_t *n_out);

/* Asynchronous fields.  *_submit enqueues a field on the context's devices
 * and returns at once with a ticket; *_collect waits for that field and
 * returns exactly what the synchronous call would (the synchronous entry
 * points above are submit + collect).  Up to three fields per mode may be in
 * flight on a context, each on its own stream, so a caller can keep the GPU
 * busy with fields i+1 and i+2 while it exchanges / submits the results of
 * field i -- the overlap the reference client gets from its pipelined loop
 * (client/src/main.rs:411-562) -- and a field's first workgroups fill the CUs
 * the previous field's last ones leave idle.  Tickets
 * are collected in any order; NICE_ERR_CAPACITY from a collect keeps the
 * results for a retry with a larger list.  Niceonly with msd_where = host runs
 * its host MSD producer inside submit. */
int nice_detailed_submit(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                         uint64_t end_hi, uint32_t base, int *ticket);
int nice_detailed_collect(nice_ctx *ctx, int ticket, uint64_t *hist, nice_number *out, size_t cap,
                          size_t *n_out);
int nice_niceonly_submit(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                         uint64_t end_hi, uint32_t base, const nice_niceonly_opts *opts, int *ticket);
int nice_niceonly_collect(nice_ctx *ctx, int ticket, nice_number *out, size_t cap, size_t *n_out,
                          nice_niceonly_stats *stats);

/* Device time of the hot kernel(s) of the last collected detailed field on a
 * device, measured with HIP events on the launch stream (kernel_ms 0 when the
 * field ran with kernel timing off). */
typedef struct {
    double kernel_ms;    /* summed over launches; 0 when the field was not timed */
    uint32_t launches;
    uint32_t fd_kernel;  /* 1 if the finite-difference kernel ran */
    uint64_t numbers;    /* numbers processed by those launches */
    uint32_t sib_lanes;  /* sibling lanes M of the FD kernel's last sibling-lane launch (0: none ran) */
    uint32_t sib_stride; /* ... and its lane stride L */
} nice_kernel_stats;
int nice_last_kernel_stats(nice_ctx *ctx, int device_index, nice_kernel_stats *out);
/* Kernel timing of later detailed fields on this context (default on): with
 * it off a field records no HIP events -- two fewer runtime calls on the
 * submit path of every field, which is what a latency-bound caller of small
 * fields pays for (the reference client never reads kernel times) -- and
 * nice_last_kernel_stats reports kernel_ms 0. */
int nice_ctx_set_kernel_timing(nice_ctx *ctx, int enable);

/* Host helpers mirroring the reference functions the client calls. */
/* std::thread::available_parallelism() (client_process_gpu.rs:598): the
 * process's CPU affinity mask, capped by the cgroup v2 cpu.max quotas of its
 * cgroup and the cgroup's ancestors (quota / period rounded down, at least 1,
 * as Rust's std does).  The host MSD pool's size when
 * nice_niceonly_opts.threads is 0. */
uint32_t nice_host_threads(void);
/* Test hook: every later sibling-lane launch of the FD kernel in this
 * process uses lane stride L (odd, <= 255) instead of the bank-conflict
 * model's pick, and fields of >= 4 super-blocks take the sibling kernel
 * whatever their size; 0 restores production.  NICE_ERR_INVALID otherwise. */
int nice_debug_force_sib_stride(uint32_t L);
/* Test hook: the cpu.max cap nice_host_threads applies for the cgroup
 * `cgroup_path` under a cgroup2 mount at `root` (0 = no quota). */
uint32_t nice_debug_cgroup_cpus(const char *root, const char *cgroup_path);
/* get_base_range_u128 (base_range.rs:43-54): 1 range, 0 none, -1 exceeds u128. */
int nice_base_range(uint32_t base, uint64_t *start_lo, uint64_t *start_hi, uint64_t *end_lo,
                    uint64_t *end_hi);
/* get_near_miss_cutoff (number_stats.rs:15-17). */
uint32_t nice_near_miss_cutoff(uint32_t base);
/* pub const GPU_BATCH_SIZE / PROCESSING_CHUNK_SIZE (client_process_gpu.rs:54, 59). */
uint64_t nice_gpu_batch_size(void);
uint64_t nice_processing_chunk_size(void);
/* gpu_supports_base (client_process_gpu.rs:473-476): every base 2..128 runs on
 * the GPU here (no CPU fallback). */
int nice_gpu_supports_base(uint32_t base);
/* 1 if detailed fields of this base inside its range use the FD kernel. */
int nice_fd_kernel_base(uint32_t base);

/* Host MSD filter, get_valid_ranges_recursive (msd_prefix_filter.rs:583-674)
 * with max depth 22 and factor 2: writes (start_lo, start_hi, end_lo, end_hi)
 * quadruples, returns the true count via *n_out. */
int nice_msd_valid_ranges(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                          uint64_t end_hi, uint32_t base, uint64_t floor_size, uint64_t *out,
                          size_t cap, size_t *n_out);
/* has_duplicate_msd_prefix (msd_prefix_filter.rs:382-563): 1 skippable, 0 not. */
int nice_msd_skippable(uint64_t start_lo, uint64_t start_hi, uint64_t end_lo, uint64_t end_hi,
                       uint32_t base);
/* StrideTable::new(base, k) (stride_filter.rs:40-87): modulus and residue count. */
int nice_stride_table(uint32_t base, uint32_t k, uint64_t *modulus, uint32_t *residues,
                      size_t cap, size_t *n_out);

/* Test hooks (no device needed): the in-range fast paths of the niceonly
 * kernels (radix_fast.hpp) evaluated on the host, bases 40/50/52/53/54/80 with n (and
 * [start, end)) inside the base's valid range.  is_nice: 1/0 like get_is_nice
 * (client_process.rs:222-253); msd: 1/0 like has_duplicate_msd_prefix on
 * [start, end - 1] (msd_prefix_filter.rs:382-563); unique: the unique-digit
 * count of n^2 and n^3 by the same limb path (get_num_unique_digits,
 * client_process.rs:47-143).  NICE_ERR_INVALID otherwise. */
int nice_check_is_nice_inrange(uint32_t base, uint64_t n_lo, uint64_t n_hi);
int nice_check_unique_inrange(uint32_t base, uint64_t n_lo, uint64_t n_hi);
int nice_check_msd_skippable_inrange(uint32_t base, uint64_t start_lo, uint64_t start_hi,
                                     uint64_t end_lo, uint64_t end_hi);
/* Limb-count cuts of the production FD kernel (fd2_detailed.hip): the n at
 * which a segment ending there needs a wider (D1, E1, E2) limb layout.  Writes
 * (lo, hi) pairs, returns the count via *n_out.  Bases without an FD kernel: 0. */
int nice_fd_segment_cuts(uint32_t base, uint64_t *out, size_t cap, size_t *n_out);

/* Diagnostics: per-n results of the device functions the kernels use. */
int nice_debug_unique_counts(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count,
                             uint32_t base, uint32_t *out);
int nice_debug_is_nice(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count, uint32_t base,
                       uint32_t *out);
/* The niceonly kernel's in-range limb path (bases 40/50/52/53/54/80, every n
 * inside the base's valid range, else NICE_ERR_INVALID): the unique-digit
 * count its niceness test compares with the base. */
int nice_debug_unique_fast(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count, uint32_t base,
                           uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
