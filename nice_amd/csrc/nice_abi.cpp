// nice_abi.cpp -- C ABI (include/nice_hip.h) over the gfx950 kernels.
//
// Replaces the reference's CUDA host pipeline (common/src/client_process_gpu.rs):
// no NVRTC (kernels are AOT code objects), one HIP stream per device, fields
// sharded across devices as contiguous n-ranges, histograms summed and
// near-miss / nice lists merged on the host, the MSD recursion on the device
// (or a multi-threaded host producer streaming range descriptors).
//
// Fields are processed asynchronously: every device owns kSlots result slots
// per mode (device state block, mapped result words, output lists, events), so
// a caller can submit field i+1 before collecting field i and the GPU never
// waits for the host between fields (nice_*_submit / nice_*_collect).  The
// synchronous reference-shaped entry points are submit + collect.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nice_hip.h"
#include "host_math.hpp"
#include "kernels.h"
#include "probe.hpp"
#include "radix_fast.hpp"

using nice::u128;

namespace {

// Per-slot state block: kHistCopies histograms of 129 u64 bins (kernels
// spread their end-of-launch atomics over the copies: hundreds of workgroups
// adding to ONE address serialise in L2), then the two list counters.
constexpr size_t kHistCopies = nice::kHistCopies;
// (+ the detailed list count and the fd2 finish's arrival counters)
constexpr size_t kDoneWords = 65;  // nice_device.hpp kDoneWords (device-only header)
constexpr size_t kStateBytes = kHistCopies * 129 * 8 + (1 + kDoneWords) * 4;
constexpr int kSlots = 3;  // fields in flight per mode and context
constexpr size_t kFinWords = 132;  // Slot::h_fin

thread_local std::string g_err;

// Slots a context rotates through (probe build: NICE_SLOTS limits it, for
// pipeline-depth experiments).
// How collect waits for a detailed field that ends in fd2's in-kernel finish:
// by polling the sequence word it publishes in mapped memory (default), or
// (probe build: NICE_SPIN=0) by the stream's completion event.
inline bool spin_wait() {
    return nice::probe_knob("NICE_SPIN", 1) != 0;
}

// Streams of a device's slots: bit 0 = the slots share ONE detailed stream
// (consecutive detailed fields run back to back instead of overlapping at
// their edges), bit 1 = they share one niceonly stream.
inline int shared_streams() {
    return (int)nice::probe_knob("NICE_SHARED_STREAMS", 0);
}

inline int slots_used() {
    return std::max(1, std::min(kSlots, (int)nice::probe_knob("NICE_SLOTS", kSlots)));
}

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(NICE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

inline u128 mk(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }
inline uint64_t lo64(u128 v) { return (uint64_t)v; }
inline uint64_t hi64(u128 v) { return (uint64_t)(v >> 64); }

constexpr uint32_t kInitialListCap = 1u << 20;  // NEAR_MISS_CAPACITY (client_process_gpu.rs:74)
constexpr uint32_t kNiceCap = 1u << 16;         // NICE_OUT_CAPACITY (:71)
constexpr uint32_t kBatchRanges = 1u << 16;     // LAUNCH_BATCH_RANGES (:583)

struct LeafBuf {
    // host pinned staging + device copy of one launch's leaf descriptors
    nice::Leaf *h = nullptr, *d = nullptr;
    uint32_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
};

struct MsdBuf {
    // device MSD: ping-pong level queues (or the fused kernel's per-workgroup
    // queues), leaf list, counters (kernels.h).
    nice::MsdNode *q[2] = {nullptr, nullptr};
    nice::ChunkNode *scratch = nullptr;
    void *wscratch = nullptr;  // msd_wave_kernel work stacks
    size_t wscratch_bytes = 0;
    nice::Leaf *leaves = nullptr;
    uint32_t *counters = nullptr;  // 32 words
    uint32_t q_cap = 0, leaf_cap = 0;
    uint64_t scratch_nodes = 0;
    // counters / nice count not known to be zero (first use, or a field that
    // did not end in the candidate kernel's epilogue)
    bool dirty = true;
};

struct ListBuf {
    uint64_t *n = nullptr;  // (lo, hi) pairs
    uint32_t *u = nullptr;  // num_uniques (detailed only)
    uint32_t cap = 0;
};

// One field in flight on one device: its own stream (consecutive fields run
// on alternate streams, so field i+1's first workgroups fill the CUs that
// field i's last ones leave idle), state block, results and MSD buffers.
struct Slot {
    hipStream_t stream = nullptr;   // detailed
    bool own_stream = false, own_nstream = false;  // false: shared with slot 0 (shared_streams)
    hipStream_t nstream = nullptr;  // niceonly: high priority, so its chain of short,
                                    // dependent MSD launches is not queued behind the
                                    // detailed kernels' workgroups
    uint64_t *d_state = nullptr;  // kHistCopies x 129 bins, then d_count
    uint32_t *d_count = nullptr;  // detailed list count
    uint32_t *d_done = nullptr;   // workgroups retired (fd2's in-kernel finish)
    uint32_t *d_nice_count = nullptr;  // niceonly list count
    uint64_t *h_fin = nullptr;    // mapped pinned: summed histogram [0..128], near-miss count [129],
                                  // sequence word [130] (kFinWords)
    uint64_t *d_fin = nullptr;    // device view of h_fin
    ListBuf det, nice;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_done = nullptr, nice_done = nullptr;
    hipEvent_t nt0 = nullptr, nt1 = nullptr;  // niceonly field span on the GPU (adaptive floor)
    uint32_t *h_msd = nullptr;    // mapped: MSD counters at the end of a niceonly field
    uint32_t *h_nice = nullptr;   // mapped: niceonly list count
    uint32_t *d_msd_mapped = nullptr, *d_nice_mapped = nullptr;  // device views
    uint32_t *d_nice_done = nullptr;  // workgroups retired (niceonly in-kernel finish)
    bool dirty = true;            // state block not known to be zero
    bool inflight = false;        // a detailed field enqueued and not yet gathered
    bool timed = false;           // the detailed field records ev0 / ev1 (kernel timing)
    bool marked = false;          // ... or an untimed end marker (ev_done) on a shared stream
    uint64_t seq = 0;             // last detailed field's sequence number
    uint32_t launches = 0;        // ... and its kernel launches (the finish kernel not counted)
    uint32_t sib[2] = {0, 0};     // ... and its last sibling-lane launch: lanes M, stride L
    bool fin_seq = false;         // ... and whether its fd2 finish publishes it
    uint32_t tag = 0;             // ... as tagged words (FieldFinish::tag; 0: bins + sequence word)
    uint32_t tag_words = 0;       // ... bins 0..tag_words-1 (and [129]) carry the tag
    MsdBuf msd;
};

struct Device {
    int id = 0;
    int num_cus = 0;
    hipStream_t aux = nullptr;    // self-check recomputes (never behind a queued field); lazily created
    uint64_t *chk_n = nullptr;    // self-check recompute buffers, grown on demand (a hipFree per
    uint32_t *chk_u = nullptr;    // collect would synchronise the whole device)
    size_t chk_cap = 0;
    Slot slot[kSlots];
    std::map<uint32_t, uint32_t *> residues;  // base*8+k -> device residue table
    std::map<uint32_t, uint32_t *> ranks;     // base*8+k -> lower_bound(residues, r), r in [0, M]
    LeafBuf desc[2];
    int desc_next = 0;
    nice_kernel_stats last{};
    int stats_slot = -1;  // slot whose events last.kernel_ms is still to be read from
};

struct StrideCache {
    std::mutex mu;
    std::map<std::pair<uint32_t, uint32_t>, std::shared_ptr<nice::StrideTable>> tables;
    std::shared_ptr<nice::StrideTable> get(uint32_t base, uint32_t k) {
        std::lock_guard<std::mutex> g(mu);
        auto key = std::make_pair(base, k);
        auto it = tables.find(key);
        if (it != tables.end()) return it->second;
        auto t = std::make_shared<nice::StrideTable>(base, k);
        tables[key] = t;
        return t;
    }
};
StrideCache g_stride;

struct Entry {
    u128 n;
    uint32_t u;
};

// A submitted field, until its results have been handed to the caller.
struct DetJob {
    bool active = false, collected = false;
    bool waiting = false;          // a collect is waiting for it outside the context lock
    std::thread::id owner;         // the submitting thread (acquire_slot's deadlock test)
    u128 s = 0, e = 0;
    uint32_t base = 0;
    std::vector<u128> bounds;      // per-device shard bounds
    std::vector<uint64_t> total;   // merged histogram (after collection)
    std::vector<Entry> all;        // merged near-miss list (after collection)
};
struct NiceJob {
    bool active = false, collected = false;
    bool waiting = false;          // a collect is waiting for it outside the context lock
    std::thread::id owner;         // the submitting thread (acquire_slot's deadlock test)
    // the submitted field, kept so that collect can re-run it (list overflow)
    u128 s = 0, e = 0;
    uint32_t base = 0;
    nice_niceonly_opts opts{};
    bool has_opts = false;
    bool on_device = false;
    bool empty = false;            // nothing enqueued (residue-empty base, no chunk dealt)
    std::vector<char> used;        // devices that ran part of the field
    nice_niceonly_stats st{};
    std::chrono::steady_clock::time_point t0;
    std::vector<Entry> all;
    bool adapt = false;            // host-MSD field on the adaptive floor: update it at collect
    uint32_t reruns = 0;           // times the field was re-run with grown device lists
};

}  // namespace

struct nice_ctx {
    std::vector<Device> devs;
    std::mutex mu;  // serialises calls on one context (client_process_gpu.rs:196-201)
    std::condition_variable freed;  // a collect released a slot (synchronous submits wait on it)
    bool timing = true;  // record HIP events around each detailed field (nice_ctx_set_kernel_timing)
    DetJob det[kSlots];
    NiceJob nice[kSlots];
    int det_next = 0, nice_next = 0;
    // threads blocked in acquire_slot (either mode): they collect nothing
    // until they get a slot, so their fields do not count as freeable
    std::vector<std::thread::id> blocked;
};

namespace {

// The slot a new field takes: the round-robin position if it is free (so
// consecutive fields alternate slots), else the next free one after it
// (tickets may be collected in any order).  -1 if every slot is in flight.
template <class Job>
int free_slot(const Job *jobs, int next) {
    const int n = slots_used();
    for (int i = 0; i < n; i++) {
        const int t = (next + i) % n;
        if (!jobs[t].active) return t;
    }
    return -1;
}

// A free slot for a new field, under ctx->mu (held by `lock`).  Without
// `wait`, NICE_ERR_BUSY when every slot is in flight (the asynchronous
// submits: the caller collects one first).  With `wait` (the synchronous
// reference-shaped calls, which the reference serves behind the context's
// Mutex, client_process_gpu.rs:199-200), block until another thread's
// collect frees one -- unless no other thread can: a field in flight can be
// freed only while a collect is waiting for it, or while its submitter is a
// thread that is not itself blocked here (a blocked thread collects nothing:
// two threads each holding tickets and each waiting for the other's slot
// would otherwise wait forever, so one of them gets NICE_ERR_BUSY).
template <class Job>
int acquire_slot(nice_ctx *ctx, std::unique_lock<std::mutex> &lock, const Job *jobs, int next, bool wait,
                 const char *mode, int *slot) {
    const std::thread::id me = std::this_thread::get_id();
    auto blocked = [&](std::thread::id id) {
        return id == me || std::find(ctx->blocked.begin(), ctx->blocked.end(), id) != ctx->blocked.end();
    };
    auto unblock = [&] {
        auto it = std::find(ctx->blocked.begin(), ctx->blocked.end(), me);
        if (it != ctx->blocked.end()) {
            ctx->blocked.erase(it);
            ctx->freed.notify_all();
        }
    };
    for (;;) {
        const int t = free_slot(jobs, next);
        if (t >= 0) {
            unblock();
            *slot = t;
            return NICE_OK;
        }
        bool freeable = false;
        for (int i = 0; i < slots_used(); i++)
            freeable |= jobs[i].active && (jobs[i].waiting || !blocked(jobs[i].owner));
        if (!wait || !freeable) {
            unblock();
            return fail(NICE_ERR_BUSY, std::string("three ") + mode +
                                           " fields already in flight on this context; collect one first");
        }
        if (std::find(ctx->blocked.begin(), ctx->blocked.end(), me) == ctx->blocked.end()) {
            ctx->blocked.push_back(me);
            // waiters that counted on this thread's fields re-check
            ctx->freed.notify_all();
        }
        ctx->freed.wait(lock);
    }
}

int ensure_listbuf(Device &d, ListBuf &l, uint32_t cap, bool with_u) {
    if (l.cap >= cap) return NICE_OK;
    HIPCHK(hipSetDevice(d.id));
    if (l.n) HIPCHK(hipFree(l.n));
    if (l.u) HIPCHK(hipFree(l.u));
    l.n = nullptr;
    l.u = nullptr;
    HIPCHK(hipMalloc(&l.n, (size_t)cap * 16));
    if (with_u) HIPCHK(hipMalloc(&l.u, (size_t)cap * 4));
    l.cap = cap;
    return NICE_OK;
}

int ensure_desc(LeafBuf &b, uint32_t cap) {
    if (b.cap >= cap) return NICE_OK;
    if (b.pending) HIPCHK(hipEventSynchronize(b.done));
    b.pending = false;
    if (b.h) {
        HIPCHK(hipHostFree(b.h));
        HIPCHK(hipFree(b.d));
    }
    HIPCHK(hipHostMalloc(&b.h, (size_t)cap * sizeof(nice::Leaf), hipHostMallocDefault));
    HIPCHK(hipMalloc(&b.d, (size_t)cap * sizeof(nice::Leaf)));
    if (!b.done) HIPCHK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
    b.cap = cap;
    return NICE_OK;
}

int ensure_msd(Slot &sl, uint32_t q_cap, uint32_t leaf_cap, uint64_t scratch_nodes, size_t wscratch_bytes = 0) {
    MsdBuf &m = sl.msd;
    if (!m.counters) HIPCHK(hipMalloc(&m.counters, nice::kMsdCounterWords * 4));
    if (m.wscratch_bytes < wscratch_bytes) {
        HIPCHK(hipStreamSynchronize(sl.nstream));
        if (m.wscratch) HIPCHK(hipFree(m.wscratch));
        HIPCHK(hipMalloc(&m.wscratch, wscratch_bytes));
        m.wscratch_bytes = wscratch_bytes;
    }
    if (m.scratch_nodes < scratch_nodes) {
        HIPCHK(hipStreamSynchronize(sl.nstream));
        if (m.scratch) HIPCHK(hipFree(m.scratch));
        HIPCHK(hipMalloc(&m.scratch, scratch_nodes * sizeof(nice::ChunkNode)));
        m.scratch_nodes = scratch_nodes;
    }
    if (m.q_cap < q_cap) {
        // this slot's previous field may still be reading the old queues
        HIPCHK(hipStreamSynchronize(sl.nstream));
        for (auto &q : m.q)
            if (q) HIPCHK(hipFree(q));
        for (auto &q : m.q) HIPCHK(hipMalloc(&q, (size_t)q_cap * sizeof(nice::MsdNode)));
        m.q_cap = q_cap;
    }
    if (m.leaf_cap < leaf_cap) {
        HIPCHK(hipStreamSynchronize(sl.nstream));
        if (m.leaves) HIPCHK(hipFree(m.leaves));
        HIPCHK(hipMalloc(&m.leaves, (size_t)leaf_cap * sizeof(nice::Leaf)));
        m.leaf_cap = leaf_cap;
    }
    return NICE_OK;
}

int slot_init(Device &d, Slot &sl, const Slot *share) {
    if (share && (shared_streams() & 1)) {
        sl.stream = share->stream;
    } else {
        HIPCHK(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
        sl.own_stream = true;
    }
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    if (nice::probe_set("NICE_NICE_PRIO") && nice::probe_knob("NICE_NICE_PRIO", 1) == 0) greatest = least;
    if (share && (shared_streams() & 2)) {
        sl.nstream = share->nstream;
    } else {
        HIPCHK(hipStreamCreateWithPriority(&sl.nstream, hipStreamNonBlocking, greatest));
        sl.own_nstream = true;
    }
    HIPCHK(hipMalloc(&sl.d_nice_count, 4));
    // hist bins and list counters in one block: one memset per field at most.
    HIPCHK(hipMalloc(&sl.d_state, kStateBytes));
    sl.d_count = (uint32_t *)(sl.d_state + kHistCopies * 129);
    sl.d_done = sl.d_count + 1;
    HIPCHK(hipHostMalloc(&sl.h_fin, kFinWords * 8, hipHostMallocMapped | hipHostMallocCoherent));
    memset(sl.h_fin, 0, kFinWords * 8);
    HIPCHK(hipHostGetDevicePointer((void **)&sl.d_fin, sl.h_fin, 0));
    HIPCHK(hipHostMalloc(&sl.h_msd, 32 * 4, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&sl.d_msd_mapped, sl.h_msd, 0));
    HIPCHK(hipHostMalloc(&sl.h_nice, 4, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&sl.d_nice_mapped, sl.h_nice, 0));
    HIPCHK(hipMalloc(&sl.d_nice_done, kDoneWords * 4));
    HIPCHK(hipMemset(sl.d_nice_done, 0, kDoneWords * 4));
    HIPCHK(hipEventCreate(&sl.ev0));
    HIPCHK(hipEventCreate(&sl.ev1));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.nice_done, hipEventDisableTiming));
    HIPCHK(hipEventCreate(&sl.nt0));
    HIPCHK(hipEventCreate(&sl.nt1));
    int rc = ensure_listbuf(d, sl.det, kInitialListCap, true);
    if (!rc) rc = ensure_listbuf(d, sl.nice, kNiceCap, false);
    return rc;
}

int device_init(Device &d, int id) {
    d.id = id;
    HIPCHK(hipSetDevice(id));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, id));
    d.num_cus = prop.multiProcessorCount;
    for (int i = 0; i < kSlots; i++) {
        int rc = slot_init(d, d.slot[i], i ? &d.slot[0] : nullptr);
        if (rc) return rc;
    }
    return NICE_OK;
}

void device_free(Device &d) {
    if (!d.slot[0].stream) return;
    (void)hipSetDevice(d.id);
    if (d.aux) (void)hipStreamSynchronize(d.aux);
    for (auto &sl : d.slot) {
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
        if (sl.nstream) (void)hipStreamSynchronize(sl.nstream);
    }
    for (auto &kv : d.residues) (void)hipFree(kv.second);
    for (auto &kv : d.ranks) (void)hipFree(kv.second);
    for (auto &b : d.desc) {
        if (b.h) {
            (void)hipHostFree(b.h);
            (void)hipFree(b.d);
        }
        if (b.done) (void)hipEventDestroy(b.done);
    }
    for (auto &sl : d.slot) {
        for (auto &q : sl.msd.q)
            if (q) (void)hipFree(q);
        if (sl.msd.leaves) (void)hipFree(sl.msd.leaves);
        if (sl.msd.counters) (void)hipFree(sl.msd.counters);
        if (sl.msd.scratch) (void)hipFree(sl.msd.scratch);
        if (sl.stream && sl.own_stream) (void)hipStreamDestroy(sl.stream);
        if (sl.nstream && sl.own_nstream) (void)hipStreamDestroy(sl.nstream);
        if (sl.d_nice_count) (void)hipFree(sl.d_nice_count);
        if (sl.d_nice_done) (void)hipFree(sl.d_nice_done);
        if (sl.d_state) (void)hipFree(sl.d_state);
        for (ListBuf *l : {&sl.det, &sl.nice}) {
            if (l->n) (void)hipFree(l->n);
            if (l->u) (void)hipFree(l->u);
        }
        if (sl.h_fin) (void)hipHostFree(sl.h_fin);
        if (sl.h_msd) (void)hipHostFree(sl.h_msd);
        if (sl.h_nice) (void)hipHostFree(sl.h_nice);
        for (hipEvent_t ev : {sl.ev0, sl.ev1, sl.ev_done, sl.nice_done, sl.nt0, sl.nt1})
            if (ev) (void)hipEventDestroy(ev);
    }
    if (d.chk_n) (void)hipFree(d.chk_n);
    if (d.chk_u) (void)hipFree(d.chk_u);
    if (d.aux) (void)hipStreamDestroy(d.aux);
    for (auto &sl : d.slot) sl.stream = nullptr;
}

int emit_list(std::vector<Entry> &all, nice_number *out, size_t cap, size_t *n_out) {
    std::sort(all.begin(), all.end(), [](const Entry &a, const Entry &b) { return a.n < b.n; });
    if (n_out) *n_out = all.size();
    const size_t c = std::min(cap, all.size());
    for (size_t i = 0; i < c; i++) {
        out[i].number_lo = lo64(all[i].n);
        out[i].number_hi = hi64(all[i].n);
        out[i].num_uniques = all[i].u;
        out[i].reserved = 0;
    }
    if (all.size() > cap)
        return fail(NICE_ERR_CAPACITY, "output list needs " + std::to_string(all.size()) +
                                           " entries, capacity " + std::to_string(cap));
    return NICE_OK;
}

// The server's submit invariants for a detailed result (api/src/main.rs:
// 309-359): the distribution sums to the field size; for every bin above the
// near-miss cutoff the count equals the number of listed numbers with that
// unique count; the list holds exactly the numbers above the cutoff.  (The
// server's last check, recomputing each listed number, runs on the device in
// nice_process_range_detailed.)  get(i) -> {n, u} of list entry i.
template <class Get>
int validate_detailed(uint32_t base, u128 size, const uint64_t *hist, size_t n, Get get) {
    u128 sum = 0;
    for (uint32_t b = 0; b <= base; b++) sum += hist[b];
    if (sum != size)
        return fail(NICE_ERR_HIP, "self-check: distribution total does not equal the field size");
    const uint32_t cutoff = nice::near_miss_cutoff(base);
    std::vector<uint64_t> per(base + 1, 0);
    for (size_t i = 0; i < n; i++) {
        const uint32_t u = get(i).u;
        if (u <= cutoff || u > base)
            return fail(NICE_ERR_HIP, "self-check: listed number " + std::to_string(i) +
                                          " has num_uniques " + std::to_string(u) +
                                          " at or below the cutoff");
        per[u]++;
    }
    u128 above = 0;
    for (uint32_t u = cutoff + 1; u <= base; u++) {
        if (per[u] != hist[u])
            return fail(NICE_ERR_HIP, "self-check: " + std::to_string(per[u]) +
                                          " listed numbers with " + std::to_string(u) +
                                          " uniques, distribution claims " + std::to_string(hist[u]));
        above += hist[u];
    }
    if (above != (u128)n) return fail(NICE_ERR_HIP, "self-check: list length does not match the distribution");
    return NICE_OK;
}

// Enqueue the detailed kernels for [s, e) on one device (async).
// Enqueue the detailed kernels for [s, e) on one device (async): generic
// kernel outside the base's valid range, FD kernel inside.  Returns in
// *finished whether the last launch also finished the field (fd2's in-kernel
// finish into the slot's mapped result words); otherwise the caller enqueues
// the epilogue kernel.
int enqueue_detailed(Device &d, Slot &sl, u128 s, u128 e, uint32_t base, bool *finished) {
    nice::DetailedLaunch p{};
    p.base = base;
    p.cutoff = nice::near_miss_cutoff(base);
    p.hist = sl.d_state;
    p.out = nice::NumOut{sl.det.n, sl.det.u, sl.d_count, sl.det.cap};
    p.launches = &sl.launches;
    p.sib = sl.sib;
    // Another detailed field of this device submitted and not yet collected:
    // the caller pipelines, so this field's launches are shaped for throughput
    // (launch_sib).  Whether that field is still running does not matter --
    // fields on the slot streams progress together and often finish
    // together, and a pick that followed their completion flipped every third
    // 2.5e8 field to the lone-field stride (8 % slower per step,
    // profiles/r06/stride/probe_pick.log).
    for (const Slot &o : d.slot)
        if (&o != &sl && o.inflight) p.overlapped = 1;
    *finished = false;
    // Small fields run wholly by fd2 publish tagged result words
    // (FieldFinish::tag): one fewer round trip to host memory at their end.
    uint32_t tag = 0;
    auto launch = [&](u128 a, u128 b, bool fd) -> int {
        if (a >= b) return NICE_OK;
        u128 cnt = b - a;
        while (cnt) {  // segments longer than 2^63 are split (count is u64)
            uint64_t c = cnt > ((u128)1 << 62) ? (1ull << 62) : (uint64_t)cnt;
            p.start_lo = lo64(a);
            p.start_hi = hi64(a);
            p.count = c;
            // the field's last launch finishes it when it is an fd2 launch
            const bool last = a + c == e;
            p.fin = last && fd ? nice::FieldFinish{sl.d_fin, sl.d_done, sl.seq, tag}
                               : nice::FieldFinish{nullptr, nullptr, 0, 0};
            if (nice::probe_set("NICE_FD2_NOFIN")) p.fin = nice::FieldFinish{nullptr, nullptr, 0, 0};  // probe: finish kernel
            const bool fd2 = fd;
            hipError_t err = fd ? nice::launch_detailed_fd2(p, d.num_cus, sl.stream)
                                : nice::launch_detailed_generic(p, d.num_cus, sl.stream);
            if (!fd) sl.launches++;
            if (err != hipSuccess)
                return fail(NICE_ERR_HIP, std::string("detailed launch: ") + hipGetErrorString(err));
            if (last) {
                *finished = fd2 && p.fin.out_mapped;
                sl.tag = *finished ? p.fin.tag : 0u;
                sl.tag_words = base + 1;
            }
            a += c;
            cnt -= c;
        }
        return NICE_OK;
    };
    u128 rs = 0, re = 0;
    const bool fd_base = nice::fd2_supported(base);
    const bool fd = fd_base && nice::base_range_cached(base, rs, re) == 1;
    // Histogram copies the field's launches flush into: a small field run
    // wholly by fd2 keeps 16 (its whole grid flushes at once, and the
    // in-kernel finish reads every copy in use); anything else all 64 (the
    // generic kernel and the finish kernel use all of them).
    const bool small_fd = fd && s >= rs && e <= re && e - s < 20000000;
    p.hist_copies = small_fd ? 16 : nice::kHistCopies;
    // (probe: NICE_FD2_UNTAGGED publishes bins + sequence word as large fields do)
    if (small_fd && !nice::probe_set("NICE_FD2_UNTAGGED")) tag = (uint32_t)sl.seq | 0x80000000u;
    sl.tag = 0;
    if (!fd) return launch(s, e, false);
    int rc;
    if ((rc = launch(s, std::min(e, rs), false))) return rc;
    if ((rc = launch(std::max(s, rs), std::min(e, re), true))) return rc;
    return launch(std::max(s, re), e, false);
}

// The event after a detailed field's last launch: the finish kernel's
// (ev_done) when the field needed one; else the kernel end (ev1) of a timed
// field, the end marker (ev_done) of an untimed one on a shared stream, or
// none: an untimed field that fd2 finishes in-kernel on its slot's own stream
// records no event at all (two fewer runtime calls per field), and the stream
// itself reports its completion.
inline hipEvent_t done_event(const Slot &sl) {
    if (!sl.fin_seq) return sl.ev_done;
    return sl.timed ? sl.ev1 : (sl.marked ? sl.ev_done : nullptr);
}

// Polls spin for the first kSpinPolls (a small field ends within tens of
// microseconds, and a sleeping waiter would add its wake-up latency), then
// yield the core between polls for kYieldPolls more, then sleep between
// polls, 20 us doubling to 200 us: a multi-second field (a split-launch
// detailed field, the massive niceonly field) must not keep a core busy per
// waiting thread beside the host MSD pool.  The sleep adds at most 200 us to
// fields that run for milliseconds.
constexpr uint32_t kSpinPolls = 1u << 14, kYieldPolls = 1u << 11;

inline void backoff(uint32_t i) {
    if (i < kSpinPolls) {
        __builtin_ia32_pause();
    } else if (i < kSpinPolls + kYieldPolls) {
        sched_yield();
    } else {
        const uint32_t k = std::min<uint32_t>((i - kSpinPolls - kYieldPolls) / 8, 3);
        std::this_thread::sleep_for(std::chrono::microseconds(std::min(200u, 20u << (2 * k))));
    }
}

// Wait for an event by polling it (see backoff).
hipError_t sync_event(hipEvent_t ev) {
    for (uint32_t i = 0;; i++) {
        const hipError_t q = hipEventQuery(ev);
        if (q != hipErrorNotReady) return q;
        backoff(i);
    }
}

// A detailed field's completion: its end event, or its slot's own stream
// when it recorded none (done_event).
hipError_t field_query(const Slot &sl) {
    const hipEvent_t ev = done_event(sl);
    return ev ? hipEventQuery(ev) : hipStreamQuery(sl.stream);
}

hipError_t field_sync(const Slot &sl) {
    for (uint32_t i = 0;; i++) {
        const hipError_t q = field_query(sl);
        if (q != hipErrorNotReady) return q;
        backoff(i);
    }
}

// The kernel time of the device's last collected field, read from its slot's
// events on demand (collect returns as soon as the results are published,
// possibly before the end-of-kernel event has completed).
int resolve_stats(Device &d) {
    if (d.stats_slot < 0) return NICE_OK;
    Slot &sl = d.slot[d.stats_slot];
    d.stats_slot = -1;
    HIPCHK(hipSetDevice(d.id));
    HIPCHK(field_sync(sl));
    float ms = 0;
    if (sl.timed) HIPCHK(hipEventElapsedTime(&ms, sl.ev0, sl.ev1));
    d.last.kernel_ms = ms;
    return NICE_OK;
}

// Wait until the detailed field in slot `sl` is finished.  A field ending in
// fd2's in-kernel finish is waited for by polling the sequence word that
// finish publishes in mapped memory -- microseconds sooner than the kernel's
// completion signal (which still follows: the last workgroup retires after
// publishing).  The completion event is queried every 4096 polls, so a failed
// launch or a finish that never publishes is reported, not spun on.
// A field's published result words: its sequence word, or (tagged fields)
// every bin word and the near-miss count carrying the field's tag.
bool published(const Slot &sl) {
    if (!sl.tag) return __atomic_load_n(&sl.h_fin[130], __ATOMIC_ACQUIRE) == sl.seq;
    if ((uint32_t)(__atomic_load_n(&sl.h_fin[129], __ATOMIC_ACQUIRE) >> 32) != sl.tag) return false;
    for (uint32_t b = 0; b < sl.tag_words; b++)
        if ((uint32_t)(__atomic_load_n(&sl.h_fin[b], __ATOMIC_ACQUIRE) >> 32) != sl.tag) return false;
    return true;
}

int wait_field(Slot &sl) {
    if (!sl.fin_seq || !spin_wait()) {
        const hipError_t q = field_sync(sl);
        if (q != hipSuccess) return fail(NICE_ERR_HIP, std::string("detailed field: ") + hipGetErrorString(q));
        return NICE_OK;
    }
    for (uint32_t i = 1;; i++) {
        if (published(sl)) return NICE_OK;
        if ((i & 4095) == 0 || i > kSpinPolls) {
            const hipError_t q = field_query(sl);
            if (q == hipSuccess) {
                if (published(sl)) return NICE_OK;
                return fail(NICE_ERR_HIP, "detailed field completed without publishing its results");
            }
            if (q != hipErrorNotReady) return fail(NICE_ERR_HIP, std::string("detailed field: ") + hipGetErrorString(q));
        }
        backoff(i);
    }
}

// Enqueue one device's shard of a detailed field into slot `sl` (async).
int enqueue_detailed_shard(Device &d, Slot &sl, u128 s, u128 e, uint32_t base, bool timing) {
    HIPCHK(hipSetDevice(d.id));
    // this slot's events are about to be re-recorded
    if (d.stats_slot == (int)(&sl - d.slot)) {
        int rc = resolve_stats(d);
        if (rc) return rc;
    }
    sl.seq++;
    sl.launches = 0;
    sl.sib[0] = sl.sib[1] = 0;
    // The state block is zeroed by the previous field's finish; a memset
    // only after an interrupted field (or the first one).
    if (sl.dirty) HIPCHK(hipMemsetAsync(sl.d_state, 0, kStateBytes, sl.stream));
    sl.dirty = true;
    sl.timed = timing;
    sl.marked = false;
    if (timing) HIPCHK(hipEventRecord(sl.ev0, sl.stream));
    bool finished = false;
    int rc = enqueue_detailed(d, sl, s, e, base, &finished);
    if (rc) return rc;
    sl.inflight = true;
    if (timing) HIPCHK(hipEventRecord(sl.ev1, sl.stream));
    sl.fin_seq = finished;
    if (!finished) {
        HIPCHK(nice::launch_detailed_finish(sl.d_state, sl.d_count, sl.d_fin, sl.stream));
        HIPCHK(hipEventRecord(sl.ev_done, sl.stream));
    } else if (!timing && !sl.own_stream) {
        // a stream shared between slots (probe build) cannot tell this
        // field's completion from a later one's: mark its end
        HIPCHK(hipEventRecord(sl.ev_done, sl.stream));
        sl.marked = true;
    }
    return NICE_OK;
}

int detailed_submit(nice_ctx *ctx, std::unique_lock<std::mutex> &lock, u128 s, u128 e, uint32_t base,
                    bool wait, int *ticket) {
    int t = -1;
    if (int rc = acquire_slot(ctx, lock, ctx->det, ctx->det_next, wait, "detailed", &t)) return rc;
    DetJob &job = ctx->det[t];
    const size_t nd = ctx->devs.size();
    const u128 size = e - s;
    // Shard bounds: contiguous, in device order (ascending n).
    job.bounds.assign(nd + 1, 0);
    for (size_t i = 0; i <= nd; i++) job.bounds[i] = s + size / nd * i + std::min<u128>(i, size % nd);
    for (size_t i = 0; i < nd; i++) {
        if (job.bounds[i] >= job.bounds[i + 1]) continue;
        int rc = enqueue_detailed_shard(ctx->devs[i], ctx->devs[i].slot[t], job.bounds[i], job.bounds[i + 1], base,
                                        ctx->timing);
        if (rc) return rc;
    }
    job.active = true;
    job.collected = false;
    job.owner = std::this_thread::get_id();
    job.s = s;
    job.e = e;
    job.base = base;
    ctx->det_next = (t + 1) % slots_used();
    *ticket = t;
    return NICE_OK;
}

// Wait for a submitted detailed field, merge the devices' results into the
// job and self-check them (the server's submit invariants).
int detailed_gather(nice_ctx *ctx, DetJob &job, int t) {
    const uint32_t base = job.base;
    const size_t nd = ctx->devs.size();
    job.total.assign(base + 1, 0);
    job.all.clear();
    std::vector<size_t> off(nd + 1, 0);  // device i's list entries: job.all[off[i], off[i + 1])
    for (size_t i = 0; i < nd; i++) {
        off[i] = job.all.size();
        Device &d = ctx->devs[i];
        Slot &sl = d.slot[t];
        d.last = nice_kernel_stats{};
        d.stats_slot = -1;
        if (job.bounds[i] >= job.bounds[i + 1]) continue;
        HIPCHK(hipSetDevice(d.id));
        int rc = wait_field(sl);
        if (rc) return rc;
        sl.dirty = false;  // the epilogue zeroed the state block
        sl.inflight = false;
        d.stats_slot = t;  // kernel_ms read on demand (resolve_stats)
        d.last.numbers = (uint64_t)(job.bounds[i + 1] - job.bounds[i]);
        d.last.launches = sl.launches;
        d.last.fd_kernel = nice::fd2_supported(base) ? 1u : 0u;
        d.last.sib_lanes = sl.sib[0];
        d.last.sib_stride = sl.sib[1];
        uint32_t cnt = (uint32_t)sl.h_fin[129];
        if (cnt > sl.det.cap) {
            // Near-miss list overflowed (e.g. out-of-range n, SURVEY hazard 9):
            // grow to the exact count and redo this shard (behind any field
            // queued after it; only this slot's completion is awaited).
            rc = ensure_listbuf(d, sl.det, cnt, true);
            if (!rc) rc = enqueue_detailed_shard(d, sl, job.bounds[i], job.bounds[i + 1], base, sl.timed);
            if (!rc) rc = wait_field(sl);
            if (rc) return rc;
            sl.dirty = false;
            sl.inflight = false;
            d.stats_slot = t;
            d.last.launches = sl.launches;
            d.last.sib_lanes = sl.sib[0];
            d.last.sib_stride = sl.sib[1];
            cnt = (uint32_t)sl.h_fin[129];
            if (cnt > sl.det.cap) return fail(NICE_ERR_HIP, "near-miss list overflow after resize");
        }
        for (uint32_t b = 0; b <= base; b++) job.total[b] += sl.tag ? (uint32_t)sl.h_fin[b] : sl.h_fin[b];
        if (cnt) {
            // the list is read after the kernel has retired (its end-of-kernel
            // cache write-back), not merely published its count
            HIPCHK(field_sync(sl));
            std::vector<uint64_t> nbuf((size_t)cnt * 2);
            std::vector<uint32_t> ubuf(cnt);
            HIPCHK(hipMemcpy(nbuf.data(), sl.det.n, (size_t)cnt * 16, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ubuf.data(), sl.det.u, (size_t)cnt * 4, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < cnt; q++) job.all.push_back({mk(nbuf[2 * q], nbuf[2 * q + 1]), ubuf[q]});
        }
    }
    off[nd] = job.all.size();
    // Self-check: the server's submit invariants (api/src/main.rs:309-359)
    // before anything is returned.
    int rc = validate_detailed(base, job.e - job.s, job.total.data(), job.all.size(),
                               [&](size_t i) { return job.all[i]; });
    if (rc) return rc;
    if (!job.all.empty()) {
        // ... and its last one: every listed number's unique count recomputed
        // by the generic per-n device function (full square / cube + digit
        // scan, a different code path from the FD kernel that listed it).
        // Each device recomputes its own shard's entries on its auxiliary
        // stream (so no queued field is waited for), all devices at once.
        std::vector<std::vector<uint32_t>> u(nd);
        std::vector<std::vector<uint64_t>> pairs(nd);
        // Devices whose aux stream still has copies from / into pairs and u:
        // any return drains them first (declared after the buffers, so it
        // runs before they are freed).
        struct Drain {
            nice_ctx *ctx;
            std::vector<char> q;
            ~Drain() {
                for (size_t j = 0; j < q.size(); j++)
                    if (q[j]) {
                        (void)hipSetDevice(ctx->devs[j].id);
                        (void)hipStreamSynchronize(ctx->devs[j].aux);
                    }
            }
        } drain{ctx, std::vector<char>(nd, 0)};
        for (size_t i = 0; i < nd; i++) {
            const size_t n = off[i + 1] - off[i];
            if (!n) continue;
            Device &d = ctx->devs[i];
            HIPCHK(hipSetDevice(d.id));
            // created on first use: an idle stream would still take one of the
            // process's few hardware queues (GPU_MAX_HW_QUEUES)
            if (!d.aux) HIPCHK(hipStreamCreateWithFlags(&d.aux, hipStreamNonBlocking));
            pairs[i].resize(2 * n);
            for (size_t q = 0; q < n; q++) {
                pairs[i][2 * q] = lo64(job.all[off[i] + q].n);
                pairs[i][2 * q + 1] = hi64(job.all[off[i] + q].n);
            }
            if (d.chk_cap < n) {
                // grown rarely (the recompute of the previous field finished
                // before its collect returned, so nothing reads the old buffers)
                if (d.chk_n) HIPCHK(hipFree(d.chk_n));
                if (d.chk_u) HIPCHK(hipFree(d.chk_u));
                d.chk_n = nullptr;
                d.chk_u = nullptr;
                d.chk_cap = 0;
                const size_t c = std::max<size_t>(n, 4096);
                HIPCHK(hipMalloc(&d.chk_n, c * 16));
                HIPCHK(hipMalloc(&d.chk_u, c * 4));
                d.chk_cap = c;
            }
            u[i].resize(n);
            drain.q[i] = 1;
            hipError_t err = hipMemcpyAsync(d.chk_n, pairs[i].data(), n * 16, hipMemcpyHostToDevice, d.aux);
            if (err == hipSuccess) err = nice::launch_unique_counts(d.chk_n, (uint32_t)n, base, d.chk_u, d.aux);
            if (err == hipSuccess) err = hipMemcpyAsync(u[i].data(), d.chk_u, n * 4, hipMemcpyDeviceToHost, d.aux);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("self-check: ") + hipGetErrorString(err));
        }
        for (size_t i = 0; i < nd; i++) {
            if (u[i].empty()) continue;
            Device &d = ctx->devs[i];
            HIPCHK(hipSetDevice(d.id));
            const hipError_t err = hipStreamSynchronize(d.aux);
            drain.q[i] = 0;
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("self-check: ") + hipGetErrorString(err));
            for (size_t q = 0; q < u[i].size(); q++)
                if (u[i][q] != job.all[off[i] + q].u)
                    return fail(NICE_ERR_HIP, "self-check: unique count of a listed number does not recompute");
        }
    }
    std::sort(job.all.begin(), job.all.end(), [](const Entry &a, const Entry &b) { return a.n < b.n; });
    return NICE_OK;
}

int detailed_collect(nice_ctx *ctx, int t, uint64_t *hist, nice_number *out, size_t cap, size_t *n_out) {
    if (t < 0 || t >= kSlots || !ctx->det[t].active)
        return fail(NICE_ERR_INVALID, "no detailed field in flight under this ticket");
    DetJob &job = ctx->det[t];
    if (!job.collected) {
        int rc = detailed_gather(ctx, job, t);
        if (rc) {
            job.active = false;  // the field is lost; its slot is reusable
            for (auto &d : ctx->devs) d.slot[t].dirty = true, d.slot[t].inflight = false;
            return rc;
        }
        job.collected = true;
    }
    std::memcpy(hist, job.total.data(), (job.base + 1) * 8);
    int rc = emit_list(job.all, out, cap, n_out);
    if (rc == NICE_ERR_CAPACITY) return rc;  // kept: the caller retries with room
    job.active = false;
    job.all = {};
    return rc;
}

}  // namespace

// The CPU path (cpu_path.cpp) reports through the same thread-local message.
namespace nice {
void set_last_error(const char *msg) { g_err = msg; }
}  // namespace nice

extern "C" {

const char *nice_last_error(void) { return g_err.c_str(); }

int nice_device_count(int *out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return NICE_OK;
}

int nice_ctx_create(const int *devices, int n_devices, nice_ctx **out) {
    if (!out) return fail(NICE_ERR_INVALID, "null out");
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have < 1)
        return fail(NICE_ERR_NO_DEVICE, "no HIP device visible");
    std::unique_ptr<nice_ctx> ctx(new nice_ctx());
    std::vector<int> ids;
    if (!devices || n_devices <= 0) ids.push_back(0);
    else ids.assign(devices, devices + n_devices);
    ctx->devs.resize(ids.size());
    for (size_t i = 0; i < ids.size(); i++) {
        if (ids[i] < 0 || ids[i] >= have)
            return fail(NICE_ERR_INVALID, "device ordinal " + std::to_string(ids[i]) + " out of range");
        int rc = device_init(ctx->devs[i], ids[i]);
        if (rc) {
            for (auto &d : ctx->devs) device_free(d);
            return rc;
        }
    }
    *out = ctx.release();
    return NICE_OK;
}

int nice_ctx_synchronize(nice_ctx *ctx) {
    if (!ctx) return fail(NICE_ERR_INVALID, "null ctx");
    std::lock_guard<std::mutex> lock(ctx->mu);
    for (auto &d : ctx->devs) {
        HIPCHK(hipSetDevice(d.id));
        for (auto &sl : d.slot) {
            HIPCHK(hipStreamSynchronize(sl.stream));
            HIPCHK(hipStreamSynchronize(sl.nstream));
        }
        if (d.aux) HIPCHK(hipStreamSynchronize(d.aux));
    }
    return NICE_OK;
}

void nice_ctx_destroy(nice_ctx *ctx) {
    if (!ctx) return;
    for (auto &d : ctx->devs) device_free(d);
    delete ctx;
}

int nice_base_range(uint32_t base, uint64_t *slo, uint64_t *shi, uint64_t *elo, uint64_t *ehi) {
    u128 s = 0, e = 0;
    int rc = nice::base_range_cached(base, s, e);
    if (rc == 1) {
        *slo = lo64(s);
        *shi = hi64(s);
        *elo = lo64(e);
        *ehi = hi64(e);
    }
    return rc;
}

uint32_t nice_near_miss_cutoff(uint32_t base) { return nice::near_miss_cutoff(base); }
uint64_t nice_gpu_batch_size(void) { return 50000000ull; }
uint64_t nice_processing_chunk_size(void) { return 1000000ull; }
int nice_gpu_supports_base(uint32_t base) { return base >= 2 && base <= 128; }
int nice_fd_kernel_base(uint32_t base) { return nice::fd2_supported(base) ? 1 : 0; }

int nice_ctx_set_kernel_timing(nice_ctx *ctx, int enable) {
    if (!ctx) return fail(NICE_ERR_INVALID, "null ctx");
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->timing = enable != 0;
    return NICE_OK;
}

int nice_last_kernel_stats(nice_ctx *ctx, int i, nice_kernel_stats *out) {
    if (!ctx || i < 0 || i >= (int)ctx->devs.size() || !out) return fail(NICE_ERR_INVALID, "bad args");
    // (under the context lock: a collect on another thread updates the
    // device's last-field record)
    std::lock_guard<std::mutex> lock(ctx->mu);
    int rc = resolve_stats(ctx->devs[i]);
    if (rc) return rc;
    *out = ctx->devs[i].last;
    return NICE_OK;
}

}  // extern "C"

namespace {

int detailed_submit_args(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo, uint64_t end_hi,
                         uint32_t base, bool wait, int *ticket) {
    if (!ctx || !ticket) return fail(NICE_ERR_INVALID, "null argument");
    if (base < 2 || base > 128) return fail(NICE_ERR_INVALID, "base must be in 2..=128");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (s >= e)
        return fail(NICE_ERR_INVALID, "Range has invalid bounds, range_start must be < range_end");
    std::unique_lock<std::mutex> lock(ctx->mu);
    return detailed_submit(ctx, lock, s, e, base, wait, ticket);
}

int detailed_collect_locked(nice_ctx *ctx, int ticket, uint64_t *hist, nice_number *out, size_t cap,
                            size_t *n_out);

}  // namespace

extern "C" {

int nice_process_range_detailed(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base, uint64_t *hist,
                                nice_number *out, size_t cap, size_t *n_out) {
    int t = -1;
    int rc = detailed_submit_args(ctx, start_lo, start_hi, end_lo, end_hi, base, true, &t);
    if (rc) return rc;
    rc = nice_detailed_collect(ctx, t, hist, out, cap, n_out);
    if (rc == NICE_ERR_CAPACITY) {
        // synchronous call: the caller retries the whole field with room
        {
            std::lock_guard<std::mutex> lock(ctx->mu);
            ctx->det[t].active = false;
            ctx->det[t].all = {};
        }
        ctx->freed.notify_all();
    }
    return rc;
}

int nice_detailed_submit(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                         uint64_t end_hi, uint32_t base, int *ticket) {
    return detailed_submit_args(ctx, start_lo, start_hi, end_lo, end_hi, base, false, ticket);
}

int nice_detailed_collect(nice_ctx *ctx, int ticket, uint64_t *hist, nice_number *out, size_t cap,
                          size_t *n_out) {
    if (!ctx || !hist) return fail(NICE_ERR_INVALID, "null argument");
    const int rc = detailed_collect_locked(ctx, ticket, hist, out, cap, n_out);
    ctx->freed.notify_all();  // the ticket's slot may be free now
    return rc;
}

}  // extern "C"

namespace {

int detailed_collect_locked(nice_ctx *ctx, int ticket, uint64_t *hist, nice_number *out, size_t cap,
                            size_t *n_out) {
    std::unique_lock<std::mutex> lock(ctx->mu);
    if (ticket < 0 || ticket >= kSlots || !ctx->det[ticket].active)
        return fail(NICE_ERR_INVALID, "no detailed field in flight under this ticket");
    DetJob &job = ctx->det[ticket];
    if (job.waiting) return fail(NICE_ERR_INVALID, "another thread is collecting this detailed field");
    if (!job.collected) {
        // Wait for every device's shard to publish WITHOUT the context lock,
        // so other threads can submit and collect other fields meanwhile (the
        // slot stays reserved: the job is active).  The gather below then
        // finds them finished.
        job.waiting = true;
        lock.unlock();
        int rc = NICE_OK;
        for (size_t i = 0; i < ctx->devs.size() && !rc; i++) {
            if (job.bounds[i] >= job.bounds[i + 1]) continue;
            const hipError_t err = hipSetDevice(ctx->devs[i].id);
            rc = err != hipSuccess ? fail(NICE_ERR_HIP, hipGetErrorString(err)) : wait_field(ctx->devs[i].slot[ticket]);
        }
        lock.lock();
        job.waiting = false;
        if (rc) {
            job.active = false;
            for (auto &d : ctx->devs) d.slot[ticket].dirty = true, d.slot[ticket].inflight = false;
            return rc;
        }
    }
    return detailed_collect(ctx, ticket, hist, out, cap, n_out);
}

}  // namespace

extern "C" {

int nice_validate_detailed(uint32_t base, uint64_t size_lo, uint64_t size_hi, const uint64_t *hist,
                           const nice_number *list, size_t n) {
    if (base < 2 || base > 128 || !hist || (n && !list)) return fail(NICE_ERR_INVALID, "bad args");
    const int rc = validate_detailed(base, mk(size_lo, size_hi), hist, n, [&](size_t i) {
        return Entry{mk(list[i].number_lo, list[i].number_hi), list[i].num_uniques};
    });
    return rc ? NICE_ERR_INVALID : NICE_OK;
}

int nice_debug_unique_counts(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count,
                             uint32_t base, uint32_t *out) {
    if (!ctx || base < 2 || base > 128) return fail(NICE_ERR_INVALID, "bad args");
    if (count == 0) return NICE_OK;
    Device &d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    uint64_t *dn;
    uint32_t *du;
    HIPCHK(hipMalloc(&dn, (size_t)count * 16));
    HIPCHK(hipMalloc(&du, (size_t)count * 4));
    HIPCHK(hipMemcpy(dn, n_pairs, (size_t)count * 16, hipMemcpyHostToDevice));
    HIPCHK(nice::launch_unique_counts(dn, count, base, du, d.slot[0].stream));
    HIPCHK(hipStreamSynchronize(d.slot[0].stream));
    HIPCHK(hipMemcpy(out, du, (size_t)count * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dn));
    HIPCHK(hipFree(du));
    return NICE_OK;
}

int nice_debug_is_nice(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count, uint32_t base,
                       uint32_t *out) {
    if (!ctx || base < 2 || base > 128) return fail(NICE_ERR_INVALID, "bad args");
    if (count == 0) return NICE_OK;
    Device &d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    uint64_t *dn;
    uint32_t *du;
    HIPCHK(hipMalloc(&dn, (size_t)count * 16));
    HIPCHK(hipMalloc(&du, (size_t)count * 4));
    HIPCHK(hipMemcpy(dn, n_pairs, (size_t)count * 16, hipMemcpyHostToDevice));
    HIPCHK(nice::launch_is_nice(dn, count, base, du, d.slot[0].stream));
    HIPCHK(hipStreamSynchronize(d.slot[0].stream));
    HIPCHK(hipMemcpy(out, du, (size_t)count * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dn));
    HIPCHK(hipFree(du));
    return NICE_OK;
}

// The bases with niceonly fast paths (niceonly.hip NICE_NICEONLY_BASES).
#define NICE_FAST_BASES(X) X(40) X(50) X(52) X(53) X(54) X(80)
static bool nice_fast_base(uint32_t base) {
    switch (base) {
#define X(b) case b:
        NICE_FAST_BASES(X)
#undef X
        return true;
    default: return false;
    }
}

int nice_debug_unique_fast(nice_ctx *ctx, const uint64_t *n_pairs, uint32_t count, uint32_t base,
                           uint32_t *out) {
    u128 rs, re;
    if (!ctx || !nice_fast_base(base) || nice::base_range_cached(base, rs, re) != 1)
        return fail(NICE_ERR_INVALID, "base without a niceonly fast path");
    for (uint32_t i = 0; i < count; i++) {
        const u128 n = mk(n_pairs[2 * i], n_pairs[2 * i + 1]);
        if (n < rs || n >= re) return fail(NICE_ERR_INVALID, "n outside the base's valid range");
    }
    if (count == 0) return NICE_OK;
    Device &d = ctx->devs[0];
    HIPCHK(hipSetDevice(d.id));
    uint64_t *dn;
    uint32_t *du;
    HIPCHK(hipMalloc(&dn, (size_t)count * 16));
    HIPCHK(hipMalloc(&du, (size_t)count * 4));
    HIPCHK(hipMemcpy(dn, n_pairs, (size_t)count * 16, hipMemcpyHostToDevice));
    HIPCHK(nice::launch_unique_fast(dn, count, base, du, d.slot[0].stream));
    HIPCHK(hipStreamSynchronize(d.slot[0].stream));
    HIPCHK(hipMemcpy(out, du, (size_t)count * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dn));
    HIPCHK(hipFree(du));
    return NICE_OK;
}

int nice_check_is_nice_inrange(uint32_t base, uint64_t lo, uint64_t hi) {
    u128 rs, re;
    const u128 n = mk(lo, hi);
    if (!nice_fast_base(base) || nice::base_range_cached(base, rs, re) != 1 || n < rs || n >= re)
        return fail(NICE_ERR_INVALID, "n outside the base's valid range (or base not 40/50/80)");
    switch (base) {
#define X(b) case b: return nice::is_nice_fast<b>(lo, hi) ? 1 : 0;
        NICE_FAST_BASES(X)
#undef X
    default: return NICE_ERR_INVALID;
    }
}

int nice_check_unique_inrange(uint32_t base, uint64_t lo, uint64_t hi) {
    u128 rs, re;
    const u128 n = mk(lo, hi);
    if (!nice_fast_base(base) || nice::base_range_cached(base, rs, re) != 1 || n < rs || n >= re)
        return fail(NICE_ERR_INVALID, "n outside the base's valid range (or base not 40/50/52/53/54/80)");
    switch (base) {
#define X(b) case b: return (int)nice::unique_fast<b>(lo, hi);
        NICE_FAST_BASES(X)
#undef X
    default: return NICE_ERR_INVALID;
    }
}

int nice_check_msd_skippable_inrange(uint32_t base, uint64_t slo, uint64_t shi, uint64_t elo,
                                     uint64_t ehi) {
    u128 rs, re;
    const u128 s = mk(slo, shi), e = mk(elo, ehi);
    if (!nice_fast_base(base) || nice::base_range_cached(base, rs, re) != 1 || s < rs || e > re || s >= e)
        return fail(NICE_ERR_INVALID, "range outside the base's valid range (or base not 40/50/80)");
    if (e - s == 1) return 0;  // a single number is never skipped (msd_prefix_filter.rs:395)
    const u128 l = e - 1;
    const uint64_t llo = lo64(l), lhi = hi64(l);
    switch (base) {
#define X(b) case b: return nice::msd_skippable_fast<b>(slo, shi, llo, lhi) ? 1 : 0;
        NICE_FAST_BASES(X)
#undef X
    default: return NICE_ERR_INVALID;
    }
}

int nice_fd_segment_cuts(uint32_t base, uint64_t *out, size_t cap, size_t *n_out) {
    std::vector<u128> c(8);
    const size_t n = nice::fd2_cuts(base, c.data(), c.size());
    for (size_t i = 0; i < n && i < cap; i++) {
        out[2 * i] = lo64(c[i]);
        out[2 * i + 1] = hi64(c[i]);
    }
    if (n_out) *n_out = n;
    return NICE_OK;
}

int nice_msd_skippable(uint64_t slo, uint64_t shi, uint64_t elo, uint64_t ehi, uint32_t base) {
    if (base < 2 || base > 128 || mk(slo, shi) >= mk(elo, ehi)) return fail(NICE_ERR_INVALID, "bad args");
    return nice::make_msd(base)->skippable(mk(slo, shi), mk(elo, ehi)) ? 1 : 0;
}

int nice_msd_valid_ranges(uint64_t slo, uint64_t shi, uint64_t elo, uint64_t ehi, uint32_t base,
                          uint64_t floor_size, uint64_t *out, size_t cap, size_t *n_out) {
    if (base < 2 || base > 128 || mk(slo, shi) >= mk(elo, ehi)) return fail(NICE_ERR_INVALID, "bad args");
    std::vector<std::pair<u128, u128>> rs;
    nice::make_msd(base)->ranges(mk(slo, shi), mk(elo, ehi), floor_size, rs);
    size_t n = rs.size();
    for (size_t i = 0; i < n && i < cap; i++) {
        out[4 * i] = lo64(rs[i].first);
        out[4 * i + 1] = hi64(rs[i].first);
        out[4 * i + 2] = lo64(rs[i].second);
        out[4 * i + 3] = hi64(rs[i].second);
    }
    *n_out = n;
    return n > cap ? fail(NICE_ERR_CAPACITY, "range list exceeds capacity") : NICE_OK;
}

int nice_stride_table(uint32_t base, uint32_t k, uint64_t *modulus, uint32_t *residues,
                      size_t cap, size_t *n_out) {
    if (base < 3 || base > 128 || k > 3) return fail(NICE_ERR_INVALID, "bad args");
    auto t = g_stride.get(base, k);
    *modulus = t->modulus;
    *n_out = t->residues.size();
    for (size_t i = 0; i < std::min(cap, t->residues.size()); i++) residues[i] = t->residues[i];
    return t->residues.size() > cap && residues ? fail(NICE_ERR_CAPACITY, "capacity") : NICE_OK;
}

// ---------------------------------------------------------------------------
// Niceonly: device MSD (level kernels) or a multi-threaded host MSD producer
// -> stride-index leaves -> the candidate kernel.
// ---------------------------------------------------------------------------

// NICE_GPU_MSD_FLOOR pins the reference GPU path's MSD floor
// (client_process_gpu.rs:161-172: parsed as f64, used when >= 1, otherwise
// ignored with a warning).  Read once, like the reference's OnceLock.
static uint64_t nbatches_of(uint64_t chunks, uint64_t per_batch) {
    return (chunks + per_batch - 1) / per_batch;
}

static uint64_t env_msd_floor() {
    static const uint64_t v = [] {
        const char *e = getenv("NICE_GPU_MSD_FLOOR");
        if (!e) return (uint64_t)0;
        char *end = nullptr;
        const double f = strtod(e, &end);
        if (end == e || *end != 0 || !(f >= 1.0) || f > 1e18) {
            fprintf(stderr, "nice: ignoring invalid NICE_GPU_MSD_FLOOR '%s'\n", e);
            return (uint64_t)0;
        }
        return (uint64_t)f;
    }();
    return v;
}

}  // extern "C"

// The reference GPU path's AdaptiveFloor (client_process_gpu.rs:96-184),
// selected by msd_floor = NICE_MSD_FLOOR_ADAPTIVE.  Process-wide, like the
// reference's OnceLock: NICE_GPU_MSD_FLOOR pins it (no adaptation); otherwise
// the seed is 512 000 / logical cores clamped to [250, 256 000], the first 3
// fields do not adapt, and after each host-MSD field the floor moves by
// msd / gpu_tail, clamped to [1/1.5, 1.5] (nice_adaptive_floor_step).
namespace {
constexpr double kFloorMin = 250.0, kFloorMax = 256000.0, kAdaptMaxStep = 1.5, kAdaptMinSecs = 0.002,
                 kAdaptBaseCoreProduct = 512000.0;
constexpr uint32_t kAdaptWarmup = 3, kAdaptPinned = 0xffffffffu;
struct AdaptiveFloor {
    double floor;
    uint32_t warmup;  // fields left before adapting; kAdaptPinned: fixed by the environment
};
std::mutex g_af_mu;

// CPUs a cgroup v2 cpu.max line grants: quota / period rounded DOWN (Rust's
// cgroups::quota_v2), 0 for "max" or an unreadable line.
unsigned cpu_max_cpus(const char *text) {
    char q[32] = {0};
    unsigned long period = 0;
    if (!text || sscanf(text, "%31s %lu", q, &period) != 2 || strcmp(q, "max") == 0 || period == 0) return 0;
    char *end = nullptr;
    const unsigned long quota = strtoul(q, &end, 10);
    if (end == q) return 0;
    const unsigned long c = quota / period;
    return c > 0xffffffffUL ? 0xffffffffu : (unsigned)c;
}
// The tightest cpu.max of the cgroup `rel` (a path below `root`) and of its
// ancestors up to root, as Rust walks them; 0 if none limits.
unsigned cgroup_cpus(const std::string &root, std::string rel) {
    unsigned best = 0;
    bool limited = false;
    for (;;) {
        while (!rel.empty() && rel.back() == '/') rel.pop_back();
        if (FILE *f = fopen((root + rel + "/cpu.max").c_str(), "r")) {
            char line[128] = {0};
            if (fgets(line, sizeof line, f)) {
                char q[32] = {0};
                if (sscanf(line, "%31s", q) == 1 && strcmp(q, "max") != 0) {
                    const unsigned c = cpu_max_cpus(line);
                    best = limited ? std::min(best, c) : c;
                    limited = true;
                }
            }
            fclose(f);
        }
        if (rel.empty()) break;
        const size_t p = rel.rfind('/');
        rel = p == std::string::npos ? std::string() : rel.substr(0, p);
    }
    return limited ? std::max(best, 1u) : 0u;
}
// std::thread::available_parallelism on Linux (library/std/src/sys/pal/unix/
// thread.rs): the affinity mask, capped by the cgroup v2 cpu.max quotas of
// the process's own cgroup (/proc/self/cgroup "0::<path>") and its ancestors
// under /sys/fs/cgroup, each quota / period rounded down, at least 1.
unsigned available_parallelism() {
    unsigned n = std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) n = (unsigned)CPU_COUNT(&set);
    std::string rel;
    if (FILE *f = fopen("/proc/self/cgroup", "r")) {
        char line[4096];
        while (fgets(line, sizeof line, f))
            if (strncmp(line, "0::", 3) == 0) {
                rel = line + 3;
                while (!rel.empty() && (rel.back() == '\n' || rel.back() == '\r')) rel.pop_back();
                break;
            }
        fclose(f);
    }
    const unsigned c = cgroup_cpus("/sys/fs/cgroup", rel);
    if (c >= 1 && c < n) n = c;
    return n ? n : 4;
}

AdaptiveFloor &adaptive_floor() {  // call under g_af_mu
    static AdaptiveFloor af = [] {
        if (const uint64_t pin = env_msd_floor()) return AdaptiveFloor{(double)pin, kAdaptPinned};
        const double seed = std::min(kFloorMax, std::max(kFloorMin, kAdaptBaseCoreProduct / available_parallelism()));
        return AdaptiveFloor{seed, kAdaptWarmup};
    }();
    return af;
}
}  // namespace

extern "C" {

double nice_adaptive_floor_step(double floor, double msd_seconds, double total_seconds) {
    const double gpu_tail = std::max(0.0, total_seconds - msd_seconds);
    const double ratio = gpu_tail < kAdaptMinSecs ? kAdaptMaxStep
                         : msd_seconds < kAdaptMinSecs ? 1.0 / kAdaptMaxStep
                                                       : msd_seconds / gpu_tail;
    const double factor = std::min(kAdaptMaxStep, std::max(1.0 / kAdaptMaxStep, ratio));
    return std::min(kFloorMax, std::max(kFloorMin, floor * factor));
}

uint32_t nice_host_threads(void) { return available_parallelism(); }

int nice_debug_force_sib_stride(uint32_t L) {
    if (L && (L % 2 == 0 || L > 255))
        return fail(NICE_ERR_INVALID, "sibling lane stride must be odd and <= 255 (0: the production pick)");
    nice::fd2_force_sib_stride(L);
    return NICE_OK;
}

uint32_t nice_debug_cgroup_cpus(const char *root, const char *cgroup_path) {
    return root ? cgroup_cpus(root, cgroup_path ? cgroup_path : "") : 0u;
}

int nice_adaptive_floor(double *floor, uint32_t *warmup) {
    std::lock_guard<std::mutex> g(g_af_mu);
    const AdaptiveFloor &af = adaptive_floor();
    if (floor) *floor = af.floor;
    if (warmup) *warmup = af.warmup;
    return NICE_OK;
}

}  // extern "C"

namespace {

// The floor a niceonly field's MSD recursion uses (resolved once per field:
// a re-run of the field keeps it).
uint64_t resolve_floor(const nice_niceonly_opts *opts) {
    uint64_t floor_size = opts && opts->msd_floor ? opts->msd_floor : env_msd_floor();
    if (opts && opts->msd_floor == NICE_MSD_FLOOR_ADAPTIVE) {
        std::lock_guard<std::mutex> g(g_af_mu);
        floor_size = (uint64_t)adaptive_floor().floor;  // gpu_msd_floor(), client_process_gpu.rs:559-561
    }
    return floor_size ? floor_size : 250;
}

// Enqueue niceonly field `job` (bounds, base, options and floor already set)
// into slot t of the context's devices.  Called under ctx->mu by submit, and
// again by collect when a device's nice list overflowed and was grown: the
// whole field re-runs (the reference CPU path returns a list of any length,
// client_process.rs:439-465; its GPU path bails at 2^16,
// client_process_gpu.rs:777-782).
int niceonly_enqueue(nice_ctx *ctx, int t, NiceJob &job) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    const u128 s = job.s, e = job.e;
    const uint32_t base = job.base;
    const nice_niceonly_opts *opts = job.has_opts ? &job.opts : nullptr;
    nice_niceonly_stats st{};
    const bool adaptive = opts && opts->msd_floor == NICE_MSD_FLOOR_ADAPTIVE;
    const uint64_t floor_size = job.st.msd_floor;
    st.msd_floor = floor_size;
    const uint32_t k = opts && opts->stride_k ? opts->stride_k : 2;
    // the reference sizes its MSD producer pool with available_parallelism()
    // (client_process_gpu.rs:598): on a 16-CPU cgroup of a 256-CPU host, 16
    int threads = opts && opts->threads > 0 ? opts->threads : (int)available_parallelism();
    if (threads < 1) threads = 1;
    const u128 chunk = opts && opts->chunk_size ? (u128)opts->chunk_size : nice::client_chunk_size(e - s);
    const uint64_t deal_stride = opts && opts->deal_stride ? opts->deal_stride : 1;
    const uint64_t deal_offset = opts ? opts->deal_offset : 0;
    if (deal_offset >= deal_stride) return fail(NICE_ERR_INVALID, "deal_offset must be < deal_stride");
    // This caller's chunks of the field's grid: c = deal_offset + i * deal_stride.
    const u128 nchunks_field = (e - s + chunk - 1) / chunk;
    const u128 mine128 = deal_offset < nchunks_field
                             ? (nchunks_field - deal_offset + deal_stride - 1) / deal_stride : 0;
    if (mine128 >> 63) return fail(NICE_ERR_INVALID, "too many MSD chunks");
    const uint64_t mine = (uint64_t)mine128;
    auto chunk_range = [&](uint64_t i, u128 &cs, u128 &ce) {
        cs = s + (u128)(deal_offset + (u128)i * deal_stride) * chunk;
        ce = std::min(e, cs + chunk);
    };

    job.used.assign(ctx->devs.size(), 0);
    job.all.clear();
    job.empty = false;
    job.collected = false;
    job.st = st;
    auto finish_submit = [&]() { return NICE_OK; };
    if (nice::residue_filter(base).empty() || mine == 0) {  // client_process_gpu.rs:525-531
        job.empty = true;
        return finish_submit();
    }
    auto table = g_stride.get(base, k);
    // Whole field inside the base's valid range: the kernels take their
    // fixed-digit-count fast paths (radix_fast.hpp).
    u128 vr_s = 0, vr_e = 0;
    const uint32_t in_range = nice::base_range_cached(base, vr_s, vr_e) == 1 && vr_s <= s && e <= vr_e ? 1u : 0u;
    const uint32_t R = (uint32_t)table->residues.size();
    const uint64_t M = table->modulus;
    if (M > 0xffffffffull) return fail(NICE_ERR_INVALID, "stride modulus exceeds u32");
    for (auto &d : ctx->devs) {
        HIPCHK(hipSetDevice(d.id));
        if (!d.residues.count(base * 8 + k)) {
            uint32_t *p;
            HIPCHK(hipMalloc(&p, (size_t)R * 4));
            HIPCHK(hipMemcpy(p, table->residues.data(), (size_t)R * 4, hipMemcpyHostToDevice));
            d.residues[base * 8 + k] = p;
            // rank[r] = lower_bound(residues, r): the device MSD turns a leaf's
            // end points into stride indices with one load each.
            std::vector<uint32_t> rank((size_t)M + 1);
            uint32_t g = 0;
            for (uint64_t r = 0; r <= M; r++) {
                while (g < R && table->residues[g] < r) g++;
                rank[r] = g;
            }
            HIPCHK(hipMalloc(&p, rank.size() * 4));
            HIPCHK(hipMemcpy(p, rank.data(), rank.size() * 4, hipMemcpyHostToDevice));
            d.ranks[base * 8 + k] = p;
        }
    }

    // Device MSD: batches of this caller's chunks, each run as init + the
    // level kernels + the candidate kernel, all stream-ordered (no host sync
    // until the end).  Batches alternate over the context's devices.
    auto run_device = [&]() -> int {
        if (chunk > ((u128)1 << 40)) return fail(NICE_ERR_INVALID, "device MSD: chunk_size too large");
        if ((e - s) >> 63) return fail(NICE_ERR_INVALID, "device MSD: field larger than 2^63");
        const uint64_t cnk = (uint64_t)chunk;
        // Nodes per level and leaves per batch are <= batch / floor + chunks
        // (every split child holds >= floor numbers); size batches for 2^27
        // (16-byte nodes: 2 x 2 GB of level queues and 3 GB of leaf records at
        // most, allocated as a field needs them).  Batches are the unit of the
        // level launches, so larger ones amortise their fixed cost: the massive
        // field (chunk 1e8) took 0.365 s at 41 chunks per batch (2^24), 0.20 s
        // at 164, 0.17 s at 328 (profiles/r02/massive_batch_sweep.log).
        const uint64_t fl = std::min<uint64_t>(floor_size, 1ull << 30);
        uint64_t cpb = std::max<uint64_t>(1, (fl << 27) / cnk);
        if (nice::probe_set("NICE_MSD_CPB")) cpb = std::max<uint64_t>(1, nice::probe_knob("NICE_MSD_CPB", 1));
        cpb = std::min(cpb, mine);
        const uint64_t batch_n = cpb * cnk;
        uint64_t per = std::min<uint64_t>(batch_n / fl + cpb, cpb << 22) + 64;
        per = std::min<uint64_t>(per, 1ull << 28);  // (the bound above stays below this)
        // leaf records: one per range plus one per kLeafPiece candidates
        const uint64_t leaf_cap = std::min<uint64_t>(per + (batch_n / nice::kLeafPiece) + 64, 0xffffffffull);
        // Chunks whose recursion fits a workgroup run fused: one launch per
        // batch, one workgroup per chunk (grid-strided), no level queues.
        const uint32_t fcap = nice::probe_set("NICE_MSD_FCAP") && cnk <= 0xffffffffull
                                  ? (uint32_t)nice::probe_knob("NICE_MSD_FCAP", 0)
                                  : nice::msd_fused_cap(cnk, floor_size);
        // Chunks too large for the fused kernel: the level BFS only down to a
        // root level `wlevel` (nodes <= 2^26 numbers, ~2048 roots per wave of
        // the fused MSD + candidate kernel), then msd_wave_kernel.  Nothing of
        // a batch grows with its survivors any more (leaves are tested inside
        // the wave that finds them), so a batch is bounded only by the level
        // queues: 2^24 nodes at the root level.  The massive field is ONE
        // batch.
        bool wave = !fcap;
        if (nice::probe_set("NICE_MSD_NOWAVE")) wave = false;  // A/B: the level-BFS + leaf-list path
        uint32_t wlevel = 0, wgrid = 0;
        uint64_t wleaf_cap = 0;
        if (wave) {
            int cus = 256;
            for (auto &d : ctx->devs) cus = std::max(cus, d.num_cus);
            wgrid = (uint32_t)cus * 16 / nice::msd_wave_waves_per_group();  // 4 waves per SIMD
            // roots per wave: 2048 (the whole massive field 0.097 s at 32, 0.080 s
            // at 2048; a 1/8 dealt share 0.0135 / 0.0101 s, scripts/roots_sweep.py)
            const uint64_t waves = (uint64_t)wgrid * nice::msd_wave_waves_per_group();
            uint64_t target = waves * 2048;
            if (nice::probe_set("NICE_MSD_ROOTS")) target = waves * nice::probe_knob("NICE_MSD_ROOTS", 1);
            uint32_t last = 0;  // first level without splits
            while (last < 22 && ((cnk + (1ull << last) - 1) >> last) >= 2 * fl) last++;
            while (wlevel < last && ((cnk + (1ull << wlevel) - 1) >> wlevel) > (1ull << 26)) wlevel++;
            for (;;) {
                // (a multi-device context gets at least one batch per device)
                const uint64_t per_dev = (mine + ctx->devs.size() - 1) / ctx->devs.size();
                cpb = std::min<uint64_t>(per_dev, std::max<uint64_t>(1, (1ull << 24) >> wlevel));
                if ((cpb << wlevel) >= target || wlevel >= last) break;
                wlevel++;
            }
            if (((cnk + (1ull << wlevel) - 1) >> wlevel) > (1ull << 26))
                return fail(NICE_ERR_INVALID, "device MSD: chunk_size too large for the floor");
            per = (cpb << wlevel) + 64;
            // leaves of the BFS levels (clipped / depth-limited nodes), in pieces
            wleaf_cap = per * (1 + (fl >> 28)) + 64;
        }
        const uint64_t nbatches = nbatches_of(mine, cpb);
        for (size_t i = 0; i < ctx->devs.size(); i++) {
            Device &d = ctx->devs[i];
            HIPCHK(hipSetDevice(d.id));
            const uint64_t fgrid = std::min<uint64_t>(cpb, (uint64_t)d.num_cus * 4);
            int r = fcap   ? ensure_msd(d.slot[t], 0, (uint32_t)leaf_cap, fgrid * 2 * fcap)
                    : wave ? ensure_msd(d.slot[t], (uint32_t)per, (uint32_t)wleaf_cap, 0,
                                        nice::msd_wave_scratch_bytes(wgrid))
                           : ensure_msd(d.slot[t], (uint32_t)per, (uint32_t)leaf_cap, 0);
            if (r) return r;
            if (i < nbatches) {
                job.used[i] = 1;
                if (d.slot[t].msd.dirty) {  // first use / after an interrupted field
                    HIPCHK(hipMemsetAsync(d.slot[t].msd.counters, 0, nice::kMsdCounterWords * 4, d.slot[t].nstream));
                    HIPCHK(hipMemsetAsync(d.slot[t].d_nice_count, 0, 4, d.slot[t].nstream));
                }
                d.slot[t].msd.dirty = true;  // until this field's epilogue is seen
            }
        }
        for (uint64_t bi = 0; bi < nbatches; bi++) {
            Device &d = ctx->devs[bi % ctx->devs.size()];
            HIPCHK(hipSetDevice(d.id));
            const bool first = bi < ctx->devs.size();  // this device's first batch of the field
            const bool last = bi + ctx->devs.size() >= nbatches;  // ... and its last
            nice::MsdLaunch mp{};
            mp.first_batch = first ? 1u : 0u;
            mp.nice_count = d.slot[t].d_nice_count;
            mp.start_lo = lo64(s);
            mp.start_hi = hi64(s);
            mp.end_lo = lo64(e);
            mp.end_hi = hi64(e);
            mp.first = bi * cpb;
            mp.nchunks = std::min(cpb, mine - bi * cpb);
            mp.deal_stride = deal_stride;
            mp.deal_offset = deal_offset;
            mp.chunk = cnk;
            mp.floor_size = floor_size;
            const MsdBuf &mb = d.slot[t].msd;
            mp.q[0] = mb.q[0];
            mp.q[1] = mb.q[1];
            mp.counters = mb.counters;
            mp.q_cap = mb.q_cap;
            mp.leaves = mb.leaves;
            mp.leaf_cap = mb.leaf_cap;
            mp.residues = d.residues[base * 8 + k];
            mp.ranks = d.ranks[base * 8 + k];
            mp.R = R;
            mp.M = (uint32_t)M;
            mp.base = base;
            mp.in_range = in_range;
            mp.probe = (uint32_t)nice::probe_knob("NICE_MSD_PROBE", 0);
            nice::NiceonlyLaunch p{};
            if (wave) {
                p.residues = mp.residues;
                p.R = R;
                p.M = (uint32_t)M;
                p.base = base;
                p.in_range = in_range;
                p.out = nice::NumOut{d.slot[t].nice.n, nullptr, d.slot[t].d_nice_count, d.slot[t].nice.cap};
                p.fin = last ? nice::NiceFinish{d.slot[t].d_msd_mapped, d.slot[t].d_nice_mapped, mb.counters,
                                                d.slot[t].d_nice_done}
                             : nice::NiceFinish{nullptr, nullptr, mb.counters, d.slot[t].d_nice_done};
                hipError_t err = nice::launch_msd_wave(mp, p, wlevel, mb.wscratch, wgrid, d.num_cus,
                                                       d.slot[t].nstream);
                if (err != hipSuccess)
                    return fail(NICE_ERR_HIP, std::string("msd wave launch: ") + hipGetErrorString(err));
                st.launches++;
                continue;
            }
            const uint32_t fgrid = (uint32_t)std::min<uint64_t>(mp.nchunks, (uint64_t)d.num_cus * 4);
            hipError_t err = fcap ? nice::launch_msd_device(mp, d.num_cus, d.slot[t].nstream, mb.scratch, fcap, fgrid)
                                  : nice::launch_msd_device(mp, d.num_cus, d.slot[t].nstream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("msd launch: ") + hipGetErrorString(err));
            p.leaves = mb.leaves;
            p.n_leaves_dev = mb.counters + 24;
            p.n_leaves = mb.leaf_cap;  // clamp for the device count
            p.residues = mp.residues;
            p.R = R;
            p.M = (uint32_t)M;
            p.base = base;
            p.in_range = in_range;
            p.out = nice::NumOut{d.slot[t].nice.n, nullptr, d.slot[t].d_nice_count, d.slot[t].nice.cap};
            // epilogue: re-zero the batch's leaf count; at the field's end the
            // results land in mapped memory (no copy launches)
            p.fin = last ? nice::NiceFinish{d.slot[t].d_msd_mapped, d.slot[t].d_nice_mapped, mb.counters,
                                            d.slot[t].d_nice_done}
                         : nice::NiceFinish{nullptr, nullptr, mb.counters, d.slot[t].d_nice_done};
            err = nice::launch_niceonly(p, d.num_cus, d.slot[t].nstream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("niceonly launch: ") + hipGetErrorString(err));
            st.launches++;
        }
        for (size_t i = 0; i < ctx->devs.size(); i++) {
            if (!job.used[i]) continue;
            Device &d = ctx->devs[i];
            HIPCHK(hipSetDevice(d.id));
            HIPCHK(hipEventRecord(d.slot[t].nice_done, d.slot[t].nstream));
        }
        return NICE_OK;
    };

    const int where = opts ? opts->msd_where : NICE_MSD_AUTO;
    if (where < NICE_MSD_AUTO || where > NICE_MSD_DEVICE) return fail(NICE_ERR_INVALID, "bad msd_where");
    const bool on_device = where == NICE_MSD_DEVICE ||
                           (where == NICE_MSD_AUTO && k == 2 && !((e - s) >> 63) && chunk <= ((u128)1 << 40));
    job.on_device = on_device;
    job.adapt = adaptive && !on_device;  // the floor balances the host MSD producer against the GPU
    int rc = NICE_OK;
    if (on_device) {
        rc = run_device();
    } else {
        for (auto &d : ctx->devs) {
            HIPCHK(hipSetDevice(d.id));
            // the adaptive floor's GPU-tail clock starts with the field (the
            // stream reaches this event as soon as it is idle)
            if (job.adapt) HIPCHK(hipEventRecord(d.slot[t].nt0, d.slot[t].nstream));
            HIPCHK(hipMemsetAsync(d.slot[t].d_nice_count, 0, 4, d.slot[t].nstream));
            d.slot[t].msd.dirty = true;  // the nice count is left set
        }
        // Producer: worker threads run the MSD filter per chunk and hand the
        // surviving ranges to this thread in chunk batches.
        std::atomic<uint64_t> next{0};
        std::mutex qmu;
        std::condition_variable qcv;
        std::deque<std::vector<std::pair<u128, u128>>> queue;
        const int n_workers = (int)std::min<uint64_t>(threads, mine);
        st.msd_threads = (uint32_t)n_workers;
        int live = n_workers;  // guarded by qmu
        std::vector<std::thread> workers;
        std::unique_ptr<nice::MsdRunner> filt = nice::make_msd(base);
        for (int t = 0; t < n_workers; t++) {
            workers.emplace_back([&]() {
                std::vector<std::pair<u128, u128>> local;
                for (;;) {
                    uint64_t i = next.fetch_add(1);
                    if (i >= mine) break;
                    u128 cs, ce;
                    chunk_range(i, cs, ce);
                    filt->ranges(cs, ce, floor_size, local);
                    if (local.size() >= 4096) {
                        std::lock_guard<std::mutex> g(qmu);
                        queue.push_back(std::move(local));
                        local = {};
                        qcv.notify_one();
                    }
                }
                std::lock_guard<std::mutex> g(qmu);
                if (!local.empty()) queue.push_back(std::move(local));
                live--;
                qcv.notify_one();
            });
        }

        // Consumer: build descriptors and launch on devices round-robin.
        size_t dev_rr = 0;
        std::vector<std::pair<u128, u128>> pend;
        auto flush = [&]() -> int {
            if (pend.empty()) return NICE_OK;
            const size_t di = dev_rr++ % ctx->devs.size();
            Device &d = ctx->devs[di];
            job.used[di] = 1;
            HIPCHK(hipSetDevice(d.id));
            LeafBuf &b = d.desc[d.desc_next];
            d.desc_next ^= 1;
            // One leaf per range, more for ranges holding over kLeafPiece
            // candidates (the kernel sums 8 leaves' counts in 32 bits).
            constexpr u128 kPiece = nice::kLeafPiece;
            size_t need = 0;
            for (auto &pr : pend) {
                const u128 c = table->index_of(pr.second) - table->index_of(pr.first);
                need += (size_t)((c + kPiece - 1) / kPiece);
            }
            int r = ensure_desc(b, (uint32_t)std::max<size_t>(need, 1));
            if (r) return r;
            if (b.pending) HIPCHK(hipEventSynchronize(b.done));
            uint32_t nr = 0;
            uint64_t total = 0;
            for (auto &pr : pend) {
                const u128 i0 = table->index_of(pr.first), i1 = table->index_of(pr.second);
                st.ranges++;
                st.range_numbers += (uint64_t)(pr.second - pr.first);
                for (u128 g = i0; g < i1; g += kPiece) {
                    // candidate g of the global residue sequence: (g / R) * M + res[g % R]
                    const u128 cyc = g / R;
                    const u128 bs = cyc * M;
                    const uint32_t cnt = (uint32_t)std::min<u128>(kPiece, i1 - g);
                    b.h[nr++] = nice::Leaf{lo64(bs), hi64(bs), (uint32_t)(g - cyc * R), cnt};
                    total += cnt;
                }
            }
            pend.clear();
            if (!nr) return NICE_OK;
            st.candidates += total;
            HIPCHK(hipMemcpyAsync(b.d, b.h, (size_t)nr * sizeof(nice::Leaf), hipMemcpyHostToDevice,
                                  d.slot[t].nstream));
            nice::NiceonlyLaunch p{};
            p.leaves = b.d;
            p.n_leaves_dev = nullptr;
            p.n_leaves = nr;
            p.residues = d.residues[base * 8 + k];
            p.R = R;
            p.M = (uint32_t)M;
            p.base = base;
            p.in_range = in_range;
            p.out = nice::NumOut{d.slot[t].nice.n, nullptr, d.slot[t].d_nice_count, d.slot[t].nice.cap};
            hipError_t err = nice::launch_niceonly(p, d.num_cus, d.slot[t].nstream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("niceonly launch: ") + hipGetErrorString(err));
            HIPCHK(hipEventRecord(b.done, d.slot[t].nstream));
            b.pending = true;
            st.launches++;
            return NICE_OK;
        };
        for (;;) {
            std::vector<std::pair<u128, u128>> item;
            {
                std::unique_lock<std::mutex> g(qmu);
                qcv.wait(g, [&] { return !queue.empty() || live == 0; });
                if (queue.empty() && live == 0) break;
                item = std::move(queue.front());
                queue.pop_front();
            }
            if (rc) continue;  // drain the producers after a failure
            pend.insert(pend.end(), item.begin(), item.end());
            if (pend.size() >= kBatchRanges) rc = flush();
        }
        for (auto &w : workers) w.join();
        st.msd_seconds = std::chrono::duration<double>(clock::now() - t0).count();
        if (!rc) rc = flush();
        // End of the field on every device: its list count, then a marker.
        for (size_t i = 0; i < ctx->devs.size() && !rc; i++) {
            Device &d = ctx->devs[i];
            job.used[i] = 1;
            HIPCHK(hipSetDevice(d.id));
            HIPCHK(hipMemcpyAsync(d.slot[t].h_nice, d.slot[t].d_nice_count, 4, hipMemcpyDeviceToHost,
                                  d.slot[t].nstream));
            HIPCHK(hipEventRecord(d.slot[t].nice_done, d.slot[t].nstream));
            if (job.adapt) HIPCHK(hipEventRecord(d.slot[t].nt1, d.slot[t].nstream));
        }
    }
    if (rc) return rc;
    job.st = st;
    return finish_submit();
}

// Read a finished niceonly field's results from the devices (its events have
// completed).  counts receives every device's list length; *over is set when
// one exceeded its device's list capacity (that device's list was not read).
int niceonly_gather(nice_ctx *ctx, NiceJob &job, int t, std::vector<uint32_t> &counts, bool *over_out) {
    counts.assign(ctx->devs.size(), 0);
    bool over = false;
    *over_out = false;
    for (size_t i = 0; i < ctx->devs.size(); i++) {
        Device &d = ctx->devs[i];
        Slot &sl = d.slot[t];
        if (!job.used[i]) continue;  // no batch of this field ran there
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(hipEventSynchronize(sl.nice_done));
        if (job.on_device) {
            const uint32_t *c = sl.h_msd;
            sl.msd.dirty = false;  // the epilogue re-zeroed counters and count
            if (nice::probe_set("NICE_MSD_TRACE")) {  // level sizes of the last batch (diagnostics)
                fprintf(stderr, "msd levels:");
                for (int lv = 0; lv < 24; lv++) fprintf(stderr, " %u", c[lv]);
                fprintf(stderr, " | ranges %u\n", c[26]);
            }
            if (c[25])
                return fail(NICE_ERR_MSD_OVERFLOW, "device MSD queue overflow (msd_floor too small "
                                               "for chunk_size); use msd_where = host");
            uint64_t cand, nums;
            std::memcpy(&cand, c + 28, 8);
            std::memcpy(&nums, c + 30, 8);
            job.st.ranges += c[26];
            job.st.candidates += cand;
            job.st.range_numbers += nums;
            job.st.square_ok += c[27];
        }
        const uint32_t cnt = *sl.h_nice;
        counts[i] = cnt;
        if (cnt > sl.nice.cap) {
            // more nice numbers than the device list holds (the kernels count
            // every hit, store those below the capacity): grow and re-run
            over = true;
            *over_out = true;
            continue;
        }
        if (cnt && !over) {
            std::vector<uint64_t> nbuf((size_t)cnt * 2);
            HIPCHK(hipMemcpy(nbuf.data(), sl.nice.n, (size_t)cnt * 16, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < cnt; q++) job.all.push_back({mk(nbuf[2 * q], nbuf[2 * q + 1]), job.base});
        }
    }
    return NICE_OK;
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

int niceonly_submit_args(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo, uint64_t end_hi,
                         uint32_t base, const nice_niceonly_opts *opts, bool wait, int *ticket) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!ctx || !ticket) return fail(NICE_ERR_INVALID, "null argument");
    if (base < 3 || base > 128) return fail(NICE_ERR_INVALID, "base must be in 3..=128");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (s >= e)
        return fail(NICE_ERR_INVALID, "Range has invalid bounds, range_start must be < range_end");
    if (opts && opts->deal_offset >= (opts->deal_stride ? opts->deal_stride : 1u))
        return fail(NICE_ERR_INVALID, "deal_offset must be < deal_stride");
    const uint64_t floor_size = resolve_floor(opts);
    std::unique_lock<std::mutex> lock(ctx->mu);
    int t = -1;
    if (int rc = acquire_slot(ctx, lock, ctx->nice, ctx->nice_next, wait, "niceonly", &t)) return rc;
    NiceJob &job = ctx->nice[t];
    job = NiceJob{};
    job.owner = std::this_thread::get_id();
    job.s = s;
    job.e = e;
    job.base = base;
    job.has_opts = opts != nullptr;
    if (opts) job.opts = *opts;
    job.st.msd_floor = floor_size;
    job.t0 = t0;
    const int rc = niceonly_enqueue(ctx, t, job);
    if (rc) return rc;
    job.active = true;
    ctx->nice_next = (t + 1) % slots_used();
    *ticket = t;
    return NICE_OK;
}

int niceonly_collect_locked(nice_ctx *ctx, int t, nice_number *out, size_t cap, size_t *n_out,
                            nice_niceonly_stats *stats) {
    std::unique_lock<std::mutex> lock(ctx->mu);
    if (t < 0 || t >= kSlots || !ctx->nice[t].active)
        return fail(NICE_ERR_INVALID, "no niceonly field in flight under this ticket");
    NiceJob &job = ctx->nice[t];
    if (job.waiting) return fail(NICE_ERR_INVALID, "another thread is collecting this niceonly field");
    if (!job.collected) {
        int rc = NICE_OK;
        if (!job.empty) {
            // Wait for the devices WITHOUT the context lock, so other threads
            // can submit and collect other fields meanwhile (the slot stays
            // reserved: the job is active).
            job.waiting = true;
            lock.unlock();
            for (size_t i = 0; i < ctx->devs.size() && !rc; i++) {
                if (!job.used[i]) continue;
                Slot &sl = ctx->devs[i].slot[t];
                hipError_t err = hipSetDevice(ctx->devs[i].id);
                if (err == hipSuccess) err = sync_event(sl.nice_done);
                if (err != hipSuccess) rc = fail(NICE_ERR_HIP, std::string("niceonly field: ") + hipGetErrorString(err));
            }
            lock.lock();
            job.waiting = false;
        }
        std::vector<uint32_t> counts;
        bool over = false;
        if (!rc && !job.empty) rc = niceonly_gather(ctx, job, t, counts, &over);
        for (uint32_t attempt = 0; !rc && !job.empty && over; attempt++) {
            if (attempt) {
                rc = fail(NICE_ERR_HIP, "niceonly list overflowed again after growing it to the field's count");
                break;
            }
            // Grow EVERY device's list to the whole field's count and re-run
            // the field (under the lock: rare).  The host MSD producer hands
            // batches to devices in the order its threads finish chunks (and
            // the re-run clears job.used), so a re-run can put the hits on a
            // device the first run never used; no device can hold more than
            // the field's total.
            uint64_t total = 0;
            for (uint32_t c : counts) total += c;
            if (total > 0xfffff000ull) {
                rc = fail(NICE_ERR_HIP, "niceonly list longer than 2^32 entries");
                break;
            }
            for (size_t i = 0; i < ctx->devs.size() && !rc; i++)
                rc = ensure_listbuf(ctx->devs[i], ctx->devs[i].slot[t].nice, ((uint32_t)total + 4095u) & ~4095u,
                                    false);
            if (!rc) rc = niceonly_enqueue(ctx, t, job);
            if (!rc) job.reruns++;
            if (!rc) rc = niceonly_gather(ctx, job, t, counts, &over);
        }
        if (rc) {
            job.active = false;
            return rc;
        }
        job.st.total_seconds =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - job.t0).count();
        job.st.reruns = job.reruns;
        job.collected = true;
        // A re-run field's MSD time covers its last run only while its total
        // spans every run: the two do not balance, so it does not move the floor.
        if (job.adapt && job.reruns == 0) {  // update_msd_floor (client_process_gpu.rs:551, 563-568, 130-157)
            // The GPU tail ends when the field's last device work does (its
            // end event), not when the caller gets round to collecting: the
            // reference times both phases inside one call (:541-551).
            double gpu_end = 0;
            for (size_t i = 0; i < ctx->devs.size(); i++) {
                if (!job.used[i]) continue;
                Slot &sl = ctx->devs[i].slot[t];
                float ms = 0;
                if (hipSetDevice(ctx->devs[i].id) == hipSuccess &&
                    hipEventElapsedTime(&ms, sl.nt0, sl.nt1) == hipSuccess)
                    gpu_end = std::max(gpu_end, ms * 1e-3);
            }
            const double total = std::max(job.st.msd_seconds, gpu_end);
            std::lock_guard<std::mutex> g(g_af_mu);
            AdaptiveFloor &af = adaptive_floor();
            if (af.warmup == kAdaptPinned) {
            } else if (af.warmup > 0) {
                af.warmup--;
            } else {
                af.floor = nice_adaptive_floor_step(af.floor, job.st.msd_seconds, total);
            }
        }
    }
    if (stats) *stats = job.st;
    const int rc = emit_list(job.all, out, cap, n_out);
    if (rc == NICE_ERR_CAPACITY) return rc;  // kept: the caller retries with room
    job.active = false;
    job.all = {};
    return rc;
}

}  // namespace

extern "C" {

int nice_niceonly_submit(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi, uint64_t end_lo,
                         uint64_t end_hi, uint32_t base, const nice_niceonly_opts *opts, int *ticket) {
    return niceonly_submit_args(ctx, start_lo, start_hi, end_lo, end_hi, base, opts, false, ticket);
}

int nice_niceonly_collect(nice_ctx *ctx, int t, nice_number *out, size_t cap, size_t *n_out,
                          nice_niceonly_stats *stats) {
    if (!ctx) return fail(NICE_ERR_INVALID, "null ctx");
    const int rc = niceonly_collect_locked(ctx, t, out, cap, n_out, stats);
    ctx->freed.notify_all();  // the ticket's slot may be free now
    return rc;
}

int nice_process_range_niceonly_ex(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                   uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                   const nice_niceonly_opts *opts, nice_number *out, size_t cap,
                                   size_t *n_out, nice_niceonly_stats *stats) {
    int t = -1;
    int rc = niceonly_submit_args(ctx, start_lo, start_hi, end_lo, end_hi, base, opts, true, &t);
    if (rc) return rc;
    rc = nice_niceonly_collect(ctx, t, out, cap, n_out, stats);
    if (rc == NICE_ERR_CAPACITY) {
        {
            std::lock_guard<std::mutex> lock(ctx->mu);
            ctx->nice[t].active = false;
            ctx->nice[t].all = {};
        }
        ctx->freed.notify_all();
    }
    return rc;
}

int nice_process_range_niceonly(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base, nice_number *out,
                                size_t cap, size_t *n_out) {
    return nice_process_range_niceonly_ex(ctx, start_lo, start_hi, end_lo, end_hi, base, nullptr,
                                          out, cap, n_out, nullptr);
}

}  // extern "C"
