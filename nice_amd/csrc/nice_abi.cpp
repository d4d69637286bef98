// nice_abi.cpp -- C ABI (include/nice_hip.h) over the gfx950 kernels.
//
// Replaces the reference's CUDA host pipeline (common/src/client_process_gpu.rs):
// no NVRTC (kernels are AOT code objects), one HIP stream per device, fields
// sharded across devices as contiguous n-ranges, histograms summed and
// near-miss / nice lists merged on the host, and a multi-threaded host MSD
// producer streaming range descriptors to the niceonly kernel.
#include <hip/hip_runtime.h>

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
#include "radix_fast.hpp"

using nice::u128;

namespace {

// Per-device state block: kHistCopies histograms of 129 u64 bins (kernels
// spread their end-of-launch atomics over the copies: hundreds of workgroups
// adding to ONE address serialise in L2), then the two list counters.
constexpr size_t kHistCopies = nice::kHistCopies;
constexpr size_t kStateBytes = kHistCopies * 129 * 8 + 2 * 4;

thread_local std::string g_err;

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
    // device MSD: ping-pong level queues, leaf list, counters (kernels.h)
    nice::MsdNode *q[2] = {nullptr, nullptr};
    nice::Leaf *leaves = nullptr;
    uint32_t *counters = nullptr;  // 32 words
    uint32_t *h_counters = nullptr;  // pinned
    uint32_t q_cap = 0, leaf_cap = 0;
};

struct Device {
    int id = 0;
    int num_cus = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_done = nullptr;
    uint64_t *d_hist = nullptr;   // kHistCopies x 129 bins, then d_count
    uint32_t *d_count = nullptr;  // list counters [0] detailed, [1] niceonly (inside d_hist's block)
    uint64_t *d_list_n = nullptr;
    uint32_t *d_list_u = nullptr;
    uint32_t list_cap = 0;
    uint64_t *h_hist = nullptr;   // pinned
    uint32_t *h_count = nullptr;  // pinned
    uint64_t *h_fin = nullptr;    // mapped pinned: summed histogram [0..128], near-miss count [129]
    uint64_t *d_fin = nullptr;    // device view of h_fin
    bool state_dirty = true;      // d_hist / d_count[0] not known to be zero
    std::map<uint32_t, uint32_t *> residues;  // base*8+k -> device residue table
    std::map<uint32_t, uint32_t *> ranks;     // base*8+k -> lower_bound(residues, r), r in [0, M]
    LeafBuf desc[2];
    int desc_next = 0;
    MsdBuf msd;
    nice_kernel_stats last{};
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

}  // namespace

struct nice_ctx {
    std::vector<Device> devs;
    std::mutex mu;  // one in-flight field per context (client_process_gpu.rs:196-201)
};

namespace {

int ensure_list(Device &d, uint32_t cap) {
    if (d.list_cap >= cap) return NICE_OK;
    HIPCHK(hipSetDevice(d.id));
    if (d.d_list_n) HIPCHK(hipFree(d.d_list_n));
    if (d.d_list_u) HIPCHK(hipFree(d.d_list_u));
    HIPCHK(hipMalloc(&d.d_list_n, (size_t)cap * 16));
    HIPCHK(hipMalloc(&d.d_list_u, (size_t)cap * 4));
    d.list_cap = cap;
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

int ensure_msd(Device &d, uint32_t q_cap, uint32_t leaf_cap) {
    MsdBuf &m = d.msd;
    if (!m.counters) {
        HIPCHK(hipMalloc(&m.counters, 32 * 4));
        HIPCHK(hipHostMalloc(&m.h_counters, 32 * 4, hipHostMallocDefault));
    }
    if (m.q_cap < q_cap) {
        for (auto &q : m.q)
            if (q) HIPCHK(hipFree(q));
        for (auto &q : m.q) HIPCHK(hipMalloc(&q, (size_t)q_cap * sizeof(nice::MsdNode)));
        m.q_cap = q_cap;
    }
    if (m.leaf_cap < leaf_cap) {
        if (m.leaves) HIPCHK(hipFree(m.leaves));
        HIPCHK(hipMalloc(&m.leaves, (size_t)leaf_cap * sizeof(nice::Leaf)));
        m.leaf_cap = leaf_cap;
    }
    return NICE_OK;
}

int device_init(Device &d, int id) {
    d.id = id;
    HIPCHK(hipSetDevice(id));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, id));
    d.num_cus = prop.multiProcessorCount;
    HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&d.ev0));
    HIPCHK(hipEventCreate(&d.ev1));
    HIPCHK(hipEventCreateWithFlags(&d.ev_done, hipEventDisableTiming));
    // hist bins and list counters in one block: one memset and one copy per field.
    HIPCHK(hipMalloc(&d.d_hist, kStateBytes));
    d.d_count = (uint32_t *)(d.d_hist + kHistCopies * 129);
    HIPCHK(hipHostMalloc(&d.h_hist, kStateBytes, hipHostMallocDefault));
    d.h_count = (uint32_t *)(d.h_hist + kHistCopies * 129);
    HIPCHK(hipHostMalloc(&d.h_fin, 130 * 8, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&d.d_fin, d.h_fin, 0));
    int rc = ensure_list(d, kInitialListCap);
    if (rc) return rc;
    return NICE_OK;
}

void device_free(Device &d) {
    if (!d.stream) return;
    (void)hipSetDevice(d.id);
    (void)hipStreamSynchronize(d.stream);
    for (auto &kv : d.residues) (void)hipFree(kv.second);
    for (auto &kv : d.ranks) (void)hipFree(kv.second);
    for (auto &b : d.desc) {
        if (b.h) {
            (void)hipHostFree(b.h);
            (void)hipFree(b.d);
        }
        if (b.done) (void)hipEventDestroy(b.done);
    }
    for (auto &q : d.msd.q)
        if (q) (void)hipFree(q);
    if (d.msd.leaves) (void)hipFree(d.msd.leaves);
    if (d.msd.counters) (void)hipFree(d.msd.counters);
    if (d.msd.h_counters) (void)hipHostFree(d.msd.h_counters);
    (void)hipFree(d.d_hist);
    (void)hipFree(d.d_list_n);
    (void)hipFree(d.d_list_u);
    (void)hipHostFree(d.h_hist);
    (void)hipHostFree(d.h_fin);
    (void)hipEventDestroy(d.ev0);
    (void)hipEventDestroy(d.ev1);
    (void)hipEventDestroy(d.ev_done);
    (void)hipStreamDestroy(d.stream);
    d.stream = nullptr;
}

struct Entry {
    u128 n;
    uint32_t u;
};

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

#ifdef NICE_PROBES
// FD kernel variant (0 = production choice; others for scripts/fd_sweep.py).
int fd_variant() {
    const char *v = getenv("NICE_FD_VARIANT");
    return v ? atoi(v) : 0;
}
#endif

// Enqueue the detailed kernels for [s, e) on one device (async).
int enqueue_detailed(Device &d, u128 s, u128 e, uint32_t base, bool &used_fd, uint64_t &fd_count) {
    nice::DetailedLaunch p{};
    p.base = base;
    p.cutoff = nice::near_miss_cutoff(base);
    p.hist = d.d_hist;
    p.out = nice::NumOut{d.d_list_n, d.d_list_u, d.d_count, d.list_cap};
    auto launch = [&](u128 a, u128 b, bool fd) -> int {
        if (a >= b) return NICE_OK;
        u128 cnt = b - a;
        while (cnt) {  // segments longer than 2^63 are split (count is u64)
            uint64_t c = cnt > ((u128)1 << 62) ? (1ull << 62) : (uint64_t)cnt;
            p.start_lo = lo64(a);
            p.start_hi = hi64(a);
            p.count = c;
#ifdef NICE_PROBES
            const int var = fd_variant();
            hipError_t err = !fd ? nice::launch_detailed_generic(p, d.num_cus, d.stream)
                             : var == 0 && nice::fd2_supported(base)
                                 ? nice::launch_detailed_fd2(p, d.num_cus, d.stream)
                                 : nice::launch_detailed_fd(p, d.num_cus, d.stream, var);
#else
            hipError_t err = fd ? nice::launch_detailed_fd2(p, d.num_cus, d.stream)
                                : nice::launch_detailed_generic(p, d.num_cus, d.stream);
#endif
            if (err != hipSuccess)
                return fail(NICE_ERR_HIP, std::string("detailed launch: ") + hipGetErrorString(err));
            if (fd) {
                used_fd = true;
                fd_count += c;
            }
            a += c;
            cnt -= c;
        }
        return NICE_OK;
    };
    u128 rs = 0, re = 0;
#ifdef NICE_PROBES
    const bool fd_base = nice::fd2_supported(base) || (fd_variant() && nice::fd_supported(base));
#else
    const bool fd_base = nice::fd2_supported(base);
#endif
    const bool fd = fd_base && nice::base_range_cached(base, rs, re) == 1;
    if (!fd) return launch(s, e, false);
    int rc;
    if ((rc = launch(s, std::min(e, rs), false))) return rc;
    if ((rc = launch(std::max(s, rs), std::min(e, re), true))) return rc;
    return launch(std::max(s, re), e, false);
}

}  // namespace

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

int nice_last_kernel_stats(nice_ctx *ctx, int i, nice_kernel_stats *out) {
    if (!ctx || i < 0 || i >= (int)ctx->devs.size() || !out) return fail(NICE_ERR_INVALID, "bad args");
    *out = ctx->devs[i].last;
    return NICE_OK;
}

int nice_process_range_detailed(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base, uint64_t *hist,
                                nice_number *out, size_t cap, size_t *n_out) {
    if (!ctx || !hist) return fail(NICE_ERR_INVALID, "null argument");
    if (base < 2 || base > 128) return fail(NICE_ERR_INVALID, "base must be in 2..=128");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (s >= e)
        return fail(NICE_ERR_INVALID, "Range has invalid bounds, range_start must be < range_end");
    std::lock_guard<std::mutex> lock(ctx->mu);
    const size_t nd = ctx->devs.size();
    const u128 size = e - s;
    // Shard bounds: contiguous, in device order (ascending n).
    std::vector<u128> bounds(nd + 1);
    for (size_t i = 0; i <= nd; i++) bounds[i] = s + size / nd * i + std::min<u128>(i, size % nd);
    for (size_t i = 0; i < nd; i++) {
        Device &d = ctx->devs[i];
        d.last = nice_kernel_stats{};
        if (bounds[i] >= bounds[i + 1]) continue;
        HIPCHK(hipSetDevice(d.id));
        // The state block is zeroed by the previous field's epilogue; a
        // memset only after an interrupted field (or the first one).
        if (d.state_dirty) HIPCHK(hipMemsetAsync(d.d_hist, 0, kStateBytes, d.stream));
        d.state_dirty = true;
        HIPCHK(hipEventRecord(d.ev0, d.stream));
        bool used_fd = false;
        uint64_t fdc = 0;
        int rc = enqueue_detailed(d, bounds[i], bounds[i + 1], base, used_fd, fdc);
        if (rc) return rc;
        HIPCHK(hipEventRecord(d.ev1, d.stream));
        HIPCHK(nice::launch_detailed_finish(d.d_hist, d.d_count, d.d_fin, d.stream));
        HIPCHK(hipEventRecord(d.ev_done, d.stream));
        d.last.fd_kernel = used_fd;
        d.last.numbers = (uint64_t)(bounds[i + 1] - bounds[i]);
        d.last.launches = 1;
    }
    std::vector<uint64_t> total(base + 1, 0);
    std::vector<Entry> all;
    for (size_t i = 0; i < nd; i++) {
        Device &d = ctx->devs[i];
        if (bounds[i] >= bounds[i + 1]) continue;
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(hipEventSynchronize(d.ev_done));
        d.state_dirty = false;  // the epilogue zeroed the state block
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, d.ev0, d.ev1));
        d.last.kernel_ms = ms;
        uint32_t cnt = (uint32_t)d.h_fin[129];
        if (cnt > d.list_cap) {
            // Near-miss list overflowed (e.g. out-of-range n, SURVEY hazard 9):
            // grow to the exact count and redo this shard.
            int rc = ensure_list(d, cnt);
            if (rc) return rc;
            d.state_dirty = true;
            bool used_fd = false;
            uint64_t fdc = 0;
            rc = enqueue_detailed(d, bounds[i], bounds[i + 1], base, used_fd, fdc);
            if (rc) return rc;
            HIPCHK(nice::launch_detailed_finish(d.d_hist, d.d_count, d.d_fin, d.stream));
            HIPCHK(hipStreamSynchronize(d.stream));
            d.state_dirty = false;
            cnt = (uint32_t)d.h_fin[129];
            if (cnt > d.list_cap) return fail(NICE_ERR_HIP, "near-miss list overflow after resize");
        }
        for (uint32_t b = 0; b <= base; b++) total[b] += d.h_fin[b];
        if (cnt) {
            std::vector<uint64_t> nbuf((size_t)cnt * 2);
            std::vector<uint32_t> ubuf(cnt);
            HIPCHK(hipMemcpy(nbuf.data(), d.d_list_n, (size_t)cnt * 16, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ubuf.data(), d.d_list_u, (size_t)cnt * 4, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < cnt; q++) all.push_back({mk(nbuf[2 * q], nbuf[2 * q + 1]), ubuf[q]});
        }
    }
    std::memcpy(hist, total.data(), (base + 1) * 8);
    // Self-check: the server's submit invariants (api/src/main.rs:309-359)
    // before anything is returned.
    int rc = validate_detailed(base, size, total.data(), all.size(), [&](size_t i) { return all[i]; });
    if (rc) return rc;
    if (!all.empty()) {
        // ... and its last one: every listed number's unique count recomputed
        // by the generic per-n device function (full square / cube + digit
        // scan, a different code path from the FD kernel that listed it).
        Device &d = ctx->devs[0];
        HIPCHK(hipSetDevice(d.id));
        const size_t n = all.size();
        std::vector<uint64_t> pairs(2 * n);
        for (size_t i = 0; i < n; i++) {
            pairs[2 * i] = lo64(all[i].n);
            pairs[2 * i + 1] = hi64(all[i].n);
        }
        uint64_t *dn = nullptr;
        uint32_t *du = nullptr;
        HIPCHK(hipMalloc(&dn, n * 16));
        HIPCHK(hipMalloc(&du, n * 4));
        std::vector<uint32_t> u(n);
        hipError_t err = hipMemcpyAsync(dn, pairs.data(), n * 16, hipMemcpyHostToDevice, d.stream);
        if (err == hipSuccess) err = nice::launch_unique_counts(dn, (uint32_t)n, base, du, d.stream);
        if (err == hipSuccess) err = hipMemcpyAsync(u.data(), du, n * 4, hipMemcpyDeviceToHost, d.stream);
        if (err == hipSuccess) err = hipStreamSynchronize(d.stream);
        (void)hipFree(dn);
        (void)hipFree(du);
        if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("self-check: ") + hipGetErrorString(err));
        for (size_t i = 0; i < n; i++)
            if (u[i] != all[i].u)
                return fail(NICE_ERR_HIP, "self-check: unique count of a listed number does not recompute");
    }
    return emit_list(all, out, cap, n_out);
}

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
    HIPCHK(nice::launch_unique_counts(dn, count, base, du, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
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
    HIPCHK(nice::launch_is_nice(dn, count, base, du, d.stream));
    HIPCHK(hipStreamSynchronize(d.stream));
    HIPCHK(hipMemcpy(out, du, (size_t)count * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dn));
    HIPCHK(hipFree(du));
    return NICE_OK;
}

int nice_check_is_nice_inrange(uint32_t base, uint64_t lo, uint64_t hi) {
    u128 rs, re;
    const u128 n = mk(lo, hi);
    if (!nice::fd2_supported(base) || nice::base_range_cached(base, rs, re) != 1 || n < rs || n >= re)
        return fail(NICE_ERR_INVALID, "n outside the base's valid range (or base not 40/50/80)");
    switch (base) {
    case 40: return nice::is_nice_fast<40>(lo, hi) ? 1 : 0;
    case 50: return nice::is_nice_fast<50>(lo, hi) ? 1 : 0;
    default: return nice::is_nice_fast<80>(lo, hi) ? 1 : 0;
    }
}

int nice_check_msd_skippable_inrange(uint32_t base, uint64_t slo, uint64_t shi, uint64_t elo,
                                     uint64_t ehi) {
    u128 rs, re;
    const u128 s = mk(slo, shi), e = mk(elo, ehi);
    if (!nice::fd2_supported(base) || nice::base_range_cached(base, rs, re) != 1 || s < rs || e > re || s >= e)
        return fail(NICE_ERR_INVALID, "range outside the base's valid range (or base not 40/50/80)");
    if (e - s == 1) return 0;  // a single number is never skipped (msd_prefix_filter.rs:395)
    const u128 l = e - 1;
    const uint64_t llo = lo64(l), lhi = hi64(l);
    switch (base) {
    case 40: return nice::msd_skippable_fast<40>(slo, shi, llo, lhi) ? 1 : 0;
    case 50: return nice::msd_skippable_fast<50>(slo, shi, llo, lhi) ? 1 : 0;
    default: return nice::msd_skippable_fast<80>(slo, shi, llo, lhi) ? 1 : 0;
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

int nice_process_range_niceonly_ex(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                   uint64_t end_lo, uint64_t end_hi, uint32_t base,
                                   const nice_niceonly_opts *opts, nice_number *out, size_t cap,
                                   size_t *n_out, nice_niceonly_stats *stats) {
    using clock = std::chrono::steady_clock;
    const auto t0 = clock::now();
    if (!ctx) return fail(NICE_ERR_INVALID, "null ctx");
    if (base < 3 || base > 128) return fail(NICE_ERR_INVALID, "base must be in 3..=128");
    const u128 s = mk(start_lo, start_hi), e = mk(end_lo, end_hi);
    if (s >= e)
        return fail(NICE_ERR_INVALID, "Range has invalid bounds, range_start must be < range_end");
    nice_niceonly_stats st{};
    uint64_t floor_size = opts && opts->msd_floor ? opts->msd_floor : env_msd_floor();
    if (!floor_size) floor_size = 250;
    const uint32_t k = opts && opts->stride_k ? opts->stride_k : 2;
    int threads = opts && opts->threads > 0 ? opts->threads : (int)std::thread::hardware_concurrency();
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

    std::lock_guard<std::mutex> lock(ctx->mu);
    if (nice::residue_filter(base).empty() || mine == 0) {  // client_process_gpu.rs:525-531
        if (stats) *stats = st;
        if (n_out) *n_out = 0;
        return NICE_OK;
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
        HIPCHK(hipMemsetAsync(d.d_count + 1, 0, 4, d.stream));
        int rc = ensure_list(d, kNiceCap);
        if (rc) return rc;
    }

    // Device MSD: batches of this caller's chunks, each run as init + the
    // level kernels + the candidate kernel, all stream-ordered (no host sync
    // until the end).  Batches alternate over the context's devices.
    auto run_device = [&]() -> int {
        if (chunk > ((u128)1 << 40)) return fail(NICE_ERR_INVALID, "device MSD: chunk_size too large");
        if ((e - s) >> 63) return fail(NICE_ERR_INVALID, "device MSD: field larger than 2^63");
        const uint64_t cnk = (uint64_t)chunk;
        // Nodes per level and leaves per batch are <= batch / floor + chunks
        // (every split child holds >= floor numbers); size batches for 2^24.
        const uint64_t fl = std::min<uint64_t>(floor_size, 1ull << 30);
        uint64_t cpb = std::max<uint64_t>(1, (fl << 24) / cnk);
        cpb = std::min(cpb, mine);
        const uint64_t batch_n = cpb * cnk;
        uint64_t per = std::min<uint64_t>(batch_n / fl + cpb, cpb << 22) + 64;
        per = std::min<uint64_t>(per, 1ull << 26);
        // leaf records: one per range plus one per kLeafPiece candidates
        const uint64_t leaf_cap = std::min<uint64_t>(per + (batch_n / nice::kLeafPiece) + 64, 0xffffffffull);
        for (auto &d : ctx->devs) {
            HIPCHK(hipSetDevice(d.id));
            int r = ensure_msd(d, (uint32_t)per, (uint32_t)leaf_cap);
            if (r) return r;
            HIPCHK(hipMemsetAsync(d.msd.counters, 0, 32 * 4, d.stream));
        }
        const uint64_t nbatches = (mine + cpb - 1) / cpb;
        for (uint64_t bi = 0; bi < nbatches; bi++) {
            Device &d = ctx->devs[bi % ctx->devs.size()];
            HIPCHK(hipSetDevice(d.id));
            if (bi >= ctx->devs.size())  // first batch per device: zeroed above
                HIPCHK(hipMemsetAsync(d.msd.counters, 0, 25 * 4, d.stream));
            nice::MsdLaunch mp{};
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
            mp.q[0] = d.msd.q[0];
            mp.q[1] = d.msd.q[1];
            mp.counters = d.msd.counters;
            mp.q_cap = d.msd.q_cap;
            mp.leaves = d.msd.leaves;
            mp.leaf_cap = d.msd.leaf_cap;
            mp.residues = d.residues[base * 8 + k];
            mp.ranks = d.ranks[base * 8 + k];
            mp.R = R;
            mp.M = (uint32_t)M;
            mp.base = base;
            mp.in_range = in_range;
#ifdef NICE_PROBES
            mp.probe = getenv("NICE_MSD_PROBE") ? (uint32_t)atoi(getenv("NICE_MSD_PROBE")) : 0u;
#endif
            hipError_t err = nice::launch_msd_device(mp, d.num_cus, d.stream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("msd launch: ") + hipGetErrorString(err));
            nice::NiceonlyLaunch p{};
            p.leaves = d.msd.leaves;
            p.n_leaves_dev = d.msd.counters + 24;
            p.n_leaves = d.msd.leaf_cap;  // clamp for the device count
            p.residues = mp.residues;
            p.R = R;
            p.M = (uint32_t)M;
            p.base = base;
            p.in_range = in_range;
            p.out = nice::NumOut{d.d_list_n, nullptr, d.d_count + 1, d.list_cap};
            err = nice::launch_niceonly(p, d.num_cus, d.stream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("niceonly launch: ") + hipGetErrorString(err));
            st.launches++;
        }
        for (auto &d : ctx->devs) {
            HIPCHK(hipSetDevice(d.id));
            HIPCHK(hipMemcpyAsync(d.msd.h_counters, d.msd.counters, 32 * 4, hipMemcpyDeviceToHost,
                                  d.stream));
            HIPCHK(hipStreamSynchronize(d.stream));
            const uint32_t *c = d.msd.h_counters;
#ifdef NICE_PROBES
            if (getenv("NICE_MSD_TRACE")) {  // level sizes of the last batch (diagnostics)
                fprintf(stderr, "msd levels:");
                for (int lv = 0; lv < 24; lv++) fprintf(stderr, " %u", c[lv]);
                fprintf(stderr, " | ranges %u\n", c[26]);
            }
#endif
            if (c[25])
                return fail(NICE_ERR_CAPACITY, "device MSD queue overflow (msd_floor too small for "
                                               "chunk_size); use msd_where = host");
            uint64_t cand, nums;
            std::memcpy(&cand, c + 28, 8);
            std::memcpy(&nums, c + 30, 8);
            st.ranges += c[26];
            st.candidates += cand;
            st.range_numbers += nums;
        }
        return NICE_OK;
    };

    const int where = opts ? opts->msd_where : NICE_MSD_AUTO;
    if (where < NICE_MSD_AUTO || where > NICE_MSD_DEVICE) return fail(NICE_ERR_INVALID, "bad msd_where");
    const bool on_device = where == NICE_MSD_DEVICE ||
                           (where == NICE_MSD_AUTO && k == 2 && !((e - s) >> 63) && chunk <= ((u128)1 << 40));
    int rc = NICE_OK;
    if (on_device) {
        rc = run_device();
    } else {
        // Producer: worker threads run the MSD filter per chunk and hand the
        // surviving ranges to this thread in chunk batches.
        std::atomic<uint64_t> next{0};
        std::mutex qmu;
        std::condition_variable qcv;
        std::deque<std::vector<std::pair<u128, u128>>> queue;
        const int n_workers = (int)std::min<uint64_t>(threads, mine);
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
            Device &d = ctx->devs[dev_rr++ % ctx->devs.size()];
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
                                  d.stream));
            nice::NiceonlyLaunch p{};
            p.leaves = b.d;
            p.n_leaves_dev = nullptr;
            p.n_leaves = nr;
            p.residues = d.residues[base * 8 + k];
            p.R = R;
            p.M = (uint32_t)M;
            p.base = base;
            p.in_range = in_range;
            p.out = nice::NumOut{d.d_list_n, nullptr, d.d_count + 1, d.list_cap};
            hipError_t err = nice::launch_niceonly(p, d.num_cus, d.stream);
            if (err != hipSuccess) return fail(NICE_ERR_HIP, std::string("niceonly launch: ") + hipGetErrorString(err));
            HIPCHK(hipEventRecord(b.done, d.stream));
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
    }
    if (rc) return rc;

    std::vector<Entry> all;
    for (auto &d : ctx->devs) {
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(hipMemcpyAsync(d.h_count + 1, d.d_count + 1, 4, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        for (auto &b : d.desc) b.pending = false;
        uint32_t cnt = d.h_count[1];
        if (cnt > d.list_cap)
            return fail(NICE_ERR_HIP, "niceonly output buffer overflow: " + std::to_string(cnt) +
                                          " (this strongly suggests a kernel bug)");
        if (cnt) {
            std::vector<uint64_t> nbuf((size_t)cnt * 2);
            HIPCHK(hipMemcpy(nbuf.data(), d.d_list_n, (size_t)cnt * 16, hipMemcpyDeviceToHost));
            for (uint32_t q = 0; q < cnt; q++) all.push_back({mk(nbuf[2 * q], nbuf[2 * q + 1]), base});
        }
    }
    st.total_seconds = std::chrono::duration<double>(clock::now() - t0).count();
    if (stats) *stats = st;
    return emit_list(all, out, cap, n_out);
}

int nice_process_range_niceonly(nice_ctx *ctx, uint64_t start_lo, uint64_t start_hi,
                                uint64_t end_lo, uint64_t end_hi, uint32_t base, nice_number *out,
                                size_t cap, size_t *n_out) {
    return nice_process_range_niceonly_ex(ctx, start_lo, start_hi, end_lo, end_hi, base, nullptr,
                                          out, cap, n_out, nullptr);
}

}  // extern "C"
