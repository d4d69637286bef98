// Launch-overhead floor on gfx950: HIP-event time of kernels that do no work
// but have the small-field fd2 launch geometry, so the event-measured kernel
// time of a 1e6 field can be split into "what any launch of this shape
// costs" and "what the fd2 kernel itself adds".
//   hipcc --offload-arch=gfx950 -O3 -o launch_floor launch_floor.hip && ./launch_floor
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

template <int LDS>
__global__ void empty_kernel(uint32_t *out) {
    __shared__ uint32_t s[LDS / 4 > 0 ? LDS / 4 : 1];
    if (LDS > 0) s[threadIdx.x % (LDS / 4 > 0 ? LDS / 4 : 1)] = threadIdx.x;
    if (out && threadIdx.x == 0 && blockIdx.x == 0xffffffffu) out[0] = s[0];
}

// The same, plus the fd2 finish pattern's cost: every workgroup one agent
// atomic, the last one to arrive writes one word to mapped host memory.
__global__ void arrive_kernel(uint32_t *ctr, uint64_t *mapped) {
    __shared__ uint32_t last;
    if (threadIdx.x == 0) last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                                 gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {
        *ctr = 0;
        __hip_atomic_store(mapped, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// fd2's two-level arrival (nice_device.hpp last_block_arrive): 64 group
// counters, then one top counter; MODE 0: nothing after, 1: the last
// workgroup's relaxed mapped store, 2: its system-scope release store.
template <int MODE>
__global__ void arrive64_kernel(uint32_t *done, uint64_t *mapped) {
    __shared__ uint32_t last;
    if (threadIdx.x == 0) {
        const uint32_t g = blockIdx.x % 64, n = gridDim.x;
        const uint32_t expect = (n - 1 - g) / 64 + 1;
        bool l = false;
        if (atomicAdd(&done[1 + g], 1u) == expect - 1) l = atomicAdd(&done[0], 1u) == 63;
        last = l;
    }
    __syncthreads();
    if (last) {
        for (uint32_t w = threadIdx.x; w < 65; w += blockDim.x)
            __hip_atomic_store(&done[w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) {
            if (MODE == 1) __hip_atomic_store(mapped, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (MODE == 2) __hip_atomic_store(mapped, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Workgroup 0 alone stores to mapped memory (no arrival): MODE 1 relaxed,
// 2 release (system scope).
template <int MODE>
__global__ void store0_kernel(uint64_t *mapped) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (MODE == 1) __hip_atomic_store(mapped, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (MODE == 2) __hip_atomic_store(mapped, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <class F>
static void timeit(const char *name, F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> v;
    for (int r = 0; r < 25; r++) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 5) v.push_back(ms * 1000.f);
    }
    std::sort(v.begin(), v.end());
    printf("%-58s median %6.2f us  min %6.2f us\n", name, v[v.size() / 2], v[0]);
}

int main() {
    uint32_t *out = nullptr, *ctr = nullptr;
    uint64_t *mapped = nullptr;
    (void)hipMalloc(&out, 4);
    (void)hipMalloc(&ctr, 65 * 4);
    (void)hipMemset(ctr, 0, 65 * 4);
    (void)hipHostMalloc(&mapped, 8, hipHostMallocMapped);
    timeit("empty, 1 x 64", [&] { hipLaunchKernelGGL(empty_kernel<0>, dim3(1), dim3(64), 0, 0, out); });
    timeit("empty, 391 x 512, 54 KB LDS (b40 1e6 geometry)",
           [&] { hipLaunchKernelGGL(empty_kernel<54016>, dim3(391), dim3(512), 0, 0, out); });
    timeit("empty, 245 x 512, 131 KB LDS (b80 1e6 geometry)",
           [&] { hipLaunchKernelGGL(empty_kernel<131072>, dim3(245), dim3(512), 0, 0, out); });
    timeit("arrive + mapped release, 391 x 512",
           [&] { hipLaunchKernelGGL(arrive_kernel, dim3(391), dim3(512), 0, 0, ctr, mapped); });
    timeit("two-level arrive (64 groups), nothing after, 391 x 512",
           [&] { hipLaunchKernelGGL(arrive64_kernel<0>, dim3(391), dim3(512), 0, 0, ctr, mapped); });
    timeit("two-level arrive, last WG relaxed mapped store",
           [&] { hipLaunchKernelGGL(arrive64_kernel<1>, dim3(391), dim3(512), 0, 0, ctr, mapped); });
    timeit("two-level arrive, last WG release mapped store",
           [&] { hipLaunchKernelGGL(arrive64_kernel<2>, dim3(391), dim3(512), 0, 0, ctr, mapped); });
    timeit("WG 0 relaxed mapped store only, 391 x 512",
           [&] { hipLaunchKernelGGL(store0_kernel<1>, dim3(391), dim3(512), 0, 0, mapped); });
    timeit("WG 0 release mapped store only, 391 x 512",
           [&] { hipLaunchKernelGGL(store0_kernel<2>, dim3(391), dim3(512), 0, 0, mapped); });
    printf("rc=%d\n", (int)hipGetLastError());
    return 0;
}
