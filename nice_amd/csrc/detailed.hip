// detailed.hip -- gfx950 kernels for detailed field processing.
//
// Replaces the reference's detailed_kernel (common/src/cuda/nice_kernels.cu:
// 486-531) and the CPU loop it mirrors (common/src/client_process.rs:150-191):
// for every n in a segment, count the distinct base-b digits of n^2 and n^3,
// histogram the counts and list the near-misses (count > cutoff).
//
// This file: the generic kernel.  Segments inside a base's valid range run
// the finite-difference kernel instead (fd2_kernel.hpp).
//
// detailed_generic_kernel  (any base 2..128, any n < 2^128)
//   Per-n multiply + chunked radix extraction with a runtime base.  Used for
//   segments outside the valid range (e.g. the reference's b10 @ 1e6 GPU
//   test, client_process_gpu.rs:1485) and for bases without an FD instance.
#include "kernels.h"
#include "nice_device.hpp"

namespace nice {

// ---------------------------------------------------------------------------
// Generic per-n kernel (runtime base).
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256)
detailed_generic_kernel(u64 start_lo, u64 start_hi, u64 count, GenericBase g, u32 cutoff,
                        u64 *__restrict__ hist_out, NumOut out) {
    __shared__ u32 hist[4][129];
    const u32 tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (u32 i = tid; i < 4 * 129; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    for (u64 idx = (u64)blockIdx.x * 256 + tid; idx < count; idx += (u64)gridDim.x * 256) {
        u64 lo = start_lo, hi = start_hi;
        add_u128(lo, hi, idx);
        u32 u = unique_generic(lo, hi, g);
        atomicAdd(&hist[wave][u], 1u);
        if (u > cutoff) {
            u32 pos = atomicAdd(out.count, 1u);
            if (pos < out.cap) {
                out.n[2 * (u64)pos] = lo;
                out.n[2 * (u64)pos + 1] = hi;
                out.u[pos] = u;
            }
        }
    }
    __syncthreads();
    hist_out += (blockIdx.x % kHistCopies) * 129;
    for (u32 b = tid; b <= g.base; b += 256) {
        u32 s = hist[0][b] + hist[1][b] + hist[2][b] + hist[3][b];
        if (s) atomicAdd((unsigned long long *)&hist_out[b], (unsigned long long)s);
    }
    (void)lane;
}

// Diagnostics: per-n unique counts / nice flags through the device functions.
__global__ void unique_counts_kernel(const u64 *n_pairs, u32 count, GenericBase g, u32 *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = unique_generic(n_pairs[2 * i], n_pairs[2 * i + 1], g);
}

// Field epilogue: sum the kHistCopies histogram copies into `out` (129 bins,
// then the near-miss count at out[129]) and zero the copies and the counter
// for the next field.  `out` is mapped pinned host memory, so the host reads
// the result straight after its completion event: no memset and no DMA copy
// on the field's critical path.
__global__ void __launch_bounds__(1024) detailed_finish_kernel(u64 *__restrict__ hist, u32 *__restrict__ count,
                                                               u64 *__restrict__ out) {
    __shared__ u64 acc[129];
    const u32 t = threadIdx.x;
    if (t < 129) acc[t] = 0;
    __syncthreads();
    for (u32 e = t; e < kHistCopies * 129; e += blockDim.x) {
        const u64 v = hist[e];
        if (v) {
            atomicAdd((unsigned long long *)&acc[e % 129], (unsigned long long)v);
            hist[e] = 0;
        }
    }
    __syncthreads();
    if (t < 129) out[t] = acc[t];
    if (t == 129) {
        out[129] = *count;
        *count = 0;
    }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
hipError_t launch_detailed_finish(uint64_t *hist, uint32_t *count, uint64_t *out_mapped, hipStream_t s) {
    hipLaunchKernelGGL(detailed_finish_kernel, dim3(1), dim3(1024), 0, s, hist, count, out_mapped);
    return hipGetLastError();
}

hipError_t launch_detailed_generic(const DetailedLaunch &p, int num_cus, hipStream_t s) {
    GenericBase g = make_generic(p.base);
    u64 grid = (p.count + 255) / 256;
    u64 cap = (u64)num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(detailed_generic_kernel, dim3((u32)grid), dim3(256), 0, s, p.start_lo,
                       p.start_hi, p.count, g, p.cutoff, p.hist, p.out);
    return hipGetLastError();
}

hipError_t launch_unique_counts(const uint64_t *n_pairs, uint32_t count, uint32_t base,
                                uint32_t *out, hipStream_t s) {
    GenericBase g = make_generic(base);
    hipLaunchKernelGGL(unique_counts_kernel, dim3((count + 255) / 256), dim3(256), 0, s, n_pairs,
                       count, g, out);
    return hipGetLastError();
}

}  // namespace nice
