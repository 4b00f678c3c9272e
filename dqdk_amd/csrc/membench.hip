/*
 * membench.hip -- the two measured bounds SURVEY §8(d) prices the path
 * against on the same GPU, in the same process as the path itself:
 *
 *  - a streaming-read kernel (16-B buffer loads, XCD-interleaved grid-stride,
 *    one xor-reduced word per block written) -> the practical HBM read rate
 *    that rx_decode's roofline fraction is also quoted against;
 *  - a random u32 atomic-increment kernel over a histogram-sized table
 *    (one device atomic per key, no batch logic) -> the bound of the
 *    per-event histogram accumulation (src/tristan.c:243).
 *
 * Measurement helpers only: nothing on the receive path calls them.
 */
#include <errno.h>

#include "../../include/dqdk_gpu.h"
#include <hip/hip_runtime.h>

namespace {

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// 16-B streaming load (nontemporal: the bytes are used once)
__device__ __forceinline__ uint4 ld_nt16(const uint4* p)
{
    const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* __restrict__ p, uint64_t n16, uint32_t* out)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = ld_nt16(p + i);
        const uint4 b = ld_nt16(p + i + stride);
        const uint4 c = ld_nt16(p + i + 2 * stride);
        const uint4 d = ld_nt16(p + i + 3 * stride);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n16; i += stride) {
        const uint4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9e3779b9u)  // practically never; keeps the loads live
        out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void random_atomic_kernel(uint32_t* __restrict__ table, const uint32_t* __restrict__ keys,
                                                            uint64_t nkeys, uint64_t entries)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nkeys; i += stride) {
        const uint32_t k = keys[i];
        if (k < entries)
            __hip_atomic_fetch_add(table + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int timed(hipStream_t s, int iters, float* ms, void (*launch)(hipStream_t, const void*), const void* ctx)
{
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess)
        return -EIO;
    if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return -EIO;
    }
    launch(s, ctx);  // warm-up
    (void)hipEventRecord(a, s);
    for (int k = 0; k < iters; k++)
        launch(s, ctx);
    (void)hipEventRecord(b, s);
    hipError_t e = hipEventSynchronize(b);
    if (e == hipSuccess)
        e = hipEventElapsedTime(ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return e == hipSuccess ? 0 : -EIO;
}

struct ReadCtx {
    const uint4* p;
    uint64_t n16;
    uint32_t* out;
    uint32_t grid;
};

struct AtomicCtx {
    uint32_t* table;
    const uint32_t* keys;
    uint64_t nkeys, entries;
    uint32_t grid;
};

void launch_read(hipStream_t s, const void* c)
{
    const ReadCtx* r = (const ReadCtx*)c;
    hipLaunchKernelGGL(stream_read_kernel, dim3(r->grid), dim3(256), 0, s, r->p, r->n16, r->out);
}

void launch_atomic(hipStream_t s, const void* c)
{
    const AtomicCtx* r = (const AtomicCtx*)c;
    hipLaunchKernelGGL(random_atomic_kernel, dim3(r->grid), dim3(256), 0, s, r->table, r->keys, r->nkeys, r->entries);
}

uint32_t cu_count()
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? (uint32_t)cus : 256u;
}

}  // namespace

extern "C" {

int dqdk_gpu_membench_read(const void* d_buf, uint64_t bytes, void* stream, int iters, double* ms_per_pass)
{
    if (!d_buf || bytes < 16 || iters <= 0 || !ms_per_pass || ((uintptr_t)d_buf & 15))
        return -EINVAL;
    uint32_t* out = nullptr;
    const uint32_t grid = cu_count() * 8u;
    if (hipMalloc(&out, grid * sizeof(uint32_t)) != hipSuccess)
        return -ENOMEM;
    ReadCtx c{(const uint4*)d_buf, bytes / 16, out, grid};
    float ms = 0.f;
    int rc = timed((hipStream_t)stream, iters, &ms, launch_read, &c);
    (void)hipFree(out);
    *ms_per_pass = (double)ms / iters;
    return rc;
}

int dqdk_gpu_membench_atomic(uint32_t* d_table, uint64_t entries, const uint32_t* d_keys, uint64_t nkeys, void* stream,
                             int iters, double* ms_per_pass)
{
    if (!d_table || !d_keys || !nkeys || iters <= 0 || !ms_per_pass)
        return -EINVAL;
    AtomicCtx c{d_table, d_keys, nkeys, entries, cu_count() * 8u};
    float ms = 0.f;
    int rc = timed((hipStream_t)stream, iters, &ms, launch_atomic, &c);
    *ms_per_pass = (double)ms / iters;
    return rc;
}

}  // extern "C"
