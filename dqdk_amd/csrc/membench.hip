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

// The receive path's memory pattern without its arithmetic: one wave per
// frame reads the frame's first `fbytes` (16-B loads, frames at `stride`) and
// writes `obytes` per frame contiguously (the decoded records), each word
// derived from the loaded data so neither side is dead.
__global__ __launch_bounds__(256) void frames_pattern_kernel(const uint8_t* __restrict__ umem, uint64_t stride,
                                                              uint32_t fbytes, uint32_t n, uint32_t* __restrict__ out,
                                                              uint32_t obytes, int wide)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    const uint32_t nch = (fbytes + 15) / 16, nwords = obytes / 4;
    for (uint32_t f = blockIdx.x * 4 + (threadIdx.x >> 6); f < n; f += nw) {
        const uint4* src = (const uint4*)(umem + (uint64_t)f * stride);
        uint32_t acc = f;
        for (uint32_t c = lane; c < nch; c += 64) {
            const uint4 a = src[c];
            acc ^= a.x ^ a.y ^ a.z ^ a.w;
        }
        if (out && wide) {  // 16-B stores (frames' record rows are contiguous: 4 words per lane)
            uint32_t* o = out + (uint64_t)f * nwords;
            for (uint32_t k = 4 * lane; k < nwords; k += 256) {
                if (k + 4 <= nwords && (((uintptr_t)(o + k)) & 15) == 0)
                    *(u32x4_t*)(o + k) = u32x4_t{acc + k, acc + k + 1, acc + k + 2, acc + k + 3};
                else
                    for (uint32_t m = k; m < k + 4 && m < nwords; m++)
                        o[m] = acc + m;
            }
        } else if (out) {
            uint32_t* o = out + (uint64_t)f * nwords;
            for (uint32_t k = lane; k < nwords; k += 64)
                o[k] = acc + k;
        } else if (acc == 0x9e3779b9u) {
            ((uint32_t*)umem)[0] = acc;  // practically never; keeps the loads live
        }
    }
}

// The same bytes moved with the most memory-level parallelism a plain kernel
// gets: a flat grid-stride walk over every 16-B chunk of every frame (four
// independent nontemporal loads in flight per lane) and, per four chunks
// read, one coalesced 16-B store into the records array (out16 chunks in
// all, the path's 4 E : frame-bytes ratio within a few percent).
__global__ __launch_bounds__(256) void frames_flat_kernel(const uint8_t* __restrict__ umem, uint64_t stride,
                                                           uint32_t cpf, uint32_t n, uint32_t* __restrict__ out,
                                                           uint64_t out16)
{
    const uint64_t total = (uint64_t)cpf * n;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t it = 0, g = t0; g < total; g += 4 * step, it++) {
        u32x4_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t gg = g + u * step;
            const uint32_t f = (uint32_t)gg / cpf, c = (uint32_t)gg - f * cpf;  // total < 2^32 (checked)
            v[u] = gg < total ? __builtin_nontemporal_load((const u32x4_t*)(umem + (uint64_t)f * stride + 16u * c))
                              : u32x4_t{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        const uint64_t w = it * step + t0;  // consecutive lanes, consecutive 16-B slots
        if (out && w < out16)
            ((u32x4_t*)out)[w] = u32x4_t{acc, acc + 1, acc + 2, acc + 3};
    }
    if (!out && acc == 0x9e3779b9u)
        ((uint32_t*)umem)[0] = acc;
}

// Plain copy with the same read:write ratio as the path but no frames:
// read 4 x 16 B per lane, write 16 B, all contiguous (the HBM rate for a
// 4:1 read:write mix).
__global__ __launch_bounds__(256) void mix41_kernel(const u32x4_t* __restrict__ src, uint64_t n16,
                                                     u32x4_t* __restrict__ dst)
{
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t it = 0, g = t0; g + 3 * step < n16; g += 4 * step, it++) {
        const u32x4_t a = __builtin_nontemporal_load(src + g);
        const u32x4_t b = __builtin_nontemporal_load(src + g + step);
        const u32x4_t c = __builtin_nontemporal_load(src + g + 2 * step);
        const u32x4_t d = __builtin_nontemporal_load(src + g + 3 * step);
        dst[it * step + t0] = a ^ b ^ c ^ d;
    }
}

// Plain 1:1 copy, 16 B per lane, four loads in flight (the guide's float4 copy).
__global__ __launch_bounds__(256) void copy11_kernel(const u32x4_t* __restrict__ src, uint64_t n16,
                                                      u32x4_t* __restrict__ dst)
{
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g + 3 * step < n16; g += 4 * step) {
        const u32x4_t a = src[g], b = src[g + step], c = src[g + 2 * step], d = src[g + 3 * step];
        dst[g] = a;
        dst[g + step] = b;
        dst[g + 2 * step] = c;
        dst[g + 3 * step] = d;
    }
}

// Write calibration for rocprofv3's WRITE_SIZE (MI355X_MICROARCH.md: exact
// only for 16-B-per-lane streaming stores): 4-B-per-lane stores of a known
// byte count.  runs == 0: every wave instruction writes 64 consecutive dwords
// (256 B, line-aligned); runs > 0: the fused decode's piece-flush shape --
// each wave instruction writes a run of `runs` (< 64) dwords starting at a
// dword offset that is not line-aligned, runs of one block following each
// other inside a private region (as a piece fills over rounds).
// Bytes written = n * (runs ? runs : 64) * 4.
__global__ __launch_bounds__(256) void store_b32_kernel(uint32_t* __restrict__ out, uint32_t n, uint32_t runs)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    const uint32_t w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t per = runs ? runs : 64u;
    // wave w writes instructions w, w + nw, ... ; with runs its instructions'
    // runs are adjacent in its own region (a piece), starting 13 dwords in
    const uint64_t region = ((uint64_t)(n / nw + 1) * per + 64) & ~31ull;
    uint64_t cur = runs ? (uint64_t)w0 * region + 13 : 0;
    for (uint32_t i = w0; i < n; i += nw) {
        const uint64_t o = runs ? cur : (uint64_t)i * 64;
        if (lane < per)
            out[o + lane] = i ^ lane;  // plain stores, as the piece flush
        cur += per;
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

struct FramesCtx {
    const uint8_t* umem;
    uint64_t stride;
    uint32_t fbytes, n;
    uint32_t* out;
    uint32_t obytes, grid;
    int flat, wide;
};

void launch_frames(hipStream_t s, const void* c)
{
    const FramesCtx* r = (const FramesCtx*)c;
    if (r->flat == 5)
        hipLaunchKernelGGL(store_b32_kernel, dim3(r->grid), dim3(256), 0, s, r->out, r->n, r->obytes / 4u);
    else if (r->flat == 4)
        hipLaunchKernelGGL(copy11_kernel, dim3(r->grid), dim3(256), 0, s, (const u32x4_t*)r->umem,
                           (uint64_t)r->n * r->stride / 16u, (u32x4_t*)r->out);
    else if (r->flat == 3)
        hipLaunchKernelGGL(mix41_kernel, dim3(r->grid), dim3(256), 0, s, (const u32x4_t*)r->umem,
                           (uint64_t)r->n * r->stride / 16u, (u32x4_t*)r->out);
    else if (r->flat == 1)
        hipLaunchKernelGGL(frames_flat_kernel, dim3(r->grid), dim3(256), 0, s, r->umem, r->stride, r->fbytes / 16u, r->n,
                           r->out, (uint64_t)r->n * r->obytes / 16u);
    else
        hipLaunchKernelGGL(frames_pattern_kernel, dim3(r->grid), dim3(256), 0, s, r->umem, r->stride, r->fbytes, r->n,
                           r->out, r->obytes, r->wide);
}

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

int dqdk_gpu_membench_frames(const void* d_umem, uint64_t stride, uint32_t frame_bytes, uint32_t n, void* d_out,
                             uint32_t out_bytes_per_frame, int flat, void* stream, int iters, double* ms_per_pass)
{
    if (flat == 5) {  // write calibration: no frames read (d_umem unused)
        if (!d_out || !n || out_bytes_per_frame > 252 || (out_bytes_per_frame & 3) || ((uintptr_t)d_out & 255) ||
            iters <= 0 || !ms_per_pass)
            return -EINVAL;
        FramesCtx c{nullptr, 0, 0, n, (uint32_t*)d_out, out_bytes_per_frame, cu_count() * 8u, 5, 0};
        float ms = 0.f;
        int rc = timed((hipStream_t)stream, iters, &ms, launch_frames, &c);
        *ms_per_pass = (double)ms / iters;
        return rc;
    }
    if (!d_umem || !n || stride < frame_bytes || (stride & 15) || (frame_bytes & 15) || ((uintptr_t)d_umem & 15) ||
        ((uintptr_t)d_out & 15) || iters <= 0 || !ms_per_pass || (out_bytes_per_frame & 3))
        return -EINVAL;
    if ((uint64_t)(frame_bytes / 16) * n >= (1ull << 32))
        return -EINVAL;
    const uint32_t grid = cu_count() * 8u;
    FramesCtx c{(const uint8_t*)d_umem, stride, frame_bytes, n, (uint32_t*)d_out, out_bytes_per_frame, grid,
                flat >= 3 ? flat : (flat & 1), flat == 2};
    float ms = 0.f;
    int rc = timed((hipStream_t)stream, iters, &ms, launch_frames, &c);
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
