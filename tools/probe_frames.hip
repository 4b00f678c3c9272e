// probe_frames.hip -- memory-pattern probe for the rx_decode design (not on
// the receive path).  Reads n frames of L bytes at `stride` (as rx_decode
// does, 16-B buffer loads) and optionally writes one dword per chunk read
// (the decoded-record stream, ~4 B per 16-B event), in these shapes:
//
//   perframe  one wave per 64-frame tile, each frame rounded up to whole
//             2-KiB windows (lane = two 16-B chunks 1 KiB apart): rx_decode's
//             current phase-B shape
//   packed    the same tile, but the tile's chunks form one dense stream:
//             a window carries the tail of one frame and the head of the next
//   flat      the whole batch as one grid-stride chunk stream
//
// x ring depth (windows in flight per wave), x grid (one tile per wave vs a
// persistent grid of resident waves walking the tiles in order).
// Prints one line per variant: GB/s of (n*L read + records written).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe_frames tools/probe_frames.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint64_t bytes)
{
    const uint64_t b = (uint64_t)p;
    const uint64_t ub = (uint64_t)rfl((uint32_t)b) | ((uint64_t)rfl((uint32_t)(b >> 32)) << 32);
    const uint32_t nrec = rfl((uint32_t)(bytes > 0x7fffffffull ? 0x7fffffffull : bytes));
    return __builtin_amdgcn_make_buffer_rsrc((void*)ub, (short)0, (int)nrec, 0x00020000);
}

constexpr uint32_t kOOB = 0x80000000u;

struct P {
    const uint8_t* umem;
    uint64_t stride;
    uint32_t L, nch, n, tile;
    uint32_t* out;
    int write;
    int persistent;
};

// chunk stream position s of a tile -> (frame, chunk) ; perframe: s = w*128 + slot
template <int RING, bool PACKED>
__global__ __launch_bounds__(256) void tile_kernel(P p)
{
    const int lane = threadIdx.x & 63;
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t gw = blockIdx.x * 4 + wave, nw = gridDim.x * 4;
    const uint32_t ntiles = (p.n + p.tile - 1) / p.tile;
    const uint32_t wpf = (p.nch + 127) / 128;  // perframe: windows per frame
    uint32_t acc = lane;
    for (uint32_t t = gw; t < ntiles; t += nw) {
        const uint32_t f0 = t * p.tile;
        const uint32_t nf = min(p.tile, p.n - f0);
        const uint64_t base = (uint64_t)f0 * p.stride;
        const __amdgpu_buffer_rsrc_t rs = rsrc(p.umem + base, (uint64_t)nf * p.stride);
        const __amdgpu_buffer_rsrc_t ws = rsrc(p.out + (uint64_t)f0 * p.nch, p.write ? (uint64_t)nf * p.nch * 4 : 0);
        const uint32_t nwin = PACKED ? (nf * p.nch + 127) / 128 : nf * wpf;
        auto off = [&](uint32_t w, uint32_t half) -> uint32_t {
            uint32_t fr, ch;
            if (PACKED) {
                const uint32_t s = w * 128 + half * 64 + lane;
                fr = s / p.nch;
                ch = s - fr * p.nch;
                if (fr >= nf)
                    return kOOB;
            } else {
                fr = w / wpf;
                ch = (w - fr * wpf) * 128 + half * 64 + lane;
                if (ch >= p.nch)
                    return kOOB;
            }
            return fr * (uint32_t)p.stride + ch * 16;
        };
        auto woff = [&](uint32_t w, uint32_t half) -> uint32_t {
            if (PACKED)
                return (w * 128 + half * 64 + lane) * 4;
            const uint32_t fr = w / wpf, ch = (w - fr * wpf) * 128 + half * 64 + lane;
            return ch < p.nch ? (fr * p.nch + ch) * 4 : kOOB;
        };
        u32x4 b0[RING], b1[RING];
#pragma unroll
        for (int d = 0; d < RING; d++) {
            const uint32_t w = d;
            b0[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, w < nwin ? off(w, 0) : kOOB, 0, 0);
            b1[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, w < nwin ? off(w, 1) : kOOB, 0, 0);
        }
        for (uint32_t k = 0; k < nwin; k += RING) {
#pragma unroll
            for (int d = 0; d < RING; d++) {
                const uint32_t w = k + d;
                const uint32_t x0 = b0[d].x ^ b0[d].y ^ b0[d].z ^ b0[d].w;
                const uint32_t x1 = b1[d].x ^ b1[d].y ^ b1[d].z ^ b1[d].w;
                acc += x0 ^ x1;
                if (p.write == 1 || p.write == 3) {
                    const int aux = p.write == 3 ? 2 : 0;
                    if (aux) {
                        __builtin_amdgcn_raw_buffer_store_b32(x0 + acc, ws, w < nwin ? woff(w, 0) : kOOB, 0, 2);
                        __builtin_amdgcn_raw_buffer_store_b32(x1 + acc, ws, w < nwin ? woff(w, 1) : kOOB, 0, 2);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b32(x0 + acc, ws, w < nwin ? woff(w, 0) : kOOB, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b32(x1 + acc, ws, w < nwin ? woff(w, 1) : kOOB, 0, 0);
                    }
                } else if (p.write) {
                    // the same bytes as 16-B stores from every 4th lane (keys gathered by DPP)
                    const uint32_t y1 = __builtin_amdgcn_mov_dpp((int)x0, 0x55, 0xf, 0xf, false);  // quad_perm [1,1,1,1]
                    const uint32_t y2 = __builtin_amdgcn_mov_dpp((int)x0, 0xaa, 0xf, 0xf, false);
                    const uint32_t y3 = __builtin_amdgcn_mov_dpp((int)x0, 0xff, 0xf, 0xf, false);
                    const uint32_t z1 = __builtin_amdgcn_mov_dpp((int)x1, 0x55, 0xf, 0xf, false);
                    const uint32_t z2 = __builtin_amdgcn_mov_dpp((int)x1, 0xaa, 0xf, 0xf, false);
                    const uint32_t z3 = __builtin_amdgcn_mov_dpp((int)x1, 0xff, 0xf, 0xf, false);
                    const bool q = (lane & 3) == 0;
                    const uint32_t o0 = w < nwin && q ? woff(w, 0) : kOOB, o1 = w < nwin && q ? woff(w, 1) : kOOB;
                    const u32x4 v0 = {x0 + acc, y1, y2, y3}, v1 = {x1 + acc, z1, z2, z3};
                    if (p.write == 4) {
                        __builtin_amdgcn_raw_buffer_store_b128(v0, ws, o0, 0, 2);
                        __builtin_amdgcn_raw_buffer_store_b128(v1, ws, o1, 0, 2);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b128(v0, ws, o0, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(v1, ws, o1, 0, 0);
                    }
                }
                const uint32_t wn = w + RING;
                b0[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, wn < nwin ? off(wn, 0) : kOOB, 0, 0);
                b1[d] = __builtin_amdgcn_raw_buffer_load_b128(rs, wn < nwin ? off(wn, 1) : kOOB, 0, 0);
            }
        }
    }
    if (acc == 0x9e3779b9u && p.out)
        p.out[0] = acc;
}

// whole batch as one chunk stream, grid-stride, 4 chunks in flight per lane
__global__ __launch_bounds__(256) void flat_kernel(P p)
{
    const uint64_t total = (uint64_t)p.nch * p.n;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t g = t0; g < total; g += 4 * step) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t gg = g + u * step;
            const uint32_t f = (uint32_t)(gg / p.nch), c = (uint32_t)(gg - (uint64_t)f * p.nch);
            v[u] = gg < total ? *(const u32x4*)(p.umem + (uint64_t)f * p.stride + 16u * c) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t x = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
            acc += x;
            const uint64_t gg = g + u * step;
            if (p.write && gg < total)
                p.out[gg] = x + acc;
        }
    }
    if (acc == 0x9e3779b9u && p.out)
        p.out[0] = acc;
}

template <typename K>
float time_kernel(K k, uint32_t grid, const P& p, int iters)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, p);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, p);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char** argv)
{
    const uint32_t L = argc > 1 ? atoi(argv[1]) : 1500;
    const uint64_t stride = argc > 2 ? atoll(argv[2]) : 4096;
    const uint32_t n = argc > 3 ? atoi(argv[3]) : (1u << 20);
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* umem;
    uint32_t* out;
    const uint32_t nch = (L + 15) / 16;
    CK(hipMalloc(&umem, (uint64_t)n * stride + 4096));
    CK(hipMalloc(&out, (uint64_t)n * nch * 4 + 4096));
    CK(hipMemset(umem, 0x5a, (uint64_t)n * stride + 4096));
    P p{umem, stride, L, nch, n, 64, out, 0, 0};
    const double rbytes = (double)n * L;
    const double wbytes = (double)n * nch * 4;
    const uint32_t ntiles = (n + 63) / 64;
    printf("L=%u stride=%lu n=%u cus=%d\n", L, (unsigned long)stride, n, cus);
    for (int write = 0; write < 5; write++) {
        p.write = write;
        const double bytes = rbytes + (write ? wbytes : 0);
        auto run = [&](const char* name, auto k, uint32_t grid) {
            const float ms = time_kernel(k, grid, p, 10);
            printf("%-28s write=%d grid=%6u  %.4f ms  %7.1f GB/s\n", name, write, grid, ms, bytes / (ms * 1e-3) / 1e9);
            fflush(stdout);
        };
        const uint32_t g1 = (ntiles + 3) / 4;  // one tile per wave
        for (uint32_t occ : {0u, 4u}) {
            const uint32_t grid = occ ? cus * occ : g1;
            char nm[64];
            snprintf(nm, sizeof nm, "perframe r4 %s", occ ? "pers" : "1tile");
            run(nm, tile_kernel<4, false>, grid);
            snprintf(nm, sizeof nm, "packed r4 %s", occ ? "pers" : "1tile");
            run(nm, tile_kernel<4, true>, grid);
            snprintf(nm, sizeof nm, "packed r8 %s", occ ? "pers" : "1tile");
            run(nm, tile_kernel<8, true>, grid);
        }
        if (write <= 1)
            run("flat", flat_kernel, cus * 8);
    }
    return 0;
}
