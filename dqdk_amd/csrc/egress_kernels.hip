/*
 * egress_kernels.hip -- histogram egress on the GPU.
 *
 * tristan_fini (src/tristan.c:197-216) walks the 2.38 GB table on the host
 * and dprintf()s "%d,%d,%u,%u\n" = channel, histogram, energy bin, count for
 * every non-zero bin in table order.  Here the table never leaves HBM: for
 * each chunk of bins the GPU
 *   csv_len     -- counts the characters of every line a 4096-bin block
 *                  will emit (one 64-B row of 16 bins per thread),
 *   csv_scan    -- exclusive-scans the block totals (one block),
 *   csv_write   -- re-reads its bins, block-scans the per-thread lengths
 *                  and writes the formatted lines at their final offsets,
 * so only the CSV text crosses PCIe.  Plus the end-of-run merge helpers
 * (u32-wrapping add of another table, non-zero count).
 */
#include "egress_kernels.h"

namespace dqdk {

namespace {

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// 16-B streaming load (nontemporal: the bytes are used once)
__device__ __forceinline__ uint4 ld_nt16(const uint4* p)
{
    const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t ndigits(uint32_t v)
{
    return 1u + (v >= 10u) + (v >= 100u) + (v >= 1000u) + (v >= 10000u) + (v >= 100000u) + (v >= 1000000u) +
           (v >= 10000000u) + (v >= 100000000u) + (v >= 1000000000u);
}

// "%d,%d,%u,%u\n" of flat bin k = (channel*6 + histogram)*65536 + energy
__device__ __forceinline__ uint32_t line_len(uint64_t k, uint32_t freq)
{
    const uint32_t ch = (uint32_t)(k / (6u * 65536u));
    const uint32_t e = (uint32_t)(k & 0xFFFFu);
    return ndigits(ch) + 1u + 1u + 1u + ndigits(e) + 1u + ndigits(freq) + 1u;
}

__device__ __forceinline__ char* put_u32(char* p, uint32_t v)
{
    const uint32_t n = ndigits(v);
    for (uint32_t d = n; d-- > 0;) {
        p[d] = (char)('0' + v % 10u);
        v /= 10u;
    }
    return p + n;
}

// Bin values [first, first + 16) of the table (value = base + low byte;
// first is a multiple of 16).
__device__ __forceinline__ void load_row(const uint32_t* hist, const uint8_t* lo, uint64_t first, uint64_t end,
                                         uint32_t v[kCsvBinsPerThread])
{
    if (first + kCsvBinsPerThread <= end) {
        const uint4* p = (const uint4*)(hist + first);
#pragma unroll
        for (int j = 0; j < kCsvBinsPerThread / 4; j++) {
            const uint4 x = ld_nt16(p + j);
            v[4 * j] = x.x;
            v[4 * j + 1] = x.y;
            v[4 * j + 2] = x.z;
            v[4 * j + 3] = x.w;
        }
        const uint4 b = ld_nt16((const uint4*)(lo + first));
        const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < kCsvBinsPerThread; j++)
            v[j] += (bw[j >> 2] >> (8 * (j & 3))) & 0xffu;
    } else {
#pragma unroll
        for (int j = 0; j < kCsvBinsPerThread; j++)
            v[j] = first + j < end ? hist[first + j] + lo[first + j] : 0u;
    }
}

// (callers that scan more than once per launch barrier between the scans:
// lds_wave is rewritten by the next one)
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T* lds_wave, T* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T t = __shfl_up(incl, o);
        if (lane >= o)
            incl += t;
    }
    if (lane == 63)
        lds_wave[w] = incl;
    __syncthreads();
    T base = 0, all = 0;
    for (int j = 0; j < (int)(blockDim.x >> 6); j++) {
        if (j < w)
            base += lds_wave[j];
        all += lds_wave[j];
    }
    *total = all;
    return base + incl - x;
}

}  // namespace

__global__ __launch_bounds__(kCsvThreads) void csv_len_kernel(const uint32_t* __restrict__ hist,
                                                             const uint8_t* __restrict__ lo, uint64_t base, uint64_t end,
                                                             uint64_t* __restrict__ blk_chars)
{
    __shared__ uint64_t lds[kCsvThreads / 64];
    const uint64_t first = base + ((uint64_t)blockIdx.x * kCsvThreads + threadIdx.x) * kCsvBinsPerThread;
    uint32_t v[kCsvBinsPerThread];
    uint64_t chars = 0;
    if (first < end) {
        load_row(hist, lo, first, end, v);
#pragma unroll
        for (int j = 0; j < kCsvBinsPerThread; j++)
            chars += v[j] ? line_len(first + j, v[j]) : 0u;
    }
    uint64_t total;
    (void)block_excl_scan<uint64_t>(chars, lds, &total);
    if (threadIdx.x == 0)
        blk_chars[blockIdx.x] = total;
}

// One block: in-place exclusive scan of nblk u64 block totals; [nblk] = grand total.
__global__ __launch_bounds__(1024) void csv_scan_kernel(uint64_t* __restrict__ blk_chars, uint32_t nblk)
{
    __shared__ uint64_t lds[16];
    uint64_t carry = 0;
    for (uint32_t c = 0; c < nblk; c += blockDim.x) {
        const uint32_t i = c + threadIdx.x;
        const uint64_t x = i < nblk ? blk_chars[i] : 0u;
        uint64_t total;
        const uint64_t ex = block_excl_scan<uint64_t>(x, lds, &total);
        if (i < nblk)
            blk_chars[i] = carry + ex;
        carry += total;
        __syncthreads();  // every wave has read lds before the next chunk's scan rewrites it
    }
    if (threadIdx.x == 0)
        blk_chars[nblk] = carry;
}

__global__ __launch_bounds__(kCsvThreads) void csv_write_kernel(const uint32_t* __restrict__ hist,
                                                               const uint8_t* __restrict__ lo, uint64_t base, uint64_t end,
                                                               const uint64_t* __restrict__ blk_off, char* __restrict__ out)
{
    __shared__ uint64_t lds[kCsvThreads / 64];
    const uint64_t first = base + ((uint64_t)blockIdx.x * kCsvThreads + threadIdx.x) * kCsvBinsPerThread;
    uint32_t v[kCsvBinsPerThread];
    uint64_t chars = 0;
    if (first < end) {
        load_row(hist, lo, first, end, v);
#pragma unroll
        for (int j = 0; j < kCsvBinsPerThread; j++)
            chars += v[j] ? line_len(first + j, v[j]) : 0u;
    }
    uint64_t total;
    const uint64_t off = blk_off[blockIdx.x] + block_excl_scan<uint64_t>(chars, lds, &total);
    if (!chars)
        return;
    char* p = out + off;
#pragma unroll 1
    for (int j = 0; j < kCsvBinsPerThread; j++) {
        if (!v[j])
            continue;
        const uint64_t k = first + j;
        const uint32_t ch = (uint32_t)(k / (6u * 65536u));
        const uint32_t h = (uint32_t)((k >> 16) % 6u);
        p = put_u32(p, ch);
        *p++ = ',';
        *p++ = (char)('0' + h);
        *p++ = ',';
        p = put_u32(p, (uint32_t)(k & 0xFFFFu));
        *p++ = ',';
        p = put_u32(p, v[j]);
        *p++ = '\n';
    }
}

// ---- raw payload stream -------------------------------------------------------
// Bytes frame i contributes: its datalen if it is an accounted OK frame (the
// frames process_frame hands to tristan_process, src/dqdk.c:243-247) whose
// payload lies inside the UMEM; 0 otherwise.  A u32-wrapped datalen (udplen
// < 8, src/dqdk.c:205) would make the reference write() ~4 GB from the frame
// and fail; such frames contribute nothing here.
__device__ __forceinline__ uint64_t raw_bytes(const RawArgs& a, uint32_t i, uint32_t limit, uint64_t* src)
{
    if (i >= limit)
        return 0;
    const dqdk_gpu_rx_result_t r = a.res[i];
    if (r.status != DQDK_RX_OK)
        return 0;
    const uint64_t p = a.desc[i].addr + r.payload_off;
    if (p > a.umem_size || r.datalen > a.umem_size - p)
        return 0;
    *src = p;
    return r.datalen;
}

__device__ __forceinline__ uint32_t raw_limit(const RawArgs& a)
{
    const uint64_t abort_idx = a.batch_scratch[0];
    return (a.flags & DQDK_GPU_F_BATCH_ABORT) ? (uint32_t)(abort_idx < a.n ? abort_idx : a.n) : a.n;
}

__global__ __launch_bounds__(kRawThreads) void raw_len_kernel(RawArgs a)
{
    __shared__ uint64_t lds[kRawThreads / 64];
    const uint32_t i = blockIdx.x * kRawThreads + threadIdx.x;
    uint64_t src = 0;
    const uint64_t b = raw_bytes(a, i, min(raw_limit(a), a.n), &src);
    uint64_t total;
    (void)block_excl_scan<uint64_t>(b, lds, &total);
    if (threadIdx.x == 0)
        a.blk[blockIdx.x] = total;
}

// One wave per frame of the block: 4-B output words, each assembled from two
// aligned source words with alignbyte; the partial words at both ends of a
// frame's output are written bytewise (they are shared with the neighbours).
__global__ __launch_bounds__(kRawThreads) void raw_copy_kernel(RawArgs a)
{
    __shared__ uint64_t lds[kRawThreads / 64];
    __shared__ uint64_t s_off[kRawThreads], s_src[kRawThreads];
    __shared__ uint32_t s_len[kRawThreads];
    const uint32_t i = blockIdx.x * kRawThreads + threadIdx.x;
    uint64_t src = 0;
    const uint64_t b = raw_bytes(a, i, min(raw_limit(a), a.n), &src);
    uint64_t total;
    const uint64_t off = a.blk[blockIdx.x] + block_excl_scan<uint64_t>(b, lds, &total);
    s_off[threadIdx.x] = off;
    s_src[threadIdx.x] = src;
    s_len[threadIdx.x] = (uint32_t)b;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int f = w; f < kRawThreads; f += kRawThreads / 64) {
        const uint64_t D = s_off[f], S = s_src[f];
        uint64_t len = s_len[f];
        if (D >= a.out_cap)
            continue;
        if (len > a.out_cap - D)
            len = a.out_cap - D;
        if (!len)
            continue;
        // a buffer resource per frame, based 16 B below the payload (the first
        // word may start up to 3 B before it) and ending at the UMEM end: every
        // offset stays far below num_records wherever the payload sits in the
        // UMEM (payloads past 2 GiB included); a payload longer than that
        // (u32-wrapped datalen in a > 2 GiB UMEM) takes plain loads
        // (readfirstlane: f is wave-uniform, so the SRD is scalar -- no waterfall loop)
        const uint64_t rb0 = S >= 16 ? (S - 16) & ~15ull : 0ull;
        const uint64_t rb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rb0) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(rb0 >> 32)) << 32);
        const uint64_t room = a.umem_size - rb;
        const bool use_rs = len + 32 <= 0x7fffffffull;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.umem + rb), (short)0,
            __builtin_amdgcn_readfirstlane((int)(room > 0x7fffffffull ? 0x7fffffffull : room)), 0x00020000);
        const uint64_t E = D + len;
        const uint64_t k0 = D >> 2, k1 = (E + 3) >> 2;  // output words touched
        for (uint64_t k = k0 + lane; k < k1; k += 64) {
            const uint64_t d = k << 2;        // first byte of the word
            const int64_t s = (int64_t)S + (int64_t)(d - D);  // source of byte d (may precede S for k0)
            const uint64_t sa = (uint64_t)(s & ~3ll);
            const uint32_t sh = (uint32_t)(s & 3);
            uint32_t w0, w1;
            if (use_rs) {
                w0 = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(sa - rb), 0, 0);
                w1 = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(sa - rb) + 4u, 0, 0);
            } else {
                w0 = *(const uint32_t*)(a.umem + sa);
                w1 = sa + 8 <= a.umem_size ? *(const uint32_t*)(a.umem + sa + 4) : 0u;
            }
            const uint32_t v = __builtin_amdgcn_alignbyte(w1, w0, sh);
            if (d >= D && d + 4 <= E) {
                *(uint32_t*)(a.out + d) = v;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (d + j >= D && d + j < E)
                        a.out[d + j] = (uint8_t)(v >> (8 * j));
            }
        }
    }
}

// ---- async consumer ------------------------------------------------------------
// One wave per burst: the histogram loop of tristan_process runs `ret` times
// over the SAME buffer (src/tristan.c:314-315), i.e. every in-bounds event of
// the burst's first payload adds ret to its bin; total_events += E once,
// total_bytes += len * ret (u32 product, :327-328).
__global__ __launch_bounds__(256) void async_histo_kernel(AsyncArgs a)
{
    const int lane = threadIdx.x & 63;
    const uint32_t k = (blockIdx.x * 256 + threadIdx.x) >> 6;
    if (k >= a.nbursts)
        return;
    const uint32_t first = a.burst[4 * k], ret = a.burst[4 * k + 1];
    if (ret == 0)
        return;
    uint32_t oob = 0;
    if (a.histo) {
        const uint32_t* ev = (const uint32_t*)(a.ring + (uint64_t)first * a.payloadsz);
        for (uint32_t e = lane; e < a.E; e += 64) {
            const uint32_t w0 = ev[4 * e], w1 = ev[4 * e + 1], w2 = ev[4 * e + 2];
            const uint32_t ch = w0 >> 16;                 // bytes 2-3 (struct energy_evt, src/tristan.h:13-25)
            const uint32_t bin = (w1 >> 8) & 0xffffu;     // energy:24 >> 8 (bytes 5-6)
            const uint32_t hc = w2 & 7u;                  // hist_class:3 (byte 8)
            if (ch >= DQDK_TRISTAN_CHANNELS || hc >= DQDK_TRISTAN_HISTS) {  // histogram_event :236-241
                oob++;
                continue;
            }
            __hip_atomic_fetch_add(&a.hist[(ch * DQDK_TRISTAN_HISTS + hc) * DQDK_TRISTAN_BINS + bin], ret,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            oob += __shfl_xor(oob, o);
    }
    if (lane == 0) {
        atomicAdd(&a.cum[6], (unsigned long long)a.E);                  // total_events
        atomicAdd(&a.cum[7], (unsigned long long)(uint32_t)(a.len * ret));  // total_bytes
        if (oob)
            atomicAdd(&a.cum[8], (unsigned long long)oob * ret);       // one log line per call per event
    }
}

// One block per burst: write(rawdata_fd, buffer, len * ret) (src/tristan.c:319)
// -- the first len * ret bytes of the burst's elements, dword-aligned.
__global__ __launch_bounds__(256) void async_raw_kernel(AsyncArgs a)
{
    const uint32_t k = blockIdx.x;
    const uint32_t first = a.burst[4 * k], ret = a.burst[4 * k + 1];
    // output offset: the bytes of bursts 0..k-1 (a multiple of 4)
    const uint64_t o4 = ((uint64_t)a.burst[4 * k + 2] | ((uint64_t)a.burst[4 * k + 3] << 32)) / 4;
    const uint64_t n4 = (uint64_t)(a.len * ret) / 4;
    const uint32_t* src = (const uint32_t*)(a.ring + (uint64_t)first * a.payloadsz);
    uint32_t* dst = (uint32_t*)a.out;
    for (uint64_t i = threadIdx.x; i < n4; i += 256)
        if (4 * (o4 + i) + 4 <= a.out_cap)
            dst[o4 + i] = src[i];
}

__global__ __launch_bounds__(256) void hist_add_kernel(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        uint4 a = ((const uint4*)dst)[i];
        const uint4 b = ld_nt16((const uint4*)src + i);
        a.x += b.x;  // u32 wrap, like the shared relaxed-atomic table
        a.y += b.y;
        a.z += b.z;
        a.w += b.w;
        ((uint4*)dst)[i] = a;
    }
}

__global__ __launch_bounds__(256) void hist_nonzero_kernel(const uint32_t* __restrict__ hist, const uint8_t* __restrict__ lo,
                                                          uint64_t n16, unsigned long long* __restrict__ count)
{
    __shared__ uint32_t lds[4];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        uint32_t v[16];
        load_row(hist, lo, 16 * i, 16 * i + 16, v);
#pragma unroll
        for (int j = 0; j < 16; j++)
            c += v[j] != 0u;
    }
    uint32_t total;
    (void)block_excl_scan<uint32_t>(c, lds, &total);
    if (threadIdx.x == 0 && total)
        atomicAdd(count, (unsigned long long)total);
}

// out[bin] = base[bin] + low[bin] for bins [16 * i0, 16 * i1) (the u32 table view).
__global__ __launch_bounds__(256) void hist_combine_kernel(const uint32_t* __restrict__ hist, const uint8_t* __restrict__ lo,
                                                          uint64_t i0, uint64_t i1, uint32_t* __restrict__ out)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < i1; i += stride) {
        uint32_t v[16];
        load_row(hist, lo, 16 * i, 16 * i + 16, v);
        uint4* o = (uint4*)(out + 16 * (i - i0));
#pragma unroll
        for (int j = 0; j < 4; j++)
            o[j] = make_uint4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    }
}

}  // namespace dqdk
