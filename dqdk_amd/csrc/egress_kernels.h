/* egress_kernels.h -- histogram egress / merge kernels (egress_kernels.hip). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqdk_gpu.h"

namespace dqdk {

constexpr int kCsvThreads = 256;
constexpr int kCsvBinsPerThread = 16;                         // one 64-B row per thread
constexpr int kCsvBinsPerBlock = kCsvThreads * kCsvBinsPerThread;  // 4096
constexpr uint64_t kCsvChunkBins = 1ull << 22;                // 4M bins (16 MB of table) per chunk
constexpr uint32_t kCsvChunkBlocks = (uint32_t)(kCsvChunkBins / kCsvBinsPerBlock);  // 1024
constexpr uint64_t kCsvMaxLine = 4 + 1 + 1 + 1 + 5 + 1 + 10 + 1;  // "1511,5,65535,4294967295\n"

// The table is value = hist[bin] + lo[bin] (rx_kernels.h): every reader takes both planes.
__global__ void csv_len_kernel(const uint32_t* hist, const uint8_t* lo, uint64_t base, uint64_t end, uint64_t* blk_chars);
__global__ void csv_scan_kernel(uint64_t* blk_chars, uint32_t nblk);
__global__ void csv_write_kernel(const uint32_t* hist, const uint8_t* lo, uint64_t base, uint64_t end, const uint64_t* blk_off,
                                 char* out);
// Raw payload stream (tristan_process write(), src/tristan.c:318-324)
constexpr int kRawThreads = 256;  // frames per block in the scan passes
struct RawArgs {
    const uint8_t* umem;
    uint64_t umem_size;
    const dqdk_gpu_desc_t* desc;
    const dqdk_gpu_rx_result_t* res;
    uint32_t n;
    uint32_t flags;
    const uint64_t* batch_scratch;  // [0] = first abort index of the batch
    uint64_t* blk;                  // [nblk + 1] block byte totals -> offsets, [nblk] = total
    uint8_t* out;
    uint64_t out_cap;
};
__global__ void raw_len_kernel(RawArgs a);
__global__ void raw_copy_kernel(RawArgs a);

// Async consumer (async_processor, src/tristan.c:332-375): burst k of the
// ring = elements [first[k], first[k] + ret[k]); tristan_process(buffer,
// len, ret) histograms the burst's FIRST payload ret times and write()s the
// burst buffer's first len * ret bytes.
struct AsyncArgs {
    const uint8_t* ring;   // nelem elements of payloadsz bytes (payloadsz % 4 == 0)
    uint32_t payloadsz;
    uint32_t E;            // events per payload (get_energy_events_count)
    uint32_t len;          // strip_wfm ? 16 : payloadsz (src/tristan.c:343)
    uint32_t nbursts;
    const uint32_t* burst; // [4 * nbursts]: first element, ret, output byte offset (lo, hi)
    int histo;
    uint32_t* hist;        // the table's u32 base plane
    uint8_t* out;          // raw stream (nullable)
    uint64_t out_cap;
    unsigned long long* cum;  // dqdk_gpu_counters_t words (total_events, total_bytes, oob_events)
};
__global__ void async_histo_kernel(AsyncArgs a);
__global__ void async_raw_kernel(AsyncArgs a);

__global__ void hist_add_kernel(uint32_t* dst, const uint32_t* src, uint64_t n16);
__global__ void hist_nonzero_kernel(const uint32_t* hist, const uint8_t* lo, uint64_t n16, unsigned long long* count);
__global__ void hist_combine_kernel(const uint32_t* hist, const uint8_t* lo, uint64_t i0, uint64_t i1, uint32_t* out);

}  // namespace dqdk
