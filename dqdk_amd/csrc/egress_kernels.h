/* egress_kernels.h -- histogram egress / merge kernels (egress_kernels.hip). */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dqdk {

constexpr int kCsvThreads = 256;
constexpr int kCsvBinsPerThread = 16;                         // one 64-B row per thread
constexpr int kCsvBinsPerBlock = kCsvThreads * kCsvBinsPerThread;  // 4096
constexpr uint64_t kCsvChunkBins = 1ull << 22;                // 4M bins (16 MB of table) per chunk
constexpr uint32_t kCsvChunkBlocks = (uint32_t)(kCsvChunkBins / kCsvBinsPerBlock);  // 1024
constexpr uint64_t kCsvMaxLine = 4 + 1 + 1 + 1 + 5 + 1 + 10 + 1;  // "1511,5,65535,4294967295\n"

__global__ void csv_len_kernel(const uint32_t* hist, uint64_t base, uint64_t end, uint64_t* blk_chars);
__global__ void csv_scan_kernel(uint64_t* blk_chars, uint32_t nblk);
__global__ void csv_write_kernel(const uint32_t* hist, uint64_t base, uint64_t end, const uint64_t* blk_off, char* out);
__global__ void hist_add_kernel(uint32_t* dst, const uint32_t* src, uint64_t n16);
__global__ void hist_nonzero_kernel(const uint32_t* hist, uint64_t n16, unsigned long long* count);

}  // namespace dqdk
