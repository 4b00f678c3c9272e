/*
 * rx_kernels.h -- gfx950 kernels of the receive hot path.
 *
 * K1 rx_decode  : per 256-frame tile, phase A = one lane per frame parses
 *                 the Eth/IPv4/UDP headers (get_udp_payload, src/dqdk.c:185-207,
 *                 + ip4_audit_checksum src/tcpip/ipv4.c:6-11 in the checksum
 *                 config), phase B = one wave per frame streams the frame
 *                 with aligned 16-B buffer loads, folds the UDP checksum
 *                 (udp_audit_checksum/udp_csum, src/tcpip/udp.c:10-20,
 *                 inet_csum.c:184-216) and decodes every 16-B energy event
 *                 into a 4-B flat histogram key (histogram_event,
 *                 src/tristan.c:233-245).
 * K2 rx_abort / rx_count : per-batch counters of fetch_xsk (src/dqdk.c:252-322)
 *                 under per-packet or batch-abort accounting.
 * K3 histogram accumulation of the keys of accounted OK frames (the relaxed
 *    atomic increment of src/tristan.c:243), two interchangeable forms:
 *    - rx_histo_atomic: one device-scope atomic per event (small batches);
 *    - partitioned: rx_part1 (keys -> 284 buckets of 2^21 bins, long runs),
 *      rx_part2 (each 16K-key chunk of a bucket sorted by 16K-bin slice in
 *      LDS, written back as u16 slice-local keys + run offsets),
 *      rx_slice_histo (gathers the slice's runs, packed-u16 LDS histogram,
 *      one coalesced read-modify-write of the slice's 16 KB low-byte plane,
 *      carries of 256 into the u32 base plane; slices with more than 65535
 *      events are listed and redone with u32 LDS bins by rx_slice_heavy).  The table is held as
 *      value = base[bin] + low[bin] (mod 2^32): the same values as the
 *      reference's u32 table, with a 4x smaller per-batch sweep.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqdk_gpu.h"

namespace dqdk {

constexpr int kTile = 256;          // frames per K1 tile = threads per block
constexpr int kWaves = kTile / 64;  // waves per block
constexpr int kUnroll = 4;          // 1-KiB windows in flight per wave in phase B

// Partitioned histogram geometry.  Keys < 1512*6*65536 = 594,542,592 < 2^30.
constexpr int kL1Shift = 21;                                // 2^21 bins (8 MB of table) per bucket
constexpr int kL1Buckets = 284;                             // ceil(594542592 / 2^21)
constexpr int kSliceBits = 14;                              // 2^14 bins per slice (32 KB packed-u16 LDS; 64 KB in the u32 form)
constexpr int kSubs = 1 << (kL1Shift - kSliceBits);         // 128 slices per bucket
constexpr int kSlices = kL1Buckets * kSubs;                 // 36352 (36288 used)
constexpr int kPartThreads = 1024;                          // part1/part2 block size
constexpr int kPartKeysPerThread = 16;
constexpr int kPartChunk = kPartThreads * kPartKeysPerThread;  // 16384 keys staged in LDS
constexpr int kSliceThreads = 512;
#ifndef DQDK_P1_KEYS
#define DQDK_P1_KEYS 32
#endif
#ifndef DQDK_P1_THREADS
#define DQDK_P1_THREADS 1024
#endif
constexpr int kP1Threads = DQDK_P1_THREADS;                 // part1 block size
constexpr int kP1Keys = DQDK_P1_KEYS;                       // keys per thread
constexpr int kP1Chunk = kP1Threads * kP1Keys;              // keys staged in LDS per block
constexpr int kP1BlocksPerCu = kP1Chunk * 4 > 80 * 1024 ? 1 : 2;  // a 128-KB stage leaves room for one block
constexpr int kP1MinWaves = kP1Threads / 64 * kP1BlocksPerCu / 4;  // waves per SIMD
constexpr uint32_t kBucketAlign = 8;  // bucket starts in part1/part2 rounded to 8 keys (16-B part2 stores)
constexpr uint32_t kStagePad = kL1Buckets * kBucketAlign;  // extra part1/part2 entries for that padding

// u32 scratch words used by the partitioned histogram
constexpr int kOffCnt1 = 0;         // [kL1Buckets + 1] keys per bucket (decode; upper bound)  -- zeroed per batch
constexpr int kOffCur1 = 288;       // [kL1Buckets] keys written per bucket (part1 cursors)   -- zeroed per batch
constexpr int kOffHeavyN = 574;     // slices listed for the u32 slice form                    -- zeroed per batch
constexpr int kZeroWords = 576;
constexpr int kOffOff1 = 576;       // [kL1Buckets + 1] bucket starts in part1/part2 (prep)
constexpr int kOffIstart = 864;     // [kL1Buckets + 1] first part2 item of each bucket (prep)
constexpr int kOffHeavy = 1152;     // [kSlices] slices with > 65535 events this batch
constexpr int kHistScratchWords = kOffHeavy + kSlices;
constexpr int kItemOffs = kSubs + 1;  // u16 run offsets per part2 item (one 16K-key chunk of a bucket)

struct RxArgs {
    const uint8_t* umem;
    uint64_t umem_size;
    const dqdk_gpu_desc_t* desc;
    uint32_t n;
    dqdk_gpu_rx_result_t* res;
    uint32_t* keys;
    uint32_t E;
    uint32_t flags;
    uint32_t port_start, port_end;
    int histo;                // the mode keeps a histogram (is_store_histo, src/tristan.c:65-70)
    uint64_t* batch_scratch;  // [0] = first abort idx, [1..12] = per-batch counters
    uint32_t* cnt1;           // partitioned histogram: bucket counts (+ KEY_NONE records for non-OK frames), or null
};

struct CountArgs {
    const dqdk_gpu_rx_result_t* res;
    uint32_t n;
    uint32_t E;
    uint32_t flags;
    int histo;
    uint64_t* batch_scratch;
    dqdk_gpu_counters_t* cum;
};

struct HistoArgs {
    const dqdk_gpu_rx_result_t* res;
    const uint32_t* keys;
    uint32_t n;
    uint32_t E;
    uint32_t flags;
    const uint64_t* batch_scratch;
    uint32_t* hist;     // table base plane (u32 per bin): the atomic path and carries add here
    uint8_t* lo;        // table low-byte plane: the partitioned path's per-batch sweep
                        // (bin value = hist[bin] + lo[bin], mod 2^32)
    uint32_t* scratch;  // kHistScratchWords
    uint32_t* part1;    // n*E keys grouped by bucket
    uint16_t* part2;    // n*E slice-local keys (key & 16383), each 16K chunk of a bucket sorted by slice
    uint16_t* runs;     // [items][kItemOffs] slice run starts inside each chunk
    // the slice pass runs over nslots staged batches: batch k's scratch,
    // part2 keys and run offsets sit k strides (elements) after the first
    uint32_t nslots;
    uint32_t scratch_stride;
    uint64_t part2_stride, runs_stride;
};

__global__ void rx_decode_kernel(RxArgs a);
__global__ void rx_abort_kernel(CountArgs a);
__global__ void rx_count_kernel(CountArgs a);
__global__ void rx_histo_atomic_kernel(HistoArgs a);
__global__ void rx_part1_kernel(HistoArgs a);
__global__ void rx_hist_prep_kernel(HistoArgs a);
__global__ void rx_part2_kernel(HistoArgs a);
__global__ void rx_slice_histo_kernel(HistoArgs a);
__global__ void rx_slice_heavy_kernel(HistoArgs a);

}  // namespace dqdk
