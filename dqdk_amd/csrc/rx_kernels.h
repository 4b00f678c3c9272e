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
 * K3 rx_histo   : histogram accumulation of the keys of accounted OK frames
 *                 (relaxed atomic increment, src/tristan.c:243).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqdk_gpu.h"

namespace dqdk {

constexpr int kTile = 256;          // frames per K1 tile = threads per block
constexpr int kWaves = kTile / 64;  // waves per block
constexpr int kUnroll = 4;          // 1-KiB windows in flight per wave in phase B

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
    uint64_t* batch_scratch;  // [0] = first abort idx, [1..16] = per-batch counters
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
    uint32_t* hist;
};

__global__ void rx_decode_kernel(RxArgs a);
__global__ void rx_abort_kernel(CountArgs a);
__global__ void rx_count_kernel(CountArgs a);
__global__ void rx_histo_kernel(HistoArgs a);

}  // namespace dqdk
