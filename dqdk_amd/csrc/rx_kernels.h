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
 *    - partitioned: keys grouped by L1 bucket of 2^21 bins (the fused decode's
 *      per-block pieces, or rx_part1 over frame-order records / the fused
 *      decode's overflow list), rx_part2 (each 16K-key chunk of a bucket
 *      sorted by 16K-bin slice in LDS, written as u16 slice-local keys + run
 *      offsets), rx_slice_histo (gathers the slice's runs over the staged
 *      batches, packed-u16 LDS histogram, one coalesced read-modify-write of
 *      the slice's 16 KB low-byte plane, carries of 256 into the u32 base
 *      plane; bins are drained into the base plane between groups of 65280
 *      events, so any spectrum fits the u16 bins).  The table is held as value =
 *      base[bin] + low[bin] (mod 2^32): the same values as the reference's
 *      u32 table, with a 4x smaller per-pass sweep.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dqdk_gpu.h"

namespace dqdk {

constexpr int kTile = 256;          // frames per K1 tile = threads per block
constexpr int kWaves = kTile / 64;  // waves per block
#ifndef DQDK_RINGW
#define DQDK_RINGW 4
#endif
constexpr int kRingW = DQDK_RINGW;  // 2-KiB windows in flight per wave in phase B
#ifndef DQDK_FRINGW
#define DQDK_FRINGW 4
#endif
constexpr int kFRingW = DQDK_FRINGW;  // the same for the fused decode (rounds are multiples of it)

// Partitioned histogram geometry.  Keys < 1512*6*65536 = 594,542,592 < 2^30.
constexpr int kL1Shift = 21;                                // 2^21 bins (8 MB of table) per bucket
constexpr int kL1Buckets = 284;                             // ceil(594542592 / 2^21)
constexpr int kSliceBits = 14;                              // 2^14 bins per slice (32 KB packed-u16 LDS)
constexpr int kSubs = 1 << (kL1Shift - kSliceBits);         // 128 slices per bucket
constexpr int kSlices = kL1Buckets * kSubs;                 // 36352 (36288 used)
constexpr int kPartThreads = 1024;                          // part1/part2 block size
#ifndef DQDK_P2_KPT
#define DQDK_P2_KPT 18
#endif
constexpr int kPartKeysPerThread = DQDK_P2_KPT;             // six key triples per lane (r06d: 15 -> 18)
static_assert(kPartKeysPerThread % 3 == 0, "a lane loads whole key triples");
#ifndef DQDK_P2_BPC
#define DQDK_P2_BPC 2
#endif
constexpr int kP2BlocksPerCu = DQDK_P2_BPC;                  // rx_part2 blocks per CU (its LDS allows two)
constexpr int kPartChunk = kPartThreads * kPartKeysPerThread;  // 18432 key slots staged in LDS (an item)
constexpr int kPartTriples = kPartChunk / 3;                // 6144 triples: a gathered item
#ifndef DQDK_SLICE_SPAN
#define DQDK_SLICE_SPAN 2
#endif
constexpr int kSliceSpan = DQDK_SLICE_SPAN;      // adjacent slices per slice-pass block (their runs are adjacent too)
constexpr int kSliceThreads = 512 * kSliceSpan;  // 32 waves per CU either way
constexpr int kSliceBlocks = kSlices / kSliceSpan;
constexpr int kSliceMaxSlots = 32;  // staged batches one slice pass can take
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
// the fused decode's overflow list: up to this many keys are added to the
// table by atomics in rx_part1, more are grouped into rx_part2 segments
#ifndef DQDK_OVF_ATOMIC_MAX
#define DQDK_OVF_ATOMIC_MAX 16384
#endif
constexpr uint32_t kOvfAtomicMax = DQDK_OVF_ATOMIC_MAX;
constexpr uint32_t kBucketAlign = 8;  // bucket starts in part1/part2 rounded to 8 keys (16-B part2 stores)
constexpr uint32_t kStagePad = kL1Buckets * kBucketAlign;  // extra part1/part2 entries for that padding

// u32 scratch words used by the partitioned histogram (one block per staged batch)
constexpr int kOffCnt1 = 0;         // [kL1Buckets + 1] keys per bucket: decode upper bound (records path) or
                                    //   overflow keys per bucket (fused path)                 -- zeroed per batch
constexpr int kOffCur1 = 288;       // [kL1Buckets] keys written per bucket by rx_part1         -- zeroed per batch
constexpr int kOffOvfN = 577;       // fused path: keys sent to the overflow list               -- zeroed per batch
constexpr int kOffFixN = 578;       // (retired in round 6: the fused decode takes back failed frames itself)
// fused path: each bucket's key triples over all its pieces (the decode's
// blocks add their pieces' by device atomics: rx_part2's segment sizes), one
// 128-B line per bucket: 256 blocks adding to words of a few shared lines
// serialise at the memory side (r06i: decode +12 %)               -- zeroed per batch
constexpr int kTotStride = 32;
constexpr int kOffPieceTotT = 608;  // [kL1Buckets] at stride kTotStride words
constexpr int kZeroWords = kOffPieceTotT + kL1Buckets * kTotStride;
constexpr int kMaxFusedGrid = 256;  // fused decode blocks (one per CU)
constexpr int kOffOff1 = kZeroWords;  // [kL1Buckets + 1] bucket starts of rx_part1's output (prep)
constexpr int kOffIstart = kOffOff1 + 288;  // [kL1Buckets + 1] first part2 item of each bucket; [284] = items (rx_part2)
// fused path: keys of each (bucket, block) piece [kL1Buckets][kMaxFusedGrid]
// (decode; rx_part2 scans a bucket's row into its pieces' starts per item)
constexpr int kOffPieceN = kOffIstart + 288;
constexpr int kOffEnd = kOffPieceN + kL1Buckets * kMaxFusedGrid;
static_assert(kOffFixN < kOffPieceTotT && kOffPieceTotT % kTotStride == 0 && kZeroWords % 16 == 0, "scratch layout");
static_assert(kOffPieceN % 4 == 0 && kMaxFusedGrid % 4 == 0, "rx_part2 loads a bucket's piece sizes 16 B at a time");
constexpr int kSegsPerBucket = 2;  // fused: the bucket's pieces (one gathered sequence), then rx_part1's overflow run
// items of a batch of nk keys: one per started chunk of each segment (a
// bucket's gathered triples number at most its keys / 3 + one per piece)
__host__ __device__ constexpr uint64_t max_items(uint64_t nk)
{
    return nk / kPartChunk + (uint64_t)kL1Buckets * (kSegsPerBucket + 1) + 1;
}
// u32 words of one staged slot's scratch
constexpr uint64_t kHistScratchWords = kOffEnd;
constexpr int kItemOffs = kSubs + 1;  // u16 run offsets per part2 item (one chunk of a segment)

// Fused decode (rx_decode_fused): 1024-thread blocks, one per CU, persistent.
// Keys of a round are counted into an LDS stage per L1 bucket (kFCap keys
// each), then appended to the block's piece of that bucket (a private
// region: no device atomics) as key triples: three 21-bit bucket-local keys
// per 8 bytes (k0 | k1 << 21 | k2 << 42; 2.67 B a key).  A round flushes
// whole triples (whole 128-B lines of 48 keys in the lines policy) and
// carries the rest; the last flush pads a piece's last triple, whose valid
// keys the piece size tells.  The fused region is [bucket][block][cap]: a
// bucket's pieces are adjacent, in block order.  Keys past kFCap in a round,
// or past a full piece, go to the block's overflow region (u32 keys), which
// rx_part1 groups afterwards.
constexpr int kFWaves = 16;
constexpr int kFThreads = kFWaves * 64;
// The frame's checksum tail is corrected in the window loop (no 16-KB
// per-frame tail copy in LDS): that room goes to the bucket stages, which
// hold their keys packed as the pieces do (three to an 8-B word): kFCapW
// words, kFCap keys per bucket.
constexpr int kFCapW = 66;
constexpr int kFCap = 3 * kFCapW;
constexpr uint32_t kTripleMask = (1u << kL1Shift) - 1;  // a bucket-local key
constexpr uint32_t kLineKeys = 48;                     // keys of one 128-B line of triples
struct FusedGeom {
    uint32_t grid;    // decode blocks
    uint32_t cap;     // keys per piece: 1.25x the block's uniform share + slack, whole 128-B lines of triples
    uint32_t words;   // u32 words per piece (cap * 2 / 3)
    uint64_t region;  // u32 words per bucket: grid pieces + 32
};
__host__ __device__ constexpr FusedGeom fused_geom(uint64_t n, uint64_t E, uint64_t cus)
{
    const uint64_t nsuper = (n + kFThreads - 1) / kFThreads;
    const uint64_t g0 = nsuper < cus ? nsuper : cus;
    const uint64_t grid = g0 < (uint64_t)kMaxFusedGrid ? (g0 ? g0 : 1) : (uint64_t)kMaxFusedGrid;
    const uint64_t spt = (nsuper + grid - 1) / grid;
    const uint64_t cap = ((spt * kFThreads * E * 5 / 4) / kL1Buckets + 64 + kLineKeys - 1) / kLineKeys * kLineKeys;
    const uint64_t words = cap / 3 * 2;
    return FusedGeom{(uint32_t)grid, (uint32_t)cap, (uint32_t)words, grid * words + 32};
}
// part1/part2 elements: the fused pieces, then rx_part1's output region
__host__ __device__ constexpr uint64_t part_elems(uint64_t nk, uint64_t fused_elems)
{
    return fused_elems + nk + kStagePad;
}

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
    // fused path (rx_decode_fused) only:
    uint32_t* scratch;        // the slot's histogram scratch (piece sizes, overflow / fixup counts)
    uint32_t* part1;          // pieces [bucket][block] of piece_cap keys (piece_words u32 words of triples)
    uint32_t piece_cap;
    uint32_t piece_words;
    uint64_t region;          // u32 words per bucket (fused_geom)
    uint32_t* ovf;            // overflow list (gridDim.x * ovf_blk_cap keys)
    uint32_t* ovf_blk;        // per-block private overflow regions (gridDim.x * ovf_blk_cap keys)
    uint32_t ovf_blk_cap;     // keys per region; past it (pathological spectra) a key is added to
    uint32_t* hist;           //   the table's base plane by a device atomic (exact: value = base + low)
    uint32_t ovf_list;        // overflow keys: 0 = to the table by device atomics at the block's end;
                              //   1 = to the overflow list (kOffCnt1 per bucket) for rx_part1's grouping
    uint32_t round_windows;   // windows per wave per round (multiple of the ring depth)
    uint32_t tile_frames;     // records path: frames per wave tile (0 = 64; fewer spread a small
                              //   batch over more waves, the host drop-in's zero-copy frames)
    // fused path, counters folded into the decode (no rx_abort / rx_count
    // launches; per-packet accounting only): the batch's accumulators
    // (kFoldWords u64, zero but the first-failure word, all ones, between
    // launches), the last block by ticket writes the batch's [first abort
    // idx, counters] to batch_scratch and adds them to cum
    uint32_t fold;
    uint32_t fmap;            // fused: 1 = interleaved frame map (see rx_decode_fused_kernel)
    uint32_t* blk_cnt;
    uint32_t* ticket;         // zero between launches
    dqdk_gpu_counters_t* cum;
};
constexpr int kFoldWords = 16;

struct CountArgs {
    const dqdk_gpu_rx_result_t* res;
    uint32_t n;
    uint32_t E;
    uint32_t flags;
    int histo;
    uint64_t* batch_scratch;
    dqdk_gpu_counters_t* cum;
    // host drop-in (dqdk_gpu_rx_batch): the results as read, and the batch's
    // [first abort idx, counters] once every block has added its counts (the
    // last block by ticket), written into pinned host memory; null: not kept
    dqdk_gpu_rx_result_t* out_res;
    uint64_t* out_batch;  // kBatchOut words
    uint32_t* ticket;     // zero between launches
};
constexpr int kBatchOut = 13;  // batch_scratch[0..12]

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
    uint32_t* part1;    // keys grouped by bucket (rx_part1's region starts at part1_base)
    uint64_t part1_base;  // first element of rx_part1's output (0, or after the fused pieces)
    uint16_t* part2;    // item i's slice-sorted u16 bins ((key & 16383) << 2) at [i * kPartChunk, + keys)
    uint16_t* runs;     // [items][kItemOffs] slice run starts inside each item
    const uint32_t* total_keys;  // rx_part1 input length on the device (overflow list), or null: limit * E
    uint32_t fused;     // the keys are the fused decode's pieces + rx_part1's run of its overflow
    uint32_t fgrid;     // fused: decode blocks (pieces per bucket)
    uint32_t piece_cap;
    uint32_t piece_words;
    uint64_t region;
    // the slice pass runs over nslots staged batches: batch k's scratch,
    // part2 keys and run offsets sit k strides (elements) after the first
    uint32_t nslots;
    uint32_t scratch_stride;
    uint64_t part2_stride, runs_stride;
    // rx_part2: the last block (ticket, zero between launches) re-zeroes
    // scratch [0, kZeroWords), the per-batch counters, once every block has
    // read them: the slot is clean for its next batch without a memset
    uint32_t* p2_ticket;
    // fused path: the last block reports the batch's overflow keys
    // (scratch[kOffOvfN]) to ovf_out, host-mapped: the host's choice of the
    // next batches' overflow form (RxArgs::ovf_list)
    uint64_t* ovf_out;
};

// Frame-processor plugin (dqdk_gpu_frame_processor, frame_processor.hip):
// the payloads of n tristan_process(payload, datalen, 1) calls
// (src/tristan.c:308-330, via process_unbuffered_frame :377-381), staged back
// to back: payload p's E events at stage + p * E * 16 (the bytes
// process_events_unrolled16 reads, :247-304), its datalen at len[p].
struct PayloadArgs {
    const uint8_t* stage;
    const uint32_t* len;
    uint32_t n;
    uint32_t E;
    int histo;                // decode events (is_store_histo, src/tristan.c:65-70)
    dqdk_gpu_rx_result_t* res;  // per call: {datalen, OK, 0, rejected events}
    uint32_t* keys;           // n * E frame-order records (DQDK_KEY_NONE: rejected)
    uint32_t* cnt1;           // partitioned histogram: keys per L1 bucket, or null
    uint64_t* batch_scratch;  // per-batch state (reset here, read by rx_count)
};

__global__ void rx_decode_kernel(RxArgs a);
__global__ void fp_decode_kernel(PayloadArgs a);
template <int kLdAux, bool kLines, bool kHeadA>
__global__ void rx_decode_fused_kernel(RxArgs a);
__global__ void rx_abort_kernel(CountArgs a);
__global__ void rx_small_kernel(RxArgs ra, CountArgs ca);  // gridDim 1, n <= kTile, records path
__global__ void rx_count_kernel(CountArgs a);
__global__ void rx_histo_atomic_kernel(HistoArgs a);
__global__ void rx_part1_kernel(HistoArgs a);
template <int kLdAux>
__global__ void rx_part2_kernel(HistoArgs a);
__global__ void rx_slice_histo_kernel(HistoArgs a);

}  // namespace dqdk
