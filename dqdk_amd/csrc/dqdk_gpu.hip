/*
 * dqdk_gpu.hip -- host runtime behind the C ABI in include/dqdk_gpu.h.
 *
 * One dqdk_gpu_queue per RX queue (the reference's dqdk_worker_t,
 * src/dqdk.h:87-105): a HIP stream, the queue's device histogram (the
 * per-GPU partial of tristan_t::histo, src/tristan.h:86), cumulative
 * counters (dqdk_stats_t + tristan_t atomics) and per-batch scratch.
 * Every batch is three short launches on the queue stream; nothing is
 * computed on the host.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "egress_kernels.h"
#include "rx_kernels.h"

using namespace dqdk;

namespace {

thread_local std::string g_err;

int fail(const char* what, hipError_t e)
{
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -EIO;
}

int fail_errno(int err, const char* what)
{
    g_err = what;
    return err;
}

#define HIPCHK(x)                           \
    do {                                    \
        hipError_t e_ = (x);                \
        if (e_ != hipSuccess)               \
            return fail(#x, e_);            \
    } while (0)

// Entry points make the queue's device current and restore the caller's on
// return (the calling thread's current device is not changed by the ABI).
struct DevGuard {
    int prev = -1;
    hipError_t e;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        e = prev == dev ? hipSuccess : hipSetDevice(dev);
    }
    ~DevGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
            (void)hipSetDevice(prev);
    }
};
#define SETDEV(dev)                                   \
    DevGuard dev_guard_(dev);                         \
    if (dev_guard_.e != hipSuccess)                   \
        return fail("hipSetDevice", dev_guard_.e)

constexpr int kStages = DQDK_GPU_TIMING_STAGES;
// (rx_fixup: on the fused path, the launch of rx_part1_kernel that groups a
// long overflow list for rx_part2 -- since round 6 only after a batch whose
// list passed kOvfAtomicMax; stage 5 is unused since rx_part2 derives its
// items itself)
enum Stage { kStDecode, kStAbort, kStCount, kStAtomic, kStPart1, kStPrep, kStPart2, kStSlice, kStUnused8, kStFixup };  // 5, 8: retired kernels
const char* const kStageNames[kStages] = {"rx_decode", "rx_abort", "rx_count",       "rx_histo_atomic",
                                          "rx_part1",  "(unused)", "rx_part2",       "rx_slice_histo",
                                          "(unused)", "rx_fixup"};
constexpr int kBatchScratch = 32;  // u64 words: [0] abort idx, [1..12] batch counters, [20] rx_count's ticket
constexpr int kTicketWord = 20;
constexpr int kFoldTicketWord = 21;  // the fused decode's folded counters (RxArgs::fold)
constexpr int kPart2TicketWord = 22;  // rx_part2's last block re-zeroes the slot's counters
// The fused pieces' offset inside their allocation can move by up to this
// many words (placement relative to the frames: DESIGN.md §5)
constexpr uint64_t kPieceShiftMax = 8u << 20;  // 32 MiB
constexpr int kProbeCands = DQDK_GPU_PROBE_CANDS;  // staging placement probe: candidate piece buffers
// each candidate once untimed (first touch), then timed twice: in order,
// then in reverse order, so a drift of the device's speed over the probe's
// batches (r06z7: the first-timed candidate 4 % slow, the original buffer
// picked against) weighs on every candidate alike
constexpr int kProbeSteps = 3 * kProbeCands;
constexpr uint32_t kProbeMinFrames = 65536;

uint32_t events_per_payload(uint32_t mode, uint32_t payloadsz)  // src/tristan.c:72-85
{
    switch (mode) {
    case DQDK_MODE_LISTMODE:
    case DQDK_MODE_ENERGYHISTO:
        return payloadsz / 16;
    case DQDK_MODE_LISTWAVE:
    case DQDK_MODE_WAVEFORM:
        return 1;
    default:
        return 0;
    }
}

struct Reg {
    void* host;
    uint64_t size;
    void* dev;
    void* base;  // the process-wide registration it holds a reference to (GReg::host)
};

// Host UMEM registrations, process-wide and reference-counted: HIP keeps one
// registration per host range, not one per caller, so several queues over
// one host buffer (a caller may hand one UMEM to several workers' queues --
// the reference allocates one per worker, src/dqdk.c:562 -- or views inside
// one) share one registration and the last of them to let go unregisters it.  (Before round 6 every queue
// registered and unregistered the range itself: the first queue's destroy
// took the mapping from under the others -- found when destroy began
// reporting the failed hipHostUnregister of the second queue.)
struct GReg {
    void* host;
    uint64_t size;
    int refs;
};
std::mutex g_reg_mu;
std::vector<GReg> g_regs;

// one reference to the registration of [host, host + size): an existing one
// at least that large, or a new one (a smaller one held by nobody else is
// replaced; one held by other queues cannot grow under them: -EBUSY)
int greg_acquire(void* host, uint64_t size, bool replacing_own, void** dev_out, bool* own_kept, void** base_out)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    *own_kept = replacing_own;  // (the caller's reference survives a failure unless released below)
    *base_out = host;
    // (a shared registration's device address is asked for on the caller's
    // device: queues over one UMEM may sit on different GPUs)
    auto dev_of = [](void* h, void** d) { return hipHostGetDevicePointer(d, h, 0); };
    if (!replacing_own) {
        // inside another queue's registration (a view of a shared UMEM)
        const uint8_t* h = (const uint8_t*)host;
        for (GReg& g : g_regs)
            if (g.host != host && (const uint8_t*)g.host <= h && h + size <= (const uint8_t*)g.host + g.size) {
                void* d = nullptr;
                HIPCHK(dev_of(g.host, &d));
                g.refs++;
                *dev_out = (uint8_t*)d + (h - (const uint8_t*)g.host);
                *base_out = g.host;
                return 0;
            }
    }
    for (size_t k = 0; k < g_regs.size(); k++) {
        GReg& g = g_regs[k];
        if (g.host != host)
            continue;
        if (g.size >= size) {
            void* d = nullptr;
            HIPCHK(dev_of(host, &d));
            if (!replacing_own)
                g.refs++;
            *dev_out = d;
            return 0;
        }
        if (g.refs > (replacing_own ? 1 : 0))
            return fail_errno(-EBUSY, "umem_register: a larger UMEM at an address other queues hold registered");
        *own_kept = false;
        g_regs.erase(g_regs.begin() + (long)k);
        HIPCHK(hipHostUnregister(host));
        break;
    }
    HIPCHK(hipHostRegister(host, size, hipHostRegisterMapped | hipHostRegisterPortable));
    void* dev = nullptr;
    const hipError_t e = dev_of(host, &dev);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host);
        return fail("hipHostGetDevicePointer", e);
    }
    g_regs.push_back({host, size, 1});
    *dev_out = dev;
    return 0;
}

// drop one reference; the last one unregisters
hipError_t greg_release(void* host)
{
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (size_t k = 0; k < g_regs.size(); k++)
        if (g_regs[k].host == host) {
            if (--g_regs[k].refs > 0)
                return hipSuccess;
            g_regs.erase(g_regs.begin() + (long)k);
            return hipHostUnregister(host);
        }
    return hipErrorHostMemoryNotRegistered;
}

// Device memory: plain (hipMalloc) or physically contiguous
// (hipDeviceMallocContiguous).  UMEM images from dqdk_gpu_device_alloc are
// contiguous (DQDK_GPU_IMAGE_ALLOC=plain: plain); the queue's table and
// staging are plain (DQDK_GPU_ALLOC = plain | contig | auto, auto =
// contiguous from 128 events per frame).  The decode's rate depends on where
// the image and the staging land physically (9000 B: 2.27 or 2.45-2.49 ms,
// repeatable per box and allocation pattern, but which pattern is fast
// differs between boxes): DESIGN.md §5.
enum AllocKind { kAllocPlain = 0, kAllocContig = 1, kAllocAuto = 2 };

int alloc_kind(const char* var, int dflt)
{
    const char* e = getenv(var);
    if (!e)
        return dflt;
    if (!strcmp(e, "contig"))
        return kAllocContig;
    if (!strcmp(e, "auto"))
        return kAllocAuto;
    return kAllocPlain;
}

int internal_alloc_kind(uint32_t E)
{
    static const int k = alloc_kind("DQDK_GPU_ALLOC", kAllocPlain);
    return k == kAllocAuto ? (E >= 128 ? kAllocContig : kAllocPlain) : k;
}

int image_alloc_kind()
{
    static const int k = alloc_kind("DQDK_GPU_IMAGE_ALLOC", kAllocContig);
    return k == kAllocAuto ? kAllocContig : k;
}

template <typename T>
hipError_t dev_alloc(T** p, size_t bytes, int kind, int* got = nullptr)
{
    void* v = nullptr;
    hipError_t e = hipErrorOutOfMemory;
    int k = kAllocPlain;
    if (kind == kAllocContig && bytes >= (1u << 21)) {
        e = hipExtMallocWithFlags(&v, bytes, hipDeviceMallocContiguous);
        k = kAllocContig;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();  // a refused contiguous request falls back to hipMalloc
        e = hipMalloc(&v, bytes);
        k = kAllocPlain;
    }
    if (got)
        *got = k;
    *p = (T*)v;
    return e;
}

void dev_free(void* p) { (void)hipFree(p); }

}  // namespace

struct dqdk_gpu_queue {
    int device = 0;
    dqdk_gpu_cfg_t cfg{};
    uint32_t E = 0;
    uint32_t max_batch = 0;
    int histo = 0;
    int cu_count = 256;
    int dec_cus = 256;             // fused decode blocks at most (DQDK_GPU_DECODE_CUS, default all CUs)
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    hipEvent_t switch_ev = nullptr;  // orders a stream switch after the old stream's work
    uint32_t* d_hist = nullptr;    // table base plane (u32/bin); value = d_hist + d_lo
    uint8_t* d_lo = nullptr;       // table low-byte plane (partitioned sweep)
    uint32_t* d_snap = nullptr;    // u32 snapshot for histogram_device_ptr (lazy)
    dqdk_gpu_counters_t* d_cum = nullptr;
    uint64_t* d_batch = nullptr;
    uint32_t* d_blkcnt = nullptr;  // fused decode: the folded counters' accumulators (kFoldWords u64)
    uint32_t* d_keys = nullptr;    // records path: frame-order keys (max_batch * E; allocated on first use)
    uint32_t* d_part1 = nullptr;   // fused path: pieces + rx_part1's copy of the overflow list (part1_elems)
    uint64_t part1_elems = 0;
    uint64_t piece_shift = 0;      // fused pieces start this many words into d_part1 (DQDK_GPU_PIECE_SHIFT)
    uint32_t* d_part1_rec = nullptr;  // records path: rx_part1's output when d_part1 is smaller (first use)
    uint32_t* d_ovf = nullptr;     // fused path: the overflow list (ovf_blk_elems keys)
    uint32_t ovf_cap_blk = 0;      // fused path: keys per block overflow region
    uint16_t* d_part2 = nullptr;
    uint16_t* d_runs = nullptr;    // part2 run offsets per item (kPartChunk keys)
    uint32_t* d_hscratch = nullptr;
    // staged slots whose per-batch counters (scratch [0, kZeroWords)) are not
    // known to be zero: set until a batch's rx_part2 (which re-zeroes them
    // at its end) is enqueued on the slot, memset on the next use otherwise
    std::vector<uint8_t> slot_dirty;
    uint32_t* d_ovf_blk = nullptr; // fused path: per-block overflow regions (in d_part1's rx_part1 region)
    uint64_t ovf_blk_elems = 0;    // grid * ovf_cap_blk
    uint64_t fused_elems = 0;      // fused path: pieces region (0: the fused path is off)
    uint64_t nk_max = 0;           // max_batch * E
    uint64_t scratch_words = 0;    // kHistScratchWords per staged slot
    int histo_path = 0;            // 0 auto, 1 atomic, 2 partitioned
    // A/B knobs (DQDK_GPU_* environment), read once by dqdk_gpu_queue_create
    // and never per batch: the engine's behaviour is fixed for the queue's life
    uint32_t fused_pol = 0;        // fused decode variant (fused_policy)
    uint32_t round_windows = 0;    // fused decode windows per wave per round (fused_round_windows)
    bool fold_off = false;         // DQDK_GPU_FOLD=0: the fused path counts in rx_abort + rx_count launches
    uint32_t fmap = 0;             // DQDK_GPU_FRAME_MAP=1: interleaved fused frame map
    bool p2zero_off = false;       // DQDK_GPU_P2ZERO=0: memset the slot's counters before every batch
    bool small_off = false;        // DQDK_GPU_SMALL=0: small batches take the three-launch form too
    uint32_t tile_frames = 0;      // DQDK_GPU_TILE_FRAMES: records-path decode frames per wave tile (0: 64)
    int ovf_list_mode = -1;        // DQDK_GPU_OVF_LIST: fused overflow keys 0 = atomics, 1 = listed + grouped (-1: by the last batch)
    // Staging placement probe: the fused decode's rate
    // depends on where its piece buffer (d_part1, the decode's write stream)
    // lands physically relative to the image it reads -- 2.12 vs 2.35 ms at
    // 1M x 9000 B, same build, same image.  The first fused batches of at
    // least kProbeMinFrames frames run on kProbeCands candidate allocations
    // in turn (each first untimed, its pages' first use, then timed twice,
    // forward and reverse order); the fastest mean is kept and the others
    // freed.  DQDK_GPU_STAGING_PROBE=0: off.
    int probe = 0;                 // next probe step (1-based), 0: off or done
    uint32_t* part1_cand[kProbeCands] = {};
    float probe_ms[kProbeCands] = {};  // summed decode ms per frame x 1e6 of each candidate
    int probe_cnt[kProbeCands] = {};   // its timed batches
    int probe_timed = -1;          // candidate of the batch whose events are pending
    uint32_t probe_n = 0;          // its frames
    hipEvent_t probe_ev[2] = {nullptr, nullptr};
    int probe_chosen = -1;         // -1: not decided
    int alloc_kind = 0;            // device memory of the table and staging (dev_alloc)
    // Partitioned batches stage their slice-sorted keys (part2 + runs +
    // scratch, one slot each); the slice pass -- which sweeps the low-byte
    // plane of every touched slice -- runs once over hist_k staged batches,
    // and before anything reads the table (hist_flush).
    uint32_t hist_k = 1;
    uint32_t hist_pending = 0;
    size_t part2_stride = 0, runs_stride = 0;  // elements per slot
    dqdk_gpu_desc_t* d_desc = nullptr;
    dqdk_gpu_rx_result_t* d_res = nullptr;
    // raw payload stream (tristan.c:318-324)
    int raw_fd = -1;
    uint64_t* d_raw_blk = nullptr;  // per-256-frame byte totals -> offsets
    // Host drop-in raw egress, double-buffered: batch b gathers its stream
    // into d_rawb[b & 1] on the queue stream, the D2H runs on raw_stream into
    // pinned h_rawb[b & 1], and its write() happens during the next batch's
    // call, while that batch's kernels run (or at the drain: queue_sync,
    // set_raw_fd, destroy).
    hipStream_t raw_stream = nullptr;
    hipEvent_t raw_ev_d2h[2] = {nullptr, nullptr};
    uint8_t* d_rawb[2] = {nullptr, nullptr};
    uint64_t d_rawb_cap[2] = {0, 0};
    uint8_t* h_rawb[2] = {nullptr, nullptr};
    uint64_t h_rawb_cap[2] = {0, 0};
    uint64_t raw_pend_len[2] = {0, 0};
    int raw_pend[2] = {0, 0};
    uint64_t raw_seq = 0;
    uint64_t* h_raw_total = nullptr;  // pinned: the batch's stream length
    int raw_deferred = 0;             // dqdk_gpu_queue_set_raw_deferred: write() during the next call
    // async consumer: per-burst first element / length / output offset
    uint32_t* d_async = nullptr;
    size_t async_cap = 0;  // bursts
    std::vector<Reg> regs;
    // Host drop-in (dqdk_gpu_rx_batch) without raw egress: the descriptors
    // are copied into pinned h_desc and read from there by the kernels
    // (zero-copy), rx_count writes the per-frame results and the batch's
    // counters straight into pinned h_res / h_batch, and the call returns at
    // ev_read: after the last kernel that reads caller memory (the frames,
    // the descriptors); the histogram kernels run on behind it.
    dqdk_gpu_desc_t* h_desc = nullptr;
    dqdk_gpu_rx_result_t* h_res = nullptr;
    uint64_t* h_batch = nullptr;
    uint64_t* h_ovf = nullptr;      // fused path: the last batch's overflow keys (host-mapped, rx_part2 writes)
    uint64_t* h_ovf_dev = nullptr;
    const dqdk_gpu_desc_t* h_desc_dev = nullptr;
    dqdk_gpu_rx_result_t* h_res_dev = nullptr;
    uint64_t* h_batch_dev = nullptr;
    hipEvent_t ev_read = nullptr;
    bool publish = false;  // this launch: rx_count publishes to h_res / h_batch, ev_read is recorded
    // stage timing
    int timing = 0;
    uint32_t stage_mask = ~0u;  // stages bracketed while timing is on
    std::vector<hipEvent_t> ev_free;
    struct Pending {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    double stage_ms[kStages] = {};
    uint64_t counts[kStages] = {};
};

namespace {

int ev_get(dqdk_gpu_queue* q, hipEvent_t* e)
{
    if (!q->ev_free.empty()) {
        *e = q->ev_free.back();
        q->ev_free.pop_back();
        return 0;
    }
    HIPCHK(hipEventCreate(e));
    return 0;
}

struct StageTimer {
    dqdk_gpu_queue* q;
    int stage;
    hipEvent_t a = nullptr, b = nullptr;
    StageTimer(dqdk_gpu_queue* q_, int s) : q(q_), stage(s)
    {
        if (q->timing && ((q->stage_mask >> stage) & 1u) && ev_get(q, &a) == 0 && ev_get(q, &b) == 0)
            (void)hipEventRecord(a, q->stream);
    }
    ~StageTimer()
    {
        if (q->timing && a && b) {
            (void)hipEventRecord(b, q->stream);
            q->pending.push_back({stage, a, b});
        }
    }
};

// The partitioned histogram sweeps every slice that receives events (up to
// the whole 2.38 GB table once per batch); per-event atomics cost ~1/18 ns
// each (measured, profiles/).  Partition once a batch carries enough events.
constexpr uint64_t kPartitionMinKeys = 4u << 20;

#ifndef DQDK_HIST_KMAX
#define DQDK_HIST_KMAX 32
#endif
#ifndef DQDK_HIST_STAGE_MB
#define DQDK_HIST_STAGE_MB 24576
#endif
constexpr size_t kHistKMax = DQDK_HIST_KMAX;  // staged batches per slice pass, at most
static_assert(kHistKMax <= (size_t)kSliceMaxSlots, "the slice pass indexes staged batches in registers");
constexpr size_t kHistStageBytes = (size_t)DQDK_HIST_STAGE_MB << 20;  // staging budget of a queue

bool use_partitioned(const dqdk_gpu_queue* q, uint32_t n)
{
    if (q->histo_path)
        return q->histo_path == 2;
    return (uint64_t)n * q->E >= kPartitionMinKeys;
}

// The slice pass over every staged partitioned batch (see hist_k).
int hist_flush(dqdk_gpu_queue* q)
{
    if (!q->hist_pending)
        return 0;
    HistoArgs ha{};
    ha.hist = q->d_hist;
    ha.lo = q->d_lo;
    ha.scratch = q->d_hscratch;
    ha.part2 = q->d_part2;
    ha.runs = q->d_runs;
    ha.nslots = q->hist_pending;
    ha.scratch_stride = (uint32_t)q->scratch_words;
    ha.part2_stride = q->part2_stride;
    ha.runs_stride = q->runs_stride;
    q->hist_pending = 0;
    {
        StageTimer t(q, kStSlice);
        hipLaunchKernelGGL(rx_slice_histo_kernel, dim3(kSliceBlocks), dim3(kSliceThreads), 0, q->stream, ha);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

// Windows per wave per fused round: the block's 16 waves stage at most
// 16 * W * min(E, 128) keys per round into 284 * kFCap slots (kFCap 198,
// keys packed three to a word).  Measured (A/B, r05l/r05m): W = 28 at 1500 B
// (fill 70 %; 24 and 32 windows slower, 32 overflowing more keys), W = 16 at
// 9000 B, where the lines policy carries up to 47 keys per bucket between
// rounds (20 windows overflowed three times as many keys to rx_part1).
//
// The pieces' runs end mid-line.  Below 128 events per frame (1500 B) the
// partial lines complete in L2 (write-back piece stores); from 128 on (9000
// B: every 2-KB window full of events) whole lines are flushed and
// remainders carried, which costs stage room, hence the smaller round (A/B,
// one box, 9000 B: decode 2.86 -> 2.44 ms; at 1500 B lines cost 0.04 ms),
// and those whole lines go out as streaming stores.  The frame loads are
// non-temporal at both sizes (r05x/r05y, 9000 B: decode 2.06 -> 2.00 ms,
// policy 1 -> 3, since the pieces stream).
// policy bit 0: whole-line flushes, bit 1: non-temporal frame loads, bit 2:
// phase A takes each frame's first line (events and checksum bytes; phase B
// then never touches that line: traffic 2.08 -> 1.96 GB at 1M x 1500 B, but
// the decode 0.432 -> 0.455 ms on one box, r04k2: the extra phase-A work
// costs more than the line, so it is off by default).  The shipped library
// holds the two default variants (3 from 128 events per frame, else 2);
// a build with -DDQDK_AB_VARIANTS holds all eight, which
// DQDK_GPU_FUSED_POLICY=<0..7> selects at queue creation (A/B, tests).
#ifndef DQDK_FUSED_POLICY
#define DQDK_FUSED_POLICY (E >= 128 ? 3u : 2u)
#endif
uint32_t fused_policy_default(uint32_t E) { return (uint32_t)(DQDK_FUSED_POLICY); }

#ifdef DQDK_AB_VARIANTS
constexpr uint32_t kFusedPolicies = 0xffu;  // every variant built
#else
constexpr uint32_t kFusedPolicies = (1u << 2) | (1u << 3);
#endif

uint32_t fused_round_windows(uint32_t E, double fill)
{
    const uint32_t epw = std::max<uint32_t>(1, std::min<uint32_t>(E, 128));
    const uint32_t w = (uint32_t)(fill / 100.0 * kFCap * kL1Buckets / (kFWaves * epw));
    const uint32_t wr = (w + kFRingW / 2) / kFRingW * kFRingW;  // nearest multiple of the ring depth
    return std::max<uint32_t>(kFRingW, std::min<uint32_t>(64, wr));
}

// Records-path buffers, allocated on the first batch that takes that path
// (the fused path, the benchmarked one, needs neither): frame-order keys
// (unless the caller passes its own record buffer) and rx_part1's grouped
// copy of them (d_part1 when it is large enough).
int ensure_records(dqdk_gpu_queue* q, bool keys, bool part1)
{
    hipError_t e;
    if (keys && !q->d_keys && (e = dev_alloc(&q->d_keys, q->nk_max * 4, q->alloc_kind)) != hipSuccess) {
        q->d_keys = nullptr;
        return (fail("hipMalloc(records)", e), -ENOMEM);
    }
    const uint64_t need = q->nk_max + kStagePad;
    if (part1 && q->part1_elems < need && !q->d_part1_rec &&
        (e = dev_alloc(&q->d_part1_rec, need * 4, q->alloc_kind)) != hipSuccess) {
        q->d_part1_rec = nullptr;
        return (fail("hipMalloc(records)", e), -ENOMEM);
    }
    return 0;
}

uint32_t* records_part1(const dqdk_gpu_queue* q)
{
    return q->part1_elems >= q->nk_max + kStagePad ? q->d_part1 : q->d_part1_rec;
}

// Launch guard: when p lies in an allocation of dqdk_gpu_device_alloc
// (UMEM images, frame staging slots: sizes known exactly), [p, p + bytes)
// must lie inside it -- the kernels' buffer descriptors and plain pointers
// reach exactly as far as the caller's sizes say (DESIGN.md section 3 lists
// each kernel's furthest byte).  Other memory is the caller's to size (HIP's
// pointer-range attribute is not reliable past 4 GiB on this stack).
std::mutex g_alloc_mu;
std::vector<std::pair<uintptr_t, uint64_t>> g_allocs;  // dqdk_gpu_device_alloc: base, size

int check_range(const void* p, uint64_t bytes, const char* what)
{
    if (!p || !bytes)
        return 0;
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_alloc_mu);
    for (const auto& r : g_allocs) {
        if (a >= r.first && a < r.first + r.second) {
            if (bytes > r.first + r.second - a) {
                g_err = std::string(what) + ": runs past the end of its dqdk_gpu_device_alloc allocation";
                return -EINVAL;
            }
            return 0;
        }
    }
    return 0;
}

// Histogram accumulation of a batch's keys (K3): frame-order records (the
// atomic path, or rx_part1 -> rx_part2 on the partitioned one), or with fg
// set the fused decode's pieces + overflow list.  The partitioned path stages
// the batch for the slice pass (hist_k batches per pass).
int launch_histo(dqdk_gpu_queue* q, uint32_t n, const dqdk_gpu_rx_result_t* d_res, const uint32_t* keys,
                 bool partitioned, const FusedGeom* fg, const RxArgs& ra, uint32_t* slot_scratch)
{
    HistoArgs ha{};
    ha.res = d_res;
    ha.keys = keys;
    ha.n = n;
    ha.E = q->E;
    ha.flags = q->cfg.flags;
    ha.batch_scratch = q->d_batch;
    ha.hist = q->d_hist;
    ha.lo = q->d_lo;
    ha.scratch = slot_scratch;
    const bool fused = fg != nullptr;
    if (partitioned && (q->hist_pending >= q->hist_k || !q->d_part2))
        return fail_errno(-EIO, "histogram: staging slot out of range");
    ha.part1 = fused ? q->d_part1 + q->piece_shift : records_part1(q);
    ha.part2 = q->d_part2 ? q->d_part2 + q->hist_pending * q->part2_stride : nullptr;
    ha.runs = q->d_runs ? q->d_runs + q->hist_pending * q->runs_stride : nullptr;
    if (fused) {
        ha.keys = q->d_ovf;                     // the overflow list
        ha.total_keys = slot_scratch + kOffOvfN;
        ha.part1_base = (uint64_t)kL1Buckets * fg->region;
        ha.fused = 1;
        ha.fgrid = fg->grid;
        ha.piece_cap = fg->cap;
        ha.piece_words = fg->words;
        ha.region = fg->region;
    }
    if (!partitioned) {
        const uint32_t grid_h = std::min<uint32_t>((n + 3) / 4, (uint32_t)q->cu_count * 8u);
        StageTimer t(q, kStAtomic);
        hipLaunchKernelGGL(rx_histo_atomic_kernel, dim3(grid_h), dim3(256), 0, q->stream, ha);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const uint64_t nkeys = (uint64_t)n * q->E;
    const uint32_t chunks = (uint32_t)((nkeys + kPartChunk - 1) / kPartChunk);
    const uint32_t grid_p = std::min<uint32_t>((uint32_t)((nkeys + kP1Chunk - 1) / kP1Chunk),
                                               (uint32_t)q->cu_count * (uint32_t)kP1BlocksPerCu);
    const uint32_t grid_l2 = std::min<uint32_t>(chunks + (uint32_t)(kL1Buckets * kSegsPerBucket),
                                                (uint32_t)q->cu_count * (uint32_t)kP2BlocksPerCu);
    // fused path: the decode takes back checksum-failed frames itself and, in
    // its usual form, adds its overflow keys to the table by device atomics
    // (round 6: one launch less per batch); after a batch with more than
    // kOvfAtomicMax overflow keys (rx_part2 reports the count into
    // host-mapped memory) the next batches list them instead (RxArgs::ovf_list)
    // and rx_part1 groups the list for rx_part2, timed as "rx_fixup"
    if (fused)
        ha.ovf_out = q->h_ovf_dev;
    if (!fused || ra.ovf_list) {
        StageTimer t(q, fused ? kStFixup : kStPart1);
        hipLaunchKernelGGL(rx_part1_kernel, dim3(grid_p), dim3(kP1Threads), 0, q->stream, ha);
    }
    ha.p2_ticket = (uint32_t*)(q->d_batch + kPart2TicketWord);
    {
        StageTimer t(q, kStPart2);
        // non-temporal key loads where the fused decode's are (fused_policy bit 1)
        if (q->fused_pol & 2u)
            hipLaunchKernelGGL(rx_part2_kernel<2>, dim3(grid_l2), dim3(kPartThreads), 0, q->stream, ha);
        else
            hipLaunchKernelGGL(rx_part2_kernel<0>, dim3(grid_l2), dim3(kPartThreads), 0, q->stream, ha);
    }
    HIPCHK(hipGetLastError());
    if (q->hist_pending < q->slot_dirty.size())
        q->slot_dirty[q->hist_pending] = 0;  // re-zeroed by this rx_part2's last block
    if (++q->hist_pending == q->hist_k)
        return hist_flush(q);
    return 0;
}

// The staged slot's per-batch counters are zero before its batch's first
// kernel: a memset only when the slot's last rx_part2 did not re-zero them
// (first use, or a batch that failed on the way); dirty until this batch's
// rx_part2 is enqueued.
int clean_slot(dqdk_gpu_queue* q, uint32_t* slot_scratch)
{
    if (q->slot_dirty.size() < q->hist_k)
        q->slot_dirty.resize(q->hist_k, 1);
    if (q->slot_dirty[q->hist_pending] || q->p2zero_off) {
        HIPCHK(hipMemsetAsync(slot_scratch, 0, kZeroWords * sizeof(uint32_t), q->stream));
        // a batch that failed on the way may have left a last-block ticket
        // raised (rx_count's, the fused decode's, rx_part2's): zero between
        // launches, else no block would ever be the last (advisor r4)
        static_assert(kFoldTicketWord == kTicketWord + 1 && kPart2TicketWord == kTicketWord + 2, "ticket words");
        HIPCHK(hipMemsetAsync(q->d_batch + kTicketWord, 0, 3 * sizeof(uint64_t), q->stream));
        // and the folded counters' accumulators: zero, the first-failure
        // word (FoldWord F_FAIL = 9) all ones, as at creation
        HIPCHK(hipMemsetAsync(q->d_blkcnt, 0, kFoldWords * sizeof(uint64_t), q->stream));
        HIPCHK(hipMemsetAsync((uint64_t*)q->d_blkcnt + 9, 0xff, sizeof(uint64_t), q->stream));
    }
    q->slot_dirty[q->hist_pending] = 1;
    return 0;
}

// Staging placement probe, before a fused batch of n frames: collects the
// previous probe batch's decode time, decides once every step is timed, and
// points d_part1 (and the overflow regions inside it) at this batch's
// candidate.  Returns the candidate to time (-1: none).
int probe_step(dqdk_gpu_queue* q, uint32_t n)
{
    if (q->probe_timed >= 0) {
        float ms = 0;
        hipError_t e = hipEventSynchronize(q->probe_ev[1]);
        if (e == hipSuccess)
            e = hipEventElapsedTime(&ms, q->probe_ev[0], q->probe_ev[1]);
        if (e != hipSuccess)
            return fail("staging probe: decode events", e);
        q->probe_ms[q->probe_timed] += ms * 1e6f / (float)q->probe_n;
        q->probe_cnt[q->probe_timed]++;
        q->probe_timed = -1;
    }
    if (!q->probe || n < kProbeMinFrames || !q->fused_elems)
        return -1;
    if (q->probe > kProbeSteps) {  // every candidate timed: keep the fastest mean
        auto mean = [&](int k) { return q->probe_cnt[k] ? q->probe_ms[k] / (float)q->probe_cnt[k] : 0.f; };
        int c = 0;
        for (int k = 1; k < kProbeCands; k++)
            if (q->part1_cand[k] && q->probe_cnt[k] && mean(k) < mean(c))
                c = k;
        q->probe_chosen = c;
        q->d_part1 = q->part1_cand[c];
        q->d_ovf_blk = q->d_part1 + q->piece_shift + q->fused_elems;
        for (int k = 1; k < kProbeCands; k++)  // (the original, candidate 0, stays if not chosen: freed with the queue)
            if (k != c) {
                dev_free(q->part1_cand[k]);
                q->part1_cand[k] = nullptr;
            }
        if (c != 0) {
            dev_free(q->part1_cand[0]);
            q->part1_cand[0] = nullptr;
        }
        q->probe = 0;
        return -1;
    }
    if (q->probe == 1) {  // the candidates, allocated beside the original (other physical pages)
        q->part1_cand[0] = q->d_part1;
        // one at a time, and only while at least as much device memory as
        // the candidate stays free (several GB each at 1M x 9000 B,
        // times the queues sharing a GPU); a candidate that does not fit is
        // simply not probed
        const uint64_t bytes = q->part1_elems * 4;
        for (int k = 1; k < kProbeCands; k++) {
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < 2 * bytes) {
                (void)hipGetLastError();
                break;
            }
            if (dev_alloc(&q->part1_cand[k], bytes, q->alloc_kind) != hipSuccess) {
                (void)hipGetLastError();
                q->part1_cand[k] = nullptr;
            }
        }
        if ((!q->probe_ev[0] && hipEventCreate(&q->probe_ev[0]) != hipSuccess) ||
            (!q->probe_ev[1] && hipEventCreate(&q->probe_ev[1]) != hipSuccess)) {
            (void)hipGetLastError();
            q->probe = 0;
            return -1;
        }
    }
    const int step = q->probe++;  // 1 .. kProbeSteps
    // steps 1..N: candidate step - 1, untimed; N+1..2N: candidate step - N - 1;
    // 2N+1..3N: candidate 3N - step (the reverse order)
    int c = step <= 2 * kProbeCands ? (step - 1) % kProbeCands : kProbeSteps - step;
    if (!q->part1_cand[c])
        c = 0;  // (a candidate that did not allocate)
    q->d_part1 = q->part1_cand[c];
    q->d_ovf_blk = q->d_part1 + q->piece_shift + q->fused_elems;
    if (step <= kProbeCands)
        return -1;  // the candidate's first batch: untimed
    q->probe_n = n;
    return c;
}

// The fused decode variant of a policy (fused_policy_default; the variants
// kFusedPolicies does not hold are not in this build's code object).
void (*fused_kernel(uint32_t pol))(RxArgs)
{
    switch (pol) {
    case 2: return rx_decode_fused_kernel<2, false, false>;
    case 3: return rx_decode_fused_kernel<2, true, false>;
#ifdef DQDK_AB_VARIANTS
    case 0: return rx_decode_fused_kernel<0, false, false>;
    case 1: return rx_decode_fused_kernel<0, true, false>;
    case 4: return rx_decode_fused_kernel<0, false, true>;
    case 5: return rx_decode_fused_kernel<0, true, true>;
    case 6: return rx_decode_fused_kernel<2, false, true>;
    case 7: return rx_decode_fused_kernel<2, true, true>;
#endif
    default: return nullptr;
    }
}

// The A/B knobs, once per queue (dqdk_gpu_queue_create).  Returns -EINVAL for
// a fused policy this build does not hold.
int read_knobs(dqdk_gpu_queue* q)
{
    auto env = [](const char* k) -> const char* {
        const char* v = getenv(k);
        return v && *v ? v : nullptr;
    };
    q->fused_pol = fused_policy_default(q->E);
    if (const char* v = env("DQDK_GPU_FUSED_POLICY")) {
        const uint32_t p = (uint32_t)atoi(v) & 7u;
        if (!((kFusedPolicies >> p) & 1u))
            return fail_errno(-EINVAL, ("queue_create: DQDK_GPU_FUSED_POLICY=" + std::to_string(p) +
                                        " is an A/B variant (build with -DDQDK_AB_VARIANTS)").c_str());
        q->fused_pol = p;
    }
#ifndef DQDK_FUSED_FILL  // stage fill target, percent (198-key stage: W = 28 at 1500 B, 16 at 9000 B; r05l)
#define DQDK_FUSED_FILL (q->E >= 128 ? 65 : 70)
#endif
    double fill = DQDK_FUSED_FILL;
    if (const char* v = env("DQDK_GPU_FUSED_FILL"))
        fill = atof(v);
    q->round_windows = fused_round_windows(q->E, fill);
    q->fold_off = env("DQDK_GPU_FOLD") && !strcmp(env("DQDK_GPU_FOLD"), "0");
    q->fmap = env("DQDK_GPU_FRAME_MAP") ? (uint32_t)(atoi(env("DQDK_GPU_FRAME_MAP")) != 0) : 0u;
    q->p2zero_off = env("DQDK_GPU_P2ZERO") && !strcmp(env("DQDK_GPU_P2ZERO"), "0");
    q->small_off = env("DQDK_GPU_SMALL") && !strcmp(env("DQDK_GPU_SMALL"), "0");
    if (const char* v = env("DQDK_GPU_OVF_LIST"))
        q->ovf_list_mode = atoi(v) != 0 ? 1 : 0;
    if (const char* v = env("DQDK_GPU_TILE_FRAMES"))  // records-path decode: frames per wave tile (1-64)
        q->tile_frames = std::min<uint32_t>(64, std::max<uint32_t>(1, (uint32_t)atoi(v)));
    // the staging probe: on unless DQDK_GPU_STAGING_PROBE=0.  (At 1500 B it
    // is worth -1 to +2 %: with only the 1500 B image allocated the original
    // buffer was 1 % faster than the probe's pick, r06z7 / r06z8; in the
    // default bench, after the other lines' allocations, 2 % slower, r06z9.
    // At 9000 B: +7 % where the original lands slow.)
    q->probe = env("DQDK_GPU_STAGING_PROBE") && !strcmp(env("DQDK_GPU_STAGING_PROBE"), "0") ? 0 : 1;
    if (const char* v = env("DQDK_GPU_PIECE_SHIFT"))  // KiB (tools/state_probe.py)
        q->piece_shift = std::min<uint64_t>((uint64_t)atoll(v) * 256u, kPieceShiftMax - 256u) & ~63ull;
    return 0;
}

int launch_batch(dqdk_gpu_queue* q, const uint8_t* d_umem, uint64_t umem_size, const dqdk_gpu_desc_t* d_desc,
                 uint32_t n, dqdk_gpu_rx_result_t* d_res, uint32_t* d_keys)
{
    RxArgs ra{};
    ra.umem = d_umem;
    ra.umem_size = umem_size;
    ra.desc = d_desc;
    ra.n = n;
    ra.res = d_res;
    ra.E = q->E;
    ra.flags = q->cfg.flags;
    ra.port_start = q->cfg.port_start;
    ra.port_end = q->cfg.port_end;
    ra.histo = q->histo;
    ra.batch_scratch = q->d_batch;
    const bool partitioned = q->histo && q->E && use_partitioned(q, n);
    // Fused decode + bucketing: the batch's keys never exist in frame order.
    // Not when the caller wants those records, nor under batch-abort
    // accounting (the frames after the first failure are known only after
    // the decode; the records path counts exactly the accounted frames).
    const FusedGeom fg = fused_geom(n, q->E, (uint64_t)q->dec_cus);
    const bool fused = partitioned && !d_keys && !(q->cfg.flags & DQDK_GPU_F_BATCH_ABORT) && q->d_ovf &&
                       !(q->cfg.flags & DQDK_GPU_F_HISTO_UNFUSED) &&
                       (uint64_t)kL1Buckets * fg.region <= q->fused_elems;
    if (!fused && q->histo && q->E) {
        if (int rc = ensure_records(q, !d_keys, partitioned))
            return rc;
    }
    uint32_t* keys = d_keys ? d_keys : q->d_keys;
    ra.keys = keys;
    uint32_t* slot_scratch = q->d_hscratch + (size_t)q->hist_pending * q->scratch_words;
    ra.cnt1 = partitioned && !fused ? slot_scratch + kOffCnt1 : nullptr;
    if (partitioned)
        if (int rc = clean_slot(q, slot_scratch))
            return rc;

    CountArgs ca{};
    ca.res = d_res;
    ca.n = n;
    ca.E = q->E;
    ca.flags = q->cfg.flags;
    ca.histo = q->histo;
    ca.batch_scratch = q->d_batch;
    ca.cum = q->d_cum;
    if (q->publish) {
        ca.out_res = q->h_res_dev;
        ca.out_batch = q->h_batch_dev;
    }
    ca.ticket = (uint32_t*)(q->d_batch + kTicketWord);

    if (fused) {
        const int probe_c = probe_step(q, n);
        if (probe_c < -1)
            return probe_c;
        ra.keys = nullptr;  // no frame-order records
        ra.scratch = slot_scratch;
        ra.part1 = q->d_part1 + q->piece_shift;
        ra.piece_cap = fg.cap;
        ra.piece_words = fg.words;
        ra.region = fg.region;
        ra.ovf = q->d_ovf;
        // overflow keys listed for rx_part1's grouping only after a batch
        // that overflowed a lot (a heuristic: either form counts every key once)
        ra.ovf_list = q->ovf_list_mode >= 0 ? (uint32_t)q->ovf_list_mode
                      : q->h_ovf && __atomic_load_n(q->h_ovf, __ATOMIC_RELAXED) > kOvfAtomicMax ? 1u : 0u;
        ra.round_windows = q->round_windows;
        const uint32_t grid = fg.grid;
        // private overflow regions of ovf_cap_blk keys (past them: the table)
        ra.ovf_blk = q->d_ovf_blk;
        ra.ovf_blk_cap = q->ovf_cap_blk;
        ra.hist = q->d_hist;
        // per-packet counters in the decode itself (the host drop-in's
        // publishing batches keep rx_count, which writes its pinned results)
        ra.fold = !q->publish && !q->fold_off;
        ra.fmap = q->fmap;
        ra.blk_cnt = q->d_blkcnt;
        ra.ticket = (uint32_t*)(q->d_batch + kFoldTicketWord);
        ra.cum = q->d_cum;
        if ((uint64_t)ra.ovf_blk_cap * grid > q->ovf_blk_elems)
            return fail_errno(-EINVAL, "fused decode: overflow regions exceed their allocation");
        StageTimer t(q, kStDecode);
        // partial-line policy by frame density (fused_policy)
        auto kern = fused_kernel(q->fused_pol);
        if (!kern)
            return fail_errno(-EINVAL, "fused decode: no such variant");
        if (probe_c >= 0) {
            HIPCHK(hipEventRecord(q->probe_ev[0], q->stream));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(kFThreads), 0, q->stream, ra);
            HIPCHK(hipEventRecord(q->probe_ev[1], q->stream));
            q->probe_timed = probe_c;
        } else {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(kFThreads), 0, q->stream, ra);
        }
    } else if (n <= (uint32_t)kTile && !q->small_off) {
        // one block: decode, abort and count in a single launch (rx_small),
        // the frames spread over all its waves (a 64-frame batch is four
        // 16-frame tiles, not one wave streaming 64 frames in a row: over
        // zero-copy host UMEM every window is a PCIe round trip)
        ra.tile_frames = std::max<uint32_t>(1, std::min<uint32_t>(64, (n + kWaves - 1) / kWaves));
        StageTimer t(q, kStDecode);
        hipLaunchKernelGGL(rx_small_kernel, dim3(1), dim3(kTile), 0, q->stream, ra, ca);
    } else {
        // per-packet counters folded into the decode, as on the fused path
        // (not under batch-abort accounting, which needs the batch's first
        // failure before it counts; not for the host drop-in's publishing
        // batches, whose rx_count writes the pinned results)
        ra.fold = !q->publish && !q->fold_off && !(q->cfg.flags & DQDK_GPU_F_BATCH_ABORT);
        ra.blk_cnt = q->d_blkcnt;
        ra.ticket = (uint32_t*)(q->d_batch + kFoldTicketWord);
        ra.cum = q->d_cum;
        ra.tile_frames = q->tile_frames;  // (0: 64-frame wave tiles)
        const uint32_t nblk = (n + kTile - 1) / kTile;
#ifndef DQDK_DEC_BLOCKS_PER_CU
#define DQDK_DEC_BLOCKS_PER_CU 16u
#endif
        const uint32_t grid_dec = std::min<uint32_t>(nblk, (uint32_t)q->cu_count * DQDK_DEC_BLOCKS_PER_CU);
        StageTimer t(q, kStDecode);
        hipLaunchKernelGGL(rx_decode_kernel, dim3(grid_dec), dim3(kTile), 0, q->stream, ra);
    }
    HIPCHK(hipGetLastError());

    if (!ra.fold && (fused || n > (uint32_t)kTile || q->small_off)) {
        const uint32_t grid_cnt = std::min<uint32_t>((n + 255) / 256, (uint32_t)q->cu_count * 4u);
        {
            StageTimer t(q, kStAbort);
            hipLaunchKernelGGL(rx_abort_kernel, dim3(grid_cnt), dim3(256), 0, q->stream, ca);
        }
        {
            StageTimer t(q, kStCount);
            const uint32_t grid_c = std::min<uint32_t>((n + 255) / 256, (uint32_t)q->cu_count);
            hipLaunchKernelGGL(rx_count_kernel, dim3(grid_c), dim3(256), 0, q->stream, ca);
        }
        HIPCHK(hipGetLastError());
    }
    // no kernel reads caller memory past this point (since round 6 the fused
    // decode takes back its checksum-failed frames itself)
    if (q->publish)
        HIPCHK(hipEventRecord(q->ev_read, q->stream));

    if (q->histo && q->E)
        return launch_histo(q, n, d_res, keys, partitioned, fused ? &fg : nullptr, ra, slot_scratch);
    return 0;
}

// The frame-processor plugin's batch (frame_processor.hip): n staged
// payloads of E * 16 bytes at d_stage (DEVICE), their datalens at d_len.
// fp_decode -> rx_count -> the records-path histogram, on the queue stream.
int launch_payloads(dqdk_gpu_queue* q, const uint8_t* d_stage, const uint32_t* d_len, uint32_t n)
{
    const bool histo = q->histo && q->E;
    const bool partitioned = histo && use_partitioned(q, n);
    uint32_t* slot_scratch =
        q->d_hscratch ? q->d_hscratch + (size_t)q->hist_pending * q->scratch_words : nullptr;
    if (partitioned)
        if (int rc = clean_slot(q, slot_scratch))
            return rc;
    if (histo) {
        if (int rc = ensure_records(q, true, partitioned))
            return rc;
    }
    PayloadArgs pa{};
    pa.stage = d_stage;
    pa.len = d_len;
    pa.n = n;
    pa.E = q->E;
    pa.histo = histo;
    pa.res = q->d_res;
    pa.keys = histo ? q->d_keys : nullptr;
    pa.cnt1 = partitioned ? slot_scratch + kOffCnt1 : nullptr;
    pa.batch_scratch = q->d_batch;
    {
        StageTimer t(q, kStDecode);
        const uint32_t grid = std::min<uint32_t>((n + kWaves - 1) / kWaves, (uint32_t)q->cu_count * 8u);
        hipLaunchKernelGGL(fp_decode_kernel, dim3(grid), dim3(kTile), 0, q->stream, pa);
    }
    CountArgs ca{};
    ca.res = q->d_res;
    ca.n = n;
    ca.E = q->E;
    ca.flags = q->cfg.flags;  // (no batch abort: the caller's fetch_xsk accounts its batches)
    ca.histo = q->histo;
    ca.batch_scratch = q->d_batch;
    ca.cum = q->d_cum;
    {
        StageTimer t(q, kStCount);
        const uint32_t grid_c = std::min<uint32_t>((n + 255) / 256, (uint32_t)q->cu_count);
        hipLaunchKernelGGL(rx_count_kernel, dim3(grid_c), dim3(256), 0, q->stream, ca);
    }
    HIPCHK(hipGetLastError());
    if (!histo)
        return 0;
    RxArgs ra{};  // (read by rx_part1 on the fused path only)
    return launch_histo(q, n, q->d_res, q->d_keys, partitioned, nullptr, ra, slot_scratch);
}

// u32 view of table bins [first, first + nbins) (multiples of 16) into d_out, async.
int combine(dqdk_gpu_queue* q, uint32_t* d_out, uint64_t first, uint64_t nbins)
{
    const uint64_t i0 = first / 16, i1 = (first + nbins) / 16;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((i1 - i0 + 255) / 256, (uint64_t)q->cu_count * 8u);
    hipLaunchKernelGGL(hist_combine_kernel, dim3(grid), dim3(256), 0, q->stream, q->d_hist, q->d_lo, i0, i1, d_out);
    HIPCHK(hipGetLastError());
    return 0;
}

// Stream the u32 table view to the host in 64M-bin chunks: fn(host chunk, first bin, bins).
template <typename F>
int stream_table(dqdk_gpu_queue* q, F fn)
{
    const uint64_t chunk = 64ull << 20;
    uint32_t* d_stage = nullptr;
    uint32_t* h_stage = nullptr;
    hipError_t e = hipMalloc(&d_stage, chunk * sizeof(uint32_t));
    if (e == hipSuccess)
        e = hipHostMalloc(&h_stage, chunk * sizeof(uint32_t), hipHostMallocDefault);
    int rc = e == hipSuccess ? 0 : fail("histogram staging", e);
    for (uint64_t o = 0; rc == 0 && o < DQDK_TRISTAN_HISTO_ENTRIES; o += chunk) {
        const uint64_t m = std::min<uint64_t>(chunk, DQDK_TRISTAN_HISTO_ENTRIES - o);
        rc = combine(q, d_stage, o, m);
        if (rc == 0 && (e = hipMemcpyAsync(h_stage, d_stage, m * sizeof(uint32_t), hipMemcpyDeviceToHost, q->stream)) != hipSuccess)
            rc = fail("hipMemcpyAsync", e);
        if (rc == 0 && (e = hipStreamSynchronize(q->stream)) != hipSuccess)
            rc = fail("hipStreamSynchronize", e);
        if (rc == 0)
            fn(h_stage, o, m);
    }
    (void)hipFree(d_stage);
    if (h_stage)
        (void)hipHostFree(h_stage);
    return rc;
}

// Enqueue the raw payload gather of the batch just launched on q->stream;
// the byte total lands in q->d_raw_blk[nblk].
int launch_raw(dqdk_gpu_queue* q, const uint8_t* d_umem, uint64_t umem_size, const dqdk_gpu_desc_t* d_desc, uint32_t n,
               const dqdk_gpu_rx_result_t* d_res, uint8_t* d_out, uint64_t out_cap, bool copy)
{
    RawArgs ra{};
    ra.umem = d_umem;
    ra.umem_size = umem_size;
    ra.desc = d_desc;
    ra.res = d_res;
    ra.n = n;
    ra.flags = q->cfg.flags;
    ra.batch_scratch = q->d_batch;
    ra.blk = q->d_raw_blk;
    ra.out = d_out;
    ra.out_cap = out_cap;
    const uint32_t nblk = (n + kRawThreads - 1) / kRawThreads;
    hipLaunchKernelGGL(raw_len_kernel, dim3(nblk), dim3(kRawThreads), 0, q->stream, ra);
    hipLaunchKernelGGL(csv_scan_kernel, dim3(1), dim3(1024), 0, q->stream, q->d_raw_blk, nblk);
    if (copy)
        hipLaunchKernelGGL(raw_copy_kernel, dim3(nblk), dim3(kRawThreads), 0, q->stream, ra);
    HIPCHK(hipGetLastError());
    return 0;
}

int raw_total(dqdk_gpu_queue* q, uint32_t n, uint64_t* total)
{
    const uint32_t nblk = (n + kRawThreads - 1) / kRawThreads;
    HIPCHK(hipMemcpyAsync(total, q->d_raw_blk + nblk, sizeof(uint64_t), hipMemcpyDeviceToHost, q->stream));
    HIPCHK(hipStreamSynchronize(q->stream));
    return 0;
}

int write_fd(int fd, const uint8_t* p, uint64_t n)
{
    for (uint64_t o = 0; o < n;) {
        const ssize_t w = write(fd, p + o, n - o > (1u << 30) ? (1u << 30) : (size_t)(n - o));
        if (w < 0) {
            if (errno == EINTR)
                continue;
            const int err = errno;
            g_err = std::string("raw write: ") + strerror(err);
            return -err;
        }
        o += (uint64_t)w;
    }
    return 0;
}

int grow_dev(uint8_t** p, uint64_t* cap, uint64_t need)
{
    if (need <= *cap)
        return 0;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(p, need));
    *cap = need;
    return 0;
}

int grow_host(uint8_t** p, uint64_t* cap, uint64_t need)
{
    if (need <= *cap)
        return 0;
    if (*p)
        (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipHostMalloc(p, need, hipHostMallocDefault));
    *cap = need;
    return 0;
}

// write() the raw stream of buffer k once its D2H has landed
int raw_write_pending(dqdk_gpu_queue* q, int k)
{
    if (!q->raw_pend[k])
        return 0;
    q->raw_pend[k] = 0;
    HIPCHK(hipEventSynchronize(q->raw_ev_d2h[k]));
    return write_fd(q->raw_fd, q->h_rawb[k], q->raw_pend_len[k]);
}

// every batch's raw stream written (older buffer first).  Both D2H copies
// are waited for even when the first write() fails: nothing may still be in
// flight into h_rawb once this returns (destroy frees it next; a copy landing
// in freed pinned memory is a GPU fault reported at some later copy, DESIGN
// section 3)
int raw_drain(dqdk_gpu_queue* q)
{
    const int last = (int)((q->raw_seq + 1) & 1);  // buffer of the most recent batch
    int rc = raw_write_pending(q, last ^ 1);
    if (!rc)
        rc = raw_write_pending(q, last);
    if (q->raw_stream) {
        const hipError_t e = hipStreamSynchronize(q->raw_stream);  // (an unwritten batch stays pending)
        if (!rc && e != hipSuccess)
            rc = fail("raw egress: hipStreamSynchronize", e);
    }
    return rc;
}

// Synchronous form (the default, as tristan_process's write, src/tristan.c:
// 318-324): size query, gather, D2H and write() of the batch, all before the
// call returns.  Device / runtime failures are returned; the write()'s own
// result goes to *werr.
int write_raw_sync(dqdk_gpu_queue* q, const uint8_t* d_umem, uint64_t umem_size, uint32_t n, int* werr)
{
    *werr = 0;
    int rc = launch_raw(q, d_umem, umem_size, q->d_desc, n, q->d_res, nullptr, 0, false);
    uint64_t total = 0;
    if (!rc)
        rc = raw_total(q, n, &total);
    if (rc || !total)
        return rc;
    if ((rc = grow_dev(&q->d_rawb[0], &q->d_rawb_cap[0], total)) || (rc = grow_host(&q->h_rawb[0], &q->h_rawb_cap[0], total)))
        return rc;
    rc = launch_raw(q, d_umem, umem_size, q->d_desc, n, q->d_res, q->d_rawb[0], q->d_rawb_cap[0], true);
    if (rc)
        return rc;
    HIPCHK(hipMemcpyAsync(q->h_rawb[0], q->d_rawb[0], total, hipMemcpyDeviceToHost, q->stream));
    HIPCHK(hipStreamSynchronize(q->stream));
    *werr = write_fd(q->raw_fd, q->h_rawb[0], total);
    return 0;
}

}  // namespace

// ---- runtime-internal entry points (queue_internal.h) -----------------------
namespace dqdk {

int queue_launch_payloads(dqdk_gpu_queue_t* q, const uint8_t* d_stage, const uint32_t* d_len, uint32_t n)
{
    if (!q || n > q->max_batch || (n && !d_len) || (n && q->histo && q->E && !d_stage))
        return fail_errno(-EINVAL, "launch_payloads: bad argument");
    if (n == 0)
        return 0;
    SETDEV(q->device);
    return launch_payloads(q, d_stage, d_len, n);
}

int queue_device(const dqdk_gpu_queue_t* q) { return q ? q->device : -1; }

uint32_t queue_events(const dqdk_gpu_queue_t* q) { return q && q->histo ? q->E : 0u; }

int set_error(int err, const char* what) { return fail_errno(err, what); }

int set_hip_error(const char* what, hipError_t e) { return fail(what, e); }

}  // namespace dqdk

extern "C" {

int dqdk_gpu_abi_version(void) { return DQDK_GPU_ABI_VERSION; }

const char* dqdk_gpu_last_error(void) { return g_err.c_str(); }

int dqdk_gpu_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

int dqdk_gpu_queue_create(int device, const dqdk_gpu_cfg_t* cfg, uint32_t max_batch, dqdk_gpu_queue_t** out)
{
    if (!cfg || !out || max_batch == 0)
        return fail_errno(-EINVAL, "queue_create: bad argument");
    *out = nullptr;
    if (cfg->mode > DQDK_MODE_ENERGYHISTO || cfg->payloadsz > (16u << 20))
        return fail_errno(-EINVAL, "queue_create: bad mode or payloadsz");
    // E <= 65535: a UDP datagram carries at most 65507 B, and the per-frame
    // out-of-bounds count (u16 in dqdk_gpu_rx_result_t) can then never clamp
    if (events_per_payload(cfg->mode, cfg->payloadsz) > 0xffffu)
        return fail_errno(-EINVAL, "queue_create: payloadsz / 16 must be <= 65535 events");
    if ((uint64_t)max_batch * events_per_payload(cfg->mode, cfg->payloadsz) >= (1ull << 31))
        return fail_errno(-EINVAL, "queue_create: max_batch * events per frame must be < 2^31");
    int ndev = dqdk_gpu_device_count();
    if (device < 0 || device >= ndev)
        return fail_errno(-ENODEV, "queue_create: no such HIP device");
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail_errno(-ENODEV, "queue_create: device is not gfx950 (MI355X)");
    SETDEV(device);

    dqdk_gpu_queue* q = new dqdk_gpu_queue();
    q->device = device;
    q->cfg = *cfg;
    q->E = events_per_payload(cfg->mode, cfg->payloadsz);
    q->max_batch = max_batch;
    q->histo = !(cfg->flags & DQDK_GPU_F_NO_HISTO) &&
               (cfg->mode == DQDK_MODE_LISTWAVE || cfg->mode == DQDK_MODE_LISTMODE ||
                cfg->mode == DQDK_MODE_ENERGYHISTO);  // is_store_histo, src/tristan.c:65-70
    q->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    q->dec_cus = q->cu_count;
    if (const char* v = getenv("DQDK_GPU_DECODE_CUS"))
        q->dec_cus = std::max(1, std::min(q->cu_count, atoi(v)));
    q->alloc_kind = internal_alloc_kind(q->E);
    if (int rc = read_knobs(q)) {
        delete q;
        return rc;
    }
    if (cfg->flags & DQDK_GPU_F_HISTO_ATOMIC)
        q->histo_path = 1;
    else if (cfg->flags & DQDK_GPU_F_HISTO_PARTITIONED)
        q->histo_path = 2;

    auto cleanup = [&](int rc) {
        const std::string why = g_err;  // (the creation failure is the one reported)
        (void)dqdk_gpu_queue_destroy(q);
        g_err = why;
        return rc;
    };
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&q->own_stream, hipStreamNonBlocking)) != hipSuccess)
        return cleanup(fail("hipStreamCreate", e));
    q->stream = q->own_stream;
    if ((e = hipMalloc(&q->d_cum, sizeof(dqdk_gpu_counters_t))) != hipSuccess ||
        (e = hipMalloc(&q->d_batch, kBatchScratch * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMalloc(&q->d_desc, (size_t)max_batch * sizeof(dqdk_gpu_desc_t))) != hipSuccess ||
        (e = hipMalloc(&q->d_res, (size_t)max_batch * sizeof(dqdk_gpu_rx_result_t))) != hipSuccess ||
        (e = hipMalloc(&q->d_raw_blk, ((size_t)max_batch / kRawThreads + 2) * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMalloc(&q->d_blkcnt, kFoldWords * sizeof(uint64_t))) != hipSuccess)
        return cleanup((fail("hipMalloc", e), -ENOMEM));
    {
        uint64_t acc0[kFoldWords] = {};
        acc0[9] = ~0ull;  // the first-failure accumulator (FoldWord F_FAIL)
        if ((e = hipMemcpy(q->d_blkcnt, acc0, sizeof(acc0), hipMemcpyHostToDevice)) != hipSuccess)
            return cleanup(fail("hipMemcpy", e));
    }
    if ((e = hipMemset(q->d_cum, 0, sizeof(dqdk_gpu_counters_t))) != hipSuccess ||
        (e = hipMemset(q->d_batch, 0, kBatchScratch * sizeof(uint64_t))) != hipSuccess)
        return cleanup(fail("hipMemset", e));
    if (q->histo) {
        // the fused path's overflow-list length, written by rx_part2 into host
        // memory the host reads without a sync (launch_histo's grouping choice)
        if ((e = hipHostMalloc(&q->h_ovf, sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent)) !=
                hipSuccess ||
            (e = hipHostGetDevicePointer((void**)&q->h_ovf_dev, q->h_ovf, 0)) != hipSuccess)
            return cleanup(fail("hipHostMalloc(overflow length)", e));
        *q->h_ovf = 0;
    }
    if (q->histo) {
        if ((e = dev_alloc(&q->d_hist, DQDK_TRISTAN_HISTO_ENTRIES * sizeof(uint32_t), q->alloc_kind)) != hipSuccess ||
            (e = dev_alloc(&q->d_lo, DQDK_TRISTAN_HISTO_ENTRIES, q->alloc_kind)) != hipSuccess)
            return cleanup((fail("hipMalloc(histogram)", e), -ENOMEM));
        if ((e = hipMemset(q->d_hist, 0, DQDK_TRISTAN_HISTO_ENTRIES * sizeof(uint32_t))) != hipSuccess ||
            (e = hipMemset(q->d_lo, 0, DQDK_TRISTAN_HISTO_ENTRIES)) != hipSuccess ||
            (e = hipStreamSynchronize(nullptr)) != hipSuccess)  // (the fills complete, or fail, here)
            return cleanup(fail("hipMemset(histogram)", e));
        if (q->E) {
            const size_t nk = (size_t)max_batch * q->E;
            q->nk_max = nk;
            q->scratch_words = kHistScratchWords;
            // part2: item i of a staged batch at [i * kPartChunk, + keys)
            q->part2_stride = (size_t)max_items(nk) * kPartChunk;
            q->runs_stride = ((size_t)max_items(nk) * kItemOffs + 7) & ~(size_t)7;
            // fused decode's per-block overflow regions: ovf_cap_blk keys each
            // (an eighth of a block's keys, at least 64K: the 9000 B batches
            // overflow ~3 % of their keys, 1500 B ones far fewer); past that
            // a key is added to the table by a device atomic (exact, rare)
            const FusedGeom fg = fused_geom(max_batch, q->E, (uint64_t)q->dec_cus);
            const uint64_t nsuper = ((uint64_t)max_batch + 64 * kFWaves - 1) / (64 * kFWaves);
            const uint64_t blk_keys = ((nsuper + fg.grid - 1) / fg.grid) * (64 * kFWaves) * q->E;
            uint64_t ocap = std::min<uint64_t>(blk_keys, std::max<uint64_t>(65536, blk_keys / 8));
            if (const char* v = getenv("DQDK_GPU_OVF_BLK"))  // (test hook: forces the atomic spill)
                ocap = std::min<uint64_t>(blk_keys, std::max<uint64_t>(64, strtoull(v, nullptr, 0)));
            q->ovf_cap_blk = (uint32_t)ocap;
            q->ovf_blk_elems = (uint64_t)fg.grid * ocap;
            // part1 holds the fused decode's pieces, then rx_part1's grouped
            // copy of the overflow list, which also backs the decode's
            // overflow regions (dead before rx_part1 writes it); the fused
            // pieces at max_batch bound those of any smaller batch; gathered
            // items address them in 32-bit byte offsets per bucket.  The
            // records path (frame-order keys) allocates its buffers on first
            // use (ensure_records): the fused path needs neither.
            q->fused_elems = fg.region * 4u < (1ull << 31) && (uint64_t)kL1Buckets * fg.region < (1ull << 32)
                                 ? (uint64_t)kL1Buckets * fg.region
                                 : 0u;
            if (q->fused_elems) {
                q->part1_elems = q->piece_shift + q->fused_elems + q->ovf_blk_elems + kStagePad;
                if ((e = dev_alloc(&q->d_part1, q->part1_elems * 4, q->alloc_kind)) != hipSuccess ||
                    (e = hipMalloc(&q->d_ovf, q->ovf_blk_elems * sizeof(uint32_t))) != hipSuccess)
                    return cleanup((fail("hipMalloc(histogram staging)", e), -ENOMEM));
                // (the overflow regions sit past every shifted piece region; rx_part1's
                // output, written once they are dead, may overlap them)
                q->d_ovf_blk = q->d_part1 + q->piece_shift + q->fused_elems;
            }
            if (cfg->flags & (DQDK_GPU_F_BATCH_ABORT | DQDK_GPU_F_HISTO_UNFUSED)) {
                if (int rc = ensure_records(q, true, true))  // records path every batch
                    return cleanup(rc);
            }
            // Stage up to kHistKMax batches per slice pass (the low-byte sweep
            // of a touched slice is amortised over them; the pass drains its
            // packed-u16 bins between groups of events, so any count of
            // events per slice fits), as many as the staging budget holds:
            // 24 GiB, or a quarter of the device memory still free (ADVICE r3:
            // several queues per GPU), halved while an allocation fails;
            // DQDK_GPU_F_HISTO_EAGER: a pass per batch.
            const size_t slot_bytes = q->part2_stride * 2 + q->runs_stride * 2 + q->scratch_words * 4;
            size_t budget = kHistStageBytes;
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b / 4 < budget)
                budget = free_b / 4;
            uint32_t k = (cfg->flags & DQDK_GPU_F_HISTO_EAGER)
                             ? 1u
                             : (uint32_t)std::max<size_t>(1, std::min(kHistKMax, budget / slot_bytes));
            for (;; k /= 2) {
                if ((e = dev_alloc(&q->d_part2, k * q->part2_stride * 2, q->alloc_kind)) == hipSuccess &&
                    (e = dev_alloc(&q->d_runs, k * q->runs_stride * sizeof(uint16_t), q->alloc_kind)) == hipSuccess &&
                    (e = dev_alloc(&q->d_hscratch, k * q->scratch_words * sizeof(uint32_t), q->alloc_kind)) == hipSuccess)
                    break;
                (void)hipGetLastError();
                dev_free(q->d_part2);
                dev_free(q->d_runs);
                dev_free(q->d_hscratch);
                q->d_part2 = nullptr;
                q->d_runs = nullptr;
                q->d_hscratch = nullptr;
                if (k == 1)
                    return cleanup((fail("hipMalloc(histogram staging)", e), -ENOMEM));
            }
            q->hist_k = k;
            // every slot's per-batch words zero from the start, so no batch
            // of the first slice pass pays clean_slot's memsets (four fill
            // launches per batch; a long capture's later passes find the
            // slots re-zeroed by rx_part2 anyway)
            if ((e = hipMemset(q->d_hscratch, 0, (size_t)k * q->scratch_words * sizeof(uint32_t))) != hipSuccess ||
                (e = hipStreamSynchronize(nullptr)) != hipSuccess)
                return cleanup(fail("hipMemset(slot scratch)", e));
            q->slot_dirty.assign(k, 0);
        }
    }
    *out = q;
    return 0;
}

int dqdk_gpu_device_alloc(int device, uint64_t size, void** d_out)
{
    if (!d_out || !size)
        return fail_errno(-EINVAL, "device_alloc: bad argument");
    *d_out = nullptr;
    if (device < 0 || device >= dqdk_gpu_device_count())
        return fail_errno(-ENODEV, "device_alloc: no such HIP device");
    SETDEV(device);
    void* p = nullptr;
    const int want = image_alloc_kind();
    int got = kAllocPlain;
    hipError_t e = dev_alloc(&p, size, want, &got);
    if (e != hipSuccess)
        return (fail("device_alloc", e), -ENOMEM);
    *d_out = p;
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        g_allocs.emplace_back((uintptr_t)p, size);
    }
    return got == kAllocContig ? 0 : 1;  // 0 only for a physically contiguous range
}

int dqdk_gpu_device_free(int device, void* d_ptr)
{
    if (!d_ptr)
        return 0;
    if (device < 0 || device >= dqdk_gpu_device_count())
        return fail_errno(-ENODEV, "device_free: no such HIP device");
    SETDEV(device);
    {
        std::lock_guard<std::mutex> lk(g_alloc_mu);
        for (size_t k = 0; k < g_allocs.size(); k++)
            if (g_allocs[k].first == (uintptr_t)d_ptr) {
                g_allocs.erase(g_allocs.begin() + (long)k);
                break;
            }
    }
    HIPCHK(hipFree(d_ptr));
    return 0;
}

int dqdk_gpu_queue_destroy(dqdk_gpu_queue_t* q)
{
    if (!q)
        return -EINVAL;
    DevGuard dev_guard_(q->device);
    // Every call is checked and the first failure returned, naming the call
    // (a fault in a queue's last work or in its teardown must
    // fail the caller that destroys it, not surface at some later copy).
    // Everything is still released whatever fails.
    int rc = 0;
    std::string first;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && !rc) {
            first = std::string("queue_destroy: ") + what + ": " + hipGetErrorString(e);
            rc = -EIO;
        }
    };
    if (dev_guard_.e != hipSuccess)
        chk(dev_guard_.e, "hipSetDevice");
    if (q->raw_fd >= 0) {  // the last batch's raw stream still goes to its file
        const int wrc = raw_drain(q);
        if (wrc) {
            fprintf(stderr, "dqdk_gpu_queue_destroy: the last deferred raw batch was not written to fd %d: %s\n",
                    q->raw_fd, strerror(-wrc));
            if (!rc) {
                first = "queue_destroy: raw drain: " + g_err;
                rc = wrc;
            }
        }
    }
    if (q->stream)
        chk(hipStreamSynchronize(q->stream), "hipStreamSynchronize(queue stream)");
    if (q->raw_stream)
        chk(hipStreamSynchronize(q->raw_stream), "hipStreamSynchronize(raw stream)");  // no D2H into h_rawb may outlive it
    for (auto& r : q->regs)
        chk(greg_release(r.base), "hipHostUnregister(umem)");
    for (auto& p : q->pending) {
        chk(hipEventDestroy(p.a), "hipEventDestroy(timing)");
        chk(hipEventDestroy(p.b), "hipEventDestroy(timing)");
    }
    for (auto ev : q->ev_free)
        chk(hipEventDestroy(ev), "hipEventDestroy(timing)");
    auto dfree = [&](void* p, const char* what) {
        if (p)
            chk(hipFree(p), what);
    };
    auto hfree = [&](void* p, const char* what) {
        if (p)
            chk(hipHostFree(p), what);
    };
    dfree(q->d_hist, "hipFree(table)");
    dfree(q->d_lo, "hipFree(table low plane)");
    dfree(q->d_snap, "hipFree(table snapshot)");
    dfree(q->d_cum, "hipFree(counters)");
    dfree(q->d_batch, "hipFree(batch scratch)");
    dfree(q->d_blkcnt, "hipFree(fold accumulators)");
    dfree(q->d_keys, "hipFree(records)");
    for (int k = 0; k < kProbeCands; k++)
        if (q->part1_cand[k] && q->part1_cand[k] != q->d_part1)
            dfree(q->part1_cand[k], "hipFree(probe candidate)");
    dfree(q->d_part1, "hipFree(pieces)");
    for (auto ev : q->probe_ev)
        if (ev)
            chk(hipEventDestroy(ev), "hipEventDestroy(probe)");
    dfree(q->d_part1_rec, "hipFree(records part1)");
    dfree(q->d_ovf, "hipFree(overflow list)");
    dfree(q->d_part2, "hipFree(part2 staging)");
    dfree(q->d_runs, "hipFree(part2 runs)");
    dfree(q->d_hscratch, "hipFree(slot scratch)");
    dfree(q->d_desc, "hipFree(descriptors)");
    dfree(q->d_res, "hipFree(results)");
    dfree(q->d_raw_blk, "hipFree(raw offsets)");
    for (int k = 0; k < 2; k++) {
        dfree(q->d_rawb[k], "hipFree(raw buffer)");
        hfree(q->h_rawb[k], "hipHostFree(raw buffer)");
        if (q->raw_ev_d2h[k])
            chk(hipEventDestroy(q->raw_ev_d2h[k]), "hipEventDestroy(raw)");
    }
    hfree(q->h_raw_total, "hipHostFree(raw total)");
    hfree(q->h_desc, "hipHostFree(pinned descriptors)");
    hfree(q->h_res, "hipHostFree(pinned results)");
    hfree(q->h_batch, "hipHostFree(pinned counters)");
    hfree(q->h_ovf, "hipHostFree(overflow length)");
    if (q->ev_read)
        chk(hipEventDestroy(q->ev_read), "hipEventDestroy(ev_read)");
    if (q->raw_stream)
        chk(hipStreamDestroy(q->raw_stream), "hipStreamDestroy(raw stream)");
    if (q->switch_ev)
        chk(hipEventDestroy(q->switch_ev), "hipEventDestroy(switch)");
    dfree(q->d_async, "hipFree(async bursts)");
    if (q->own_stream)
        chk(hipStreamDestroy(q->own_stream), "hipStreamDestroy(queue stream)");
    // and nothing of the device's still-running work faulted: a sticky error
    // of this queue's kernels or copies is reported here, by the destroy
    chk(hipDeviceSynchronize(), "hipDeviceSynchronize");
    delete q;
    if (rc)
        g_err = first;
    return rc;
}

int dqdk_gpu_queue_set_stream(dqdk_gpu_queue_t* q, void* s)
{
    if (!q)
        return -EINVAL;
    hipStream_t ns = (hipStream_t)s;  // verbatim: NULL is the legacy default stream
    if (ns == q->stream)
        return 0;
    // work already enqueued on the old stream (a batch, staged slice passes)
    // is ordered before anything enqueued on the new one
    SETDEV(q->device);
    if (!q->switch_ev)
        HIPCHK(hipEventCreateWithFlags(&q->switch_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(q->switch_ev, q->stream));
    HIPCHK(hipStreamWaitEvent(ns, q->switch_ev, 0));
    q->stream = ns;
    return 0;
}

void* dqdk_gpu_queue_own_stream(dqdk_gpu_queue_t* q) { return q ? (void*)q->own_stream : nullptr; }

void* dqdk_gpu_queue_stream(dqdk_gpu_queue_t* q) { return q ? (void*)q->stream : nullptr; }

int dqdk_gpu_rx_batch_device(dqdk_gpu_queue_t* q, const uint8_t* d_umem, uint64_t umem_size,
                             const dqdk_gpu_desc_t* d_desc, uint32_t n, dqdk_gpu_rx_result_t* d_results,
                             uint32_t* d_keys)
{
    if (!q || !d_umem || !d_desc || !d_results)
        return fail_errno(-EINVAL, "rx_batch_device: null argument");
    if (n > q->max_batch)
        return fail_errno(-EINVAL, "rx_batch_device: n > max_batch");
    if (umem_size % 16)
        return fail_errno(-EINVAL, "rx_batch_device: umem_size must be a multiple of 16");
    if (n == 0)
        return 0;
    SETDEV(q->device);
    int rc;
    if ((rc = check_range(d_umem, umem_size, "rx_batch_device: d_umem")) ||
        (rc = check_range(d_desc, (uint64_t)n * sizeof(dqdk_gpu_desc_t), "rx_batch_device: d_desc")) ||
        (rc = check_range(d_results, (uint64_t)n * sizeof(dqdk_gpu_rx_result_t), "rx_batch_device: d_results")) ||
        (rc = check_range(d_keys, (uint64_t)n * q->E * 4u, "rx_batch_device: d_keys")))
        return rc;
    return launch_batch(q, d_umem, umem_size, d_desc, n, d_results, d_keys);
}

int dqdk_gpu_queue_sync(dqdk_gpu_queue_t* q)
{
    if (!q)
        return -EINVAL;
    SETDEV(q->device);
    if (int rc = raw_drain(q))
        return rc;
    HIPCHK(hipStreamSynchronize(q->stream));
    return 0;
}

int dqdk_gpu_umem_register(dqdk_gpu_queue_t* q, void* umem, uint64_t size)
{
    if (!q || !umem || !size)
        return -EINVAL;
    SETDEV(q->device);
    bool own = false;
    for (size_t k = 0; k < q->regs.size(); k++) {
        if (q->regs[k].host != umem)
            continue;
        if (q->regs[k].size >= size)
            return 0;
        // the same address with more bytes (a larger buffer in the old one's
        // place, or a grown view): the registration is replaced, never
        // reused past its end (this queue's work on it drained first)
        HIPCHK(hipStreamSynchronize(q->stream));
        void* const old_base = q->regs[k].base;
        q->regs.erase(q->regs.begin() + (long)k);
        if (old_base != umem)  // (it was a view inside another registration: that reference goes)
            HIPCHK(greg_release(old_base));
        else
            own = true;
        break;
    }
    void* dev = nullptr;
    void* base = umem;
    bool kept = false;
    if (int rc = greg_acquire(umem, size, own, &dev, &kept, &base)) {
        if (kept)  // (the smaller registration this queue held: still its reference, released later)
            q->regs.push_back({umem, 0, nullptr, umem});
        return rc;
    }
    q->regs.push_back({umem, size, dev, base});
    return 0;
}

int dqdk_gpu_umem_unregister(dqdk_gpu_queue_t* q, void* umem)
{
    if (!q)
        return -EINVAL;
    for (size_t k = 0; k < q->regs.size(); k++) {
        if (q->regs[k].host == umem) {
            SETDEV(q->device);
            HIPCHK(hipStreamSynchronize(q->stream));
            void* const base = q->regs[k].base;
            q->regs.erase(q->regs.begin() + (long)k);
            HIPCHK(greg_release(base));
            return 0;
        }
    }
    return -ENOENT;
}

int dqdk_gpu_rx_batch(dqdk_gpu_queue_t* q, const uint8_t* umem, uint64_t umem_size, const dqdk_gpu_desc_t* d,
                      uint32_t n, dqdk_gpu_rx_result_t* per_pkt, dqdk_gpu_counters_t* delta)
{
    if (!q || !umem || !d || !per_pkt)
        return fail_errno(-EINVAL, "rx_batch: null argument");
    if (n > q->max_batch)
        return fail_errno(-EINVAL, "rx_batch: n > max_batch");
    if (umem_size % 16)
        return fail_errno(-EINVAL, "rx_batch: umem_size must be a multiple of 16");
    if (n == 0) {
        if (delta)
            memset(delta, 0, sizeof(*delta));
        return 0;
    }
    SETDEV(q->device);
    const Reg* reg = nullptr;
    for (auto& r : q->regs)
        if ((const uint8_t*)r.host <= umem && umem + umem_size <= (const uint8_t*)r.host + r.size)
            reg = &r;
    if (!reg) {  // the worker registers its UMEM once (src/dqdk-mem.c:12-28 mmap+mlock)
        int rc = dqdk_gpu_umem_register(q, (void*)umem, umem_size);
        if (rc)
            return rc;
        for (auto& r : q->regs)
            if ((const uint8_t*)r.host <= umem && umem + umem_size <= (const uint8_t*)r.host + r.size)
                reg = &r;
        if (!reg)
            return fail_errno(-EINVAL, "rx_batch: umem not covered by its registration");
    }
    const uint8_t* dev_umem = (const uint8_t*)reg->dev + (umem - (const uint8_t*)reg->host);
    if (q->raw_fd < 0) {
        // the fast form: pinned descriptors / results / counters, return at ev_read
        if (!q->h_desc) {
            const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
            hipError_t e;
            if ((e = hipHostMalloc(&q->h_desc, (size_t)q->max_batch * sizeof(dqdk_gpu_desc_t), fl)) != hipSuccess ||
                (e = hipHostMalloc(&q->h_res, (size_t)q->max_batch * sizeof(dqdk_gpu_rx_result_t), fl)) != hipSuccess ||
                (e = hipHostMalloc(&q->h_batch, kBatchScratch * sizeof(uint64_t), fl)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&q->h_desc_dev, q->h_desc, 0)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&q->h_res_dev, q->h_res, 0)) != hipSuccess ||
                (e = hipHostGetDevicePointer((void**)&q->h_batch_dev, q->h_batch, 0)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&q->ev_read, hipEventDisableTiming)) != hipSuccess)
                return fail("rx_batch: pinned buffers", e);
        }
        memcpy(q->h_desc, d, (size_t)n * sizeof(*d));
        q->publish = true;
        int rc = launch_batch(q, dev_umem, umem_size, q->h_desc_dev, n, q->d_res, nullptr);
        q->publish = false;
        hipError_t e = rc ? hipSuccess : hipEventSynchronize(q->ev_read);
        if (rc || e != hipSuccess) {  // nothing of the batch may still run once we return
            const hipError_t e2 = hipStreamSynchronize(q->stream);
            return rc ? rc : fail("rx_batch: hipEventSynchronize", e != hipSuccess ? e : e2);
        }
        memcpy(per_pkt, q->h_res, (size_t)n * sizeof(*per_pkt));
        if (delta)
            memcpy(delta, &q->h_batch[1], sizeof(*delta));
        return 0;
    }
    HIPCHK(hipMemcpyAsync(q->d_desc, d, (size_t)n * sizeof(*d), hipMemcpyHostToDevice, q->stream));
    // Once the batch is enqueued, no path returns before the queue stream has
    // drained: its kernels read the caller's frames (valid only until this
    // call returns, src/dqdk.c:300) and its copies land in per_pkt and in this
    // frame's b[].
    auto drained = [&](int err) {
        const hipError_t e = hipStreamSynchronize(q->stream);
        return err ? err : e != hipSuccess ? fail("hipStreamSynchronize", e) : 0;
    };
    int rc = launch_batch(q, dev_umem, umem_size, q->d_desc, n, q->d_res, nullptr);
    if (rc)
        return drained(rc);
    const bool raw = q->raw_fd >= 0 && q->raw_deferred;
    int swerr = 0;  // the synchronous form's write() result, returned once the batch is delivered
    const int k = (int)(q->raw_seq & 1);
    uint64_t cap = 0;
    hipError_t e = hipSuccess;
    if (raw) {
        // the batch's raw stream (tristan.c:318-324) is gathered into buffer k
        // now (the frames are valid only until this call returns, dqdk.c:300);
        // capacity: the frames' bytes (a payload lies inside its frame unless
        // its datalen wrapped, handled below by a second gather)
        if (!q->raw_stream) {
            if ((e = hipStreamCreateWithFlags(&q->raw_stream, hipStreamNonBlocking)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&q->raw_ev_d2h[0], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&q->raw_ev_d2h[1], hipEventDisableTiming)) != hipSuccess ||
                (e = hipHostMalloc(&q->h_raw_total, sizeof(uint64_t), hipHostMallocDefault)) != hipSuccess)
                return drained(fail("raw egress setup", e));
        }
        uint64_t guess = 0;
        for (uint32_t i = 0; i < n; i++)
            guess += d[i].len;
        if ((rc = grow_dev(&q->d_rawb[k], &q->d_rawb_cap[k], std::max<uint64_t>(guess, 4096))) != 0)
            return drained(rc);
        cap = q->d_rawb_cap[k];
        if ((rc = launch_raw(q, dev_umem, umem_size, q->d_desc, n, q->d_res, q->d_rawb[k], cap, true)) != 0)
            return drained(rc);
        const uint32_t nblk = (n + kRawThreads - 1) / kRawThreads;
        if ((e = hipMemcpyAsync(q->h_raw_total, q->d_raw_blk + nblk, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                q->stream)) != hipSuccess)
            return drained(fail("hipMemcpyAsync", e));
    } else if (q->raw_fd >= 0 && (rc = write_raw_sync(q, dev_umem, umem_size, n, &swerr)) != 0) {
        return drained(rc);
    }
    uint64_t b[kBatchScratch];
    if ((e = hipMemcpyAsync(per_pkt, q->d_res, (size_t)n * sizeof(*per_pkt), hipMemcpyDeviceToHost, q->stream)) !=
            hipSuccess ||
        (e = hipMemcpyAsync(b, q->d_batch, sizeof(b), hipMemcpyDeviceToHost, q->stream)) != hipSuccess)
        return drained(fail("hipMemcpyAsync", e));
    // the previous batch's raw stream goes to its file while this batch runs;
    // a failed write() is returned after this batch is complete (its own raw
    // stream still queued for the next write)
    const int werr = raw ? raw_write_pending(q, k ^ 1) : 0;
    if ((rc = drained(0)) != 0)
        return rc;
    if (delta)
        memcpy(delta, &b[1], sizeof(*delta));
    if (raw) {
        const uint64_t total = *q->h_raw_total;
        if (total > cap) {  // wrapped datalen inside the UMEM: gather again at full size
            // (capacity grows geometrically and is kept: batches with such
            // frames reallocate rarely)
            if ((rc = grow_dev(&q->d_rawb[k], &q->d_rawb_cap[k], std::max(total, 2 * cap))) != 0 ||
                (rc = launch_raw(q, dev_umem, umem_size, q->d_desc, n, q->d_res, q->d_rawb[k], total, true)) != 0)
                return drained(rc);
        }
        if (total) {
            if ((rc = grow_host(&q->h_rawb[k], &q->h_rawb_cap[k], total)) != 0)
                return drained(rc);
            if ((e = hipEventRecord(q->raw_ev_d2h[k], q->stream)) != hipSuccess ||  // after the gather
                (e = hipStreamWaitEvent(q->raw_stream, q->raw_ev_d2h[k], 0)) != hipSuccess ||
                (e = hipMemcpyAsync(q->h_rawb[k], q->d_rawb[k], total, hipMemcpyDeviceToHost, q->raw_stream)) !=
                    hipSuccess ||
                (e = hipEventRecord(q->raw_ev_d2h[k], q->raw_stream)) != hipSuccess)
                return drained(fail("raw egress D2H", e));
            q->raw_pend[k] = 1;
            q->raw_pend_len[k] = total;
        }
        q->raw_seq++;
        if (total > cap && (rc = drained(0)) != 0)  // the second gather read the frames: done before returning
            return rc;
    }
    return werr ? werr : swerr;
}

int dqdk_gpu_counters_get(dqdk_gpu_queue_t* q, dqdk_gpu_counters_t* out)
{
    if (!q || !out)
        return -EINVAL;
    SETDEV(q->device);
    HIPCHK(hipMemcpyAsync(out, q->d_cum, sizeof(*out), hipMemcpyDeviceToHost, q->stream));
    HIPCHK(hipStreamSynchronize(q->stream));
    return 0;
}

int dqdk_gpu_counters_reset(dqdk_gpu_queue_t* q)
{
    if (!q)
        return -EINVAL;
    SETDEV(q->device);
    HIPCHK(hipMemsetAsync(q->d_cum, 0, sizeof(dqdk_gpu_counters_t), q->stream));
    return 0;
}

int dqdk_gpu_histogram_get(dqdk_gpu_queue_t* q, uint32_t* host_hist)
{
    if (!q || !host_hist)
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_get: queue has no histogram");
    SETDEV(q->device);
    if (int rc = hist_flush(q))
        return rc;
    return stream_table(q, [&](const uint32_t* h, uint64_t o, uint64_t m) {
        memcpy(host_hist + o, h, m * sizeof(uint32_t));
    });
}

int dqdk_gpu_histogram_accumulate(dqdk_gpu_queue_t* q, uint32_t* host_hist)
{
    if (!q || !host_hist)
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_accumulate: queue has no histogram");
    SETDEV(q->device);
    if (int rc = hist_flush(q))
        return rc;
    return stream_table(q, [&](const uint32_t* h, uint64_t o, uint64_t m) {
        for (uint64_t k = 0; k < m; k++)
            host_hist[o + k] += h[k];  // u32 wrap, like the shared atomic table
    });
}

int dqdk_gpu_histogram_reset(dqdk_gpu_queue_t* q)
{
    if (!q)
        return -EINVAL;
    if (!q->d_hist)
        return 0;
    SETDEV(q->device);
    q->hist_pending = 0;  // staged batches are dropped with the table
    HIPCHK(hipMemsetAsync(q->d_hist, 0, DQDK_TRISTAN_HISTO_ENTRIES * sizeof(uint32_t), q->stream));
    HIPCHK(hipMemsetAsync(q->d_lo, 0, DQDK_TRISTAN_HISTO_ENTRIES, q->stream));
    return 0;
}

uint32_t* dqdk_gpu_histogram_device_ptr(dqdk_gpu_queue_t* q)
{
    if (!q || !q->d_hist)
        return nullptr;
    DevGuard dev_guard_(q->device);
    if (dev_guard_.e != hipSuccess)
        return nullptr;
    if (!q->d_snap && dev_alloc(&q->d_snap, DQDK_TRISTAN_HISTO_ENTRIES * sizeof(uint32_t), q->alloc_kind) != hipSuccess) {
        q->d_snap = nullptr;
        return nullptr;
    }
    if (hist_flush(q) != 0 || combine(q, q->d_snap, 0, DQDK_TRISTAN_HISTO_ENTRIES) != 0 ||
        hipStreamSynchronize(q->stream) != hipSuccess)
        return nullptr;
    return q->d_snap;
}

int dqdk_gpu_timing_enable(dqdk_gpu_queue_t* q, int on)
{
    if (!q)
        return -EINVAL;
    q->timing = on ? 1 : 0;
    return 0;
}

int dqdk_gpu_timing_stages(dqdk_gpu_queue_t* q, uint32_t stage_mask)
{
    if (!q)
        return -EINVAL;
    q->stage_mask = stage_mask;
    return 0;
}

int dqdk_gpu_queue_staging_probe(dqdk_gpu_queue_t* q, int* chosen, float* ns_per_frame, int ncand)
{
    if (!q)
        return -EINVAL;
    if (chosen)  // (-2: off, or given up -- no probe step left and nothing kept)
        *chosen = q->probe == 0 && q->probe_chosen < 0 ? -2 : q->probe_chosen;
    for (int k = 0; ns_per_frame && k < ncand && k < kProbeCands; k++)
        ns_per_frame[k] = q->probe_cnt[k] ? q->probe_ms[k] / (float)q->probe_cnt[k] : 0.f;
    return kProbeCands;
}

int dqdk_gpu_timing_read(dqdk_gpu_queue_t* q, double* stage_ms, uint64_t* counts, int nstages)
{
    if (!q)
        return -EINVAL;
    SETDEV(q->device);
    HIPCHK(hipStreamSynchronize(q->stream));
    for (auto& p : q->pending) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        q->stage_ms[p.stage] += ms;
        q->counts[p.stage] += 1;
        q->ev_free.push_back(p.a);
        q->ev_free.push_back(p.b);
    }
    q->pending.clear();
    for (int k = 0; k < nstages && k < kStages; k++) {
        if (stage_ms)
            stage_ms[k] = q->stage_ms[k];
        if (counts)
            counts[k] = q->counts[k];
        q->stage_ms[k] = 0;
        q->counts[k] = 0;
    }
    return 0;
}

int dqdk_gpu_raw_compact_device(dqdk_gpu_queue_t* q, const uint8_t* d_umem, uint64_t umem_size,
                                const dqdk_gpu_desc_t* d_desc, uint32_t n, const dqdk_gpu_rx_result_t* d_results,
                                uint8_t* d_out, uint64_t out_cap, uint64_t* total)
{
    if (!q || !d_umem || !d_desc || !d_results || (!d_out && out_cap))
        return fail_errno(-EINVAL, "raw_compact_device: null argument");
    if (n > q->max_batch)
        return fail_errno(-EINVAL, "raw_compact_device: n > max_batch");
    if (n == 0) {
        if (total)
            *total = 0;
        return 0;
    }
    SETDEV(q->device);
    int rc = launch_raw(q, d_umem, umem_size, d_desc, n, d_results, d_out, out_cap, d_out != nullptr);
    if (!rc && total)
        rc = raw_total(q, n, total);
    return rc;
}

int dqdk_gpu_async_process_device(dqdk_gpu_queue_t* q, const uint8_t* d_ring, uint64_t nelem, const uint32_t* bursts,
                                  uint32_t nbursts, int strip_wfm, uint8_t* d_out, uint64_t out_cap, uint64_t* total)
{
    if (!q || (!d_ring && nelem) || (!bursts && nbursts) || (!d_out && out_cap))
        return fail_errno(-EINVAL, "async_process_device: null argument");
    const uint32_t P = q->cfg.payloadsz;
    // cne_ring elements are multiples of 4 B (src/ds/cne_ring.c:41): the
    // reference cannot create its ring otherwise
    if (P == 0 || (P & 3))
        return fail_errno(-EINVAL, "async_process_device: payloadsz must be a non-zero multiple of 4");
    const uint32_t len = strip_wfm ? 16u : P;  // src/tristan.c:343
    std::vector<uint32_t> b((size_t)nbursts * 4);
    uint64_t e0 = 0, off = 0;
    for (uint32_t k = 0; k < nbursts; k++) {
        if (e0 + bursts[k] > nelem || e0 + bursts[k] > 0xffffffffull)
            return fail_errno(-EINVAL, "async_process_device: bursts overrun the ring");
        b[4 * k] = (uint32_t)e0;
        b[4 * k + 1] = bursts[k];
        b[4 * k + 2] = (uint32_t)off;
        b[4 * k + 3] = (uint32_t)(off >> 32);
        off += (uint32_t)(len * bursts[k]);
        e0 += bursts[k];
    }
    if (total)
        *total = off;
    if (nbursts == 0)
        return 0;
    SETDEV(q->device);
    if (q->async_cap < nbursts) {
        HIPCHK(hipStreamSynchronize(q->stream));
        (void)hipFree(q->d_async);
        q->d_async = nullptr;
        q->async_cap = 0;
        HIPCHK(hipMalloc(&q->d_async, (size_t)nbursts * 4 * sizeof(uint32_t)));
        q->async_cap = nbursts;
    }
    HIPCHK(hipMemcpyAsync(q->d_async, b.data(), b.size() * sizeof(uint32_t), hipMemcpyHostToDevice, q->stream));
    AsyncArgs aa{};
    aa.ring = d_ring;
    aa.payloadsz = P;
    aa.E = q->E;
    aa.len = len;
    aa.nbursts = nbursts;
    aa.burst = q->d_async;
    aa.histo = q->histo && q->E;
    aa.hist = q->d_hist;
    aa.out = d_out;
    aa.out_cap = out_cap;
    aa.cum = (unsigned long long*)q->d_cum;
    hipLaunchKernelGGL(async_histo_kernel, dim3((nbursts + 3) / 4), dim3(256), 0, q->stream, aa);
    if (d_out)
        hipLaunchKernelGGL(async_raw_kernel, dim3(nbursts), dim3(256), 0, q->stream, aa);
    HIPCHK(hipGetLastError());
    // b is host memory the copy reads: complete before returning
    HIPCHK(hipStreamSynchronize(q->stream));
    return 0;
}

int dqdk_gpu_queue_set_raw_fd(dqdk_gpu_queue_t* q, int fd)
{
    if (!q)
        return -EINVAL;
    if (q->raw_fd >= 0 && fd != q->raw_fd) {  // what went to the old fd is written there first
        SETDEV(q->device);
        if (int rc = raw_drain(q))
            return rc;
    }
    q->raw_fd = fd;
    return 0;
}

int dqdk_gpu_queue_set_raw_deferred(dqdk_gpu_queue_t* q, int on)
{
    if (!q)
        return -EINVAL;
    if (q->raw_deferred && !on && q->raw_fd >= 0) {  // what is pending is written first
        SETDEV(q->device);
        if (int rc = raw_drain(q))
            return rc;
    }
    q->raw_deferred = on != 0;
    return 0;
}

int dqdk_gpu_histogram_batches_per_pass(dqdk_gpu_queue_t* q) { return q ? (int)q->hist_k : -EINVAL; }

int dqdk_gpu_histogram_flush(dqdk_gpu_queue_t* q)
{
    if (!q)
        return -EINVAL;
    if (!q->d_hist)
        return 0;
    SETDEV(q->device);
    return hist_flush(q);
}

int dqdk_gpu_histogram_copy(dqdk_gpu_queue_t* q, uint32_t* d_dst)
{
    if (!q || !d_dst)
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_copy: queue has no histogram");
    SETDEV(q->device);
    if (int rc = hist_flush(q))
        return rc;
    return combine(q, d_dst, 0, DQDK_TRISTAN_HISTO_ENTRIES);
}

int dqdk_gpu_histogram_add(dqdk_gpu_queue_t* q, const uint32_t* d_src)
{
    if (!q || !d_src || ((uintptr_t)d_src & 15))
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_add: queue has no histogram");
    SETDEV(q->device);
    const uint64_t n16 = DQDK_TRISTAN_HISTO_ENTRIES / 4;
    hipLaunchKernelGGL(hist_add_kernel, dim3((uint32_t)q->cu_count * 8u), dim3(256), 0, q->stream, q->d_hist, d_src, n16);
    HIPCHK(hipGetLastError());
    return 0;
}

int dqdk_gpu_histogram_nonzero(dqdk_gpu_queue_t* q, uint64_t* count)
{
    if (!q || !count)
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_nonzero: queue has no histogram");
    SETDEV(q->device);
    if (int rc = hist_flush(q))
        return rc;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(*d)));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(*d), q->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(hist_nonzero_kernel, dim3((uint32_t)q->cu_count * 8u), dim3(256), 0, q->stream, q->d_hist,
                           q->d_lo, DQDK_TRISTAN_HISTO_ENTRIES / 16, d);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess)
        e = hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, q->stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(q->stream);
    (void)hipFree(d);
    if (e != hipSuccess)
        return fail("histogram_nonzero", e);
    *count = h;
    return 0;
}

namespace {

int write_all(int fd, const char* p, uint64_t n)
{
    while (n) {
        const ssize_t w = write(fd, p, n > (1u << 30) ? (1u << 30) : (size_t)n);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            const int err = errno;
            g_err = std::string("histogram_write_csv: write: ") + strerror(err);
            return -err;
        }
        p += w;
        n -= (uint64_t)w;
    }
    return 0;
}

}  // namespace

int dqdk_gpu_histogram_write_csv(dqdk_gpu_queue_t* q, int fd, uint64_t* bytes_written)
{
    if (!q || fd < 0)
        return -EINVAL;
    if (!q->d_hist)
        return fail_errno(-ENOENT, "histogram_write_csv: queue has no histogram");
    SETDEV(q->device);
    if (int rc = hist_flush(q))
        return rc;
    static const char header[] = "Channel,Histo,Energy,Freq\n";  // src/tristan.c:198
    int rc = write_all(fd, header, sizeof(header) - 1);
    if (rc)
        return rc;
    uint64_t total = sizeof(header) - 1;

    // Two text buffers: the GPU formats chunk c+1 while the host writes chunk c.
    const uint64_t cap = kCsvChunkBins * kCsvMaxLine;
    uint64_t* d_blk[2] = {nullptr, nullptr};
    char* d_txt[2] = {nullptr, nullptr};
    char* h_txt[2] = {nullptr, nullptr};
    uint64_t* h_len = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int b = 0; b < 2 && e == hipSuccess; b++) {
        e = hipMalloc(&d_blk[b], (kCsvChunkBlocks + 1) * sizeof(uint64_t));
        if (e == hipSuccess)
            e = hipMalloc(&d_txt[b], cap);
        if (e == hipSuccess)
            e = hipHostMalloc(&h_txt[b], cap, hipHostMallocDefault);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&done[b], hipEventDisableTiming);
    }
    if (e == hipSuccess)
        e = hipHostMalloc(&h_len, 2 * sizeof(uint64_t), hipHostMallocDefault);

    const uint64_t N = DQDK_TRISTAN_HISTO_ENTRIES;
    const uint64_t nchunks = (N + kCsvChunkBins - 1) / kCsvChunkBins;
    // Enqueue chunk c into buffer b: format on the GPU, copy the text back.
    // The text length is needed before the copy, so each chunk's length is
    // read back with a small copy and the text copy is sized on the host.
    auto format = [&](uint64_t c, int b) -> hipError_t {
        const uint64_t base = c * kCsvChunkBins, end = std::min(N, base + kCsvChunkBins);
        const uint32_t nblk = (uint32_t)((end - base + kCsvBinsPerBlock - 1) / kCsvBinsPerBlock);
        hipLaunchKernelGGL(csv_len_kernel, dim3(nblk), dim3(kCsvThreads), 0, q->stream, q->d_hist, q->d_lo, base, end,
                           d_blk[b]);
        hipLaunchKernelGGL(csv_scan_kernel, dim3(1), dim3(1024), 0, q->stream, d_blk[b], nblk);
        hipLaunchKernelGGL(csv_write_kernel, dim3(nblk), dim3(kCsvThreads), 0, q->stream, q->d_hist, q->d_lo, base, end, d_blk[b],
                           d_txt[b]);
        hipError_t r = hipGetLastError();
        if (r == hipSuccess)
            r = hipMemcpyAsync(&h_len[b], d_blk[b] + nblk, sizeof(uint64_t), hipMemcpyDeviceToHost, q->stream);
        if (r == hipSuccess)
            r = hipStreamSynchronize(q->stream);
        if (r == hipSuccess && h_len[b])
            r = hipMemcpyAsync(h_txt[b], d_txt[b], h_len[b], hipMemcpyDeviceToHost, q->stream);
        if (r == hipSuccess)
            r = hipEventRecord(done[b], q->stream);
        return r;
    };
    if (e == hipSuccess && nchunks)
        e = format(0, 0);
    for (uint64_t c = 0; e == hipSuccess && rc == 0 && c < nchunks; c++) {
        const int b = (int)(c & 1);
        e = hipEventSynchronize(done[b]);
        const uint64_t len = h_len[b];
        if (e == hipSuccess && c + 1 < nchunks)
            e = format(c + 1, b ^ 1);  // formats while this thread writes chunk c
        if (e == hipSuccess && len) {
            rc = write_all(fd, h_txt[b], len);
            total += len;
        }
    }
    (void)hipStreamSynchronize(q->stream);
    for (int b = 0; b < 2; b++) {
        (void)hipFree(d_blk[b]);
        (void)hipFree(d_txt[b]);
        (void)hipHostFree(h_txt[b]);
        if (done[b])
            (void)hipEventDestroy(done[b]);
    }
    (void)hipHostFree(h_len);
    if (e != hipSuccess)
        return fail("histogram_write_csv", e);
    if (rc)
        return rc;
    if (bytes_written)
        *bytes_written = total;
    return 0;
}

int dqdk_gpu_tristan_summary(const dqdk_gpu_counters_t* const* per_queue, int nqueues, const uint64_t* runtime_ns,
                             const char* directory, char* buf, uint64_t bufsz)
{
    if (!per_queue || nqueues < 0 || !buf || !bufsz)
        return -EINVAL;
    unsigned long long ev = 0, by = 0, pk = 0;
    uint64_t rt = 0;
    for (int k = 0; k < nqueues; k++) {
        if (!per_queue[k])
            return -EINVAL;
        ev += per_queue[k]->total_events;  // tristan_t atomics (src/tristan.c:172-175)
        by += per_queue[k]->total_bytes;
        pk += per_queue[k]->rcvd_pkts;     // sum of worker rcvd_pkts (:177-183)
        if (runtime_ns && runtime_ns[k] > rt)
            rt = runtime_ns[k];            // max worker runtime
    }
    const int n = snprintf(buf, bufsz,
                           "{ \"total_received_events\": %llu,\"total_received_bytes\": %llu, "
                           "\"total_received_packets\": %llu, \"dqdk_runtime_ms\": %.2lf, \"directory\": \"%s\"}",
                           ev, by, pk, (double)rt / 1e6, directory ? directory : "(null)");
    if (n < 0)
        return -EINVAL;
    return n;  // like snprintf: characters the full string needs
}

const char* dqdk_gpu_timing_stage_name(int stage) { return stage >= 0 && stage < kStages ? kStageNames[stage] : nullptr; }

}  // extern "C"
