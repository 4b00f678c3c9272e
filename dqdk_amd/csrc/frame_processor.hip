/*
 * frame_processor.hip -- DQDK's frame-processor plugin API on the GPU engine
 * (include/dqdk_gpu.h, "frame-processor plugin").
 *
 * The reference hands every valid frame's UDP payload to the registered
 * dqdk_frame_processor_t (src/dqdk.h:84-85) from process_frame
 * (src/dqdk.c:231-250), on the worker's pthread; TRISTAN's is
 * process_unbuffered_frame (src/tristan.c:377-381) -> tristan_process(data,
 * datalen, 1) (:308-330), which bins the E = payloadsz/16 events at the
 * payload (process_events_unrolled16 :247-304 -> histogram_event :233-245),
 * adds datalen to total_bytes and E to total_events, and returns 0.
 *
 * Here every call is a copy: the E * 16 bytes tristan_process would read go
 * into the worker's current pinned staging slot (the copy post_async makes
 * into its ring, src/dqdk.c:220-229) and the call returns 0.  A full slot is
 * copied H2D on the worker's queue stream and decoded there (fp_decode ->
 * rx_count -> the records-path histogram, dqdk_gpu.hip launch_payloads),
 * asynchronously; the slot is written again only after its copy has landed
 * (an event per slot), which is the only time the worker thread can wait.
 *
 * Per-worker state is keyed by the dqdk_worker pointer (a thread-local cache
 * in front of a locked registry): worker->private is the tristan_t all
 * queues share, and dqdk_worker_t's layout (libxdp ring structs) is not
 * needed.  Each worker owns one GPU queue (its own table; no cross-worker
 * locking on the path); dqdk_gpu_fp_fini merges the tables once, like the
 * per-GPU partials of the batch entry points.
 */
#include <errno.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "queue_internal.h"

namespace {

constexpr uint32_t kFpMaxSlots = 64;

struct FpWorker {
    const void* key = nullptr;  // the dqdk_worker pointer
    int device = 0;
    const uint8_t* umem_lo = nullptr;  // optional UMEM bound (dqdk_gpu_fp_bind)
    const uint8_t* umem_hi = nullptr;
    dqdk_gpu_queue_t* q = nullptr;
    hipStream_t stream = nullptr;
    uint32_t S = 0;            // staged bytes per call: E * 16 (0: the mode keeps no histogram)
    uint32_t P = 0;            // calls per slot
    uint32_t nslots = 0;
    uint8_t* h_stage = nullptr;  // pinned [nslots][P][S]
    uint32_t* h_len = nullptr;   // pinned [nslots][P]
    uint8_t* d_stage = nullptr;  // [P][S]
    uint32_t* d_len = nullptr;   // [P]
    hipEvent_t ev[kFpMaxSlots] = {};  // slot k's H2D copy has landed
    uint32_t cur = 0, fill = 0;
    int err = 0;  // sticky: the first failure, returned by every later call
};

std::mutex g_mu;
bool g_init = false;
dqdk_gpu_fp_cfg_t g_cfg{};
std::vector<std::unique_ptr<FpWorker>> g_workers;
uint32_t g_rr = 0;                    // round-robin device cursor
std::atomic<uint64_t> g_gen{1};       // bumped by fini: invalidates thread caches
// test hook (DQDK_GPU_FP_PEER_MERGE=1 at fp_init): fini's CSV merge takes the
// cross-device branch (table copied on the worker's GPU, hipMemcpyPeer, add)
// for every worker, a worker on w0's own GPU included (a peer copy within one
// device is legal), so a one-GPU box exercises that branch's allocation,
// copy and free ordering
bool g_peer_merge = false;

struct Cache {
    const void* key = nullptr;
    FpWorker* s = nullptr;
    uint64_t gen = 0;
};
thread_local Cache t_cache;

struct DevScope {  // make `dev` current, restore the caller's on exit
    int prev = -1;
    hipError_t e;
    explicit DevScope(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        e = prev == dev ? hipSuccess : hipSetDevice(dev);
    }
    ~DevScope()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
            (void)hipSetDevice(prev);
    }
};

// Returns the queue's sync / destroy result (a fault of the worker's last
// work fails fp_fini, not a later call).
int fp_close(FpWorker* s)
{
    int rc = 0;
    if (s->q) {
        DevScope g(s->device);
        rc = dqdk_gpu_queue_sync(s->q);
        for (uint32_t k = 0; k < kFpMaxSlots; k++)
            if (s->ev[k])
                (void)hipEventDestroy(s->ev[k]);
        (void)hipFree(s->d_stage);
        (void)hipFree(s->d_len);
        if (s->h_stage)
            (void)hipHostFree(s->h_stage);
        if (s->h_len)
            (void)hipHostFree(s->h_len);
        const int drc = dqdk_gpu_queue_destroy(s->q);
        if (!rc)
            rc = drc;
    }
    *s = FpWorker{};
    return rc;
}

// Queue, pinned slots and device buffers of a new worker (under g_mu).
int fp_open(FpWorker* s)
{
    dqdk_gpu_cfg_t c = g_cfg.cfg;
    // the header checks (and the batch accounting) stay in the caller's
    // get_udp_payload / fetch_xsk: only the histogram strategy applies here
    c.flags &= DQDK_GPU_F_NO_HISTO | DQDK_GPU_F_HISTO_ATOMIC | DQDK_GPU_F_HISTO_PARTITIONED |
               DQDK_GPU_F_HISTO_EAGER;
    s->P = g_cfg.slot_payloads;
    s->nslots = g_cfg.nslots;
    int rc = dqdk_gpu_queue_create(s->device, &c, s->P, &s->q);
    if (rc)
        return rc;
    DevScope g(s->device);
    if (g.e != hipSuccess)
        return dqdk::set_hip_error("hipSetDevice", g.e);
    s->stream = (hipStream_t)dqdk_gpu_queue_stream(s->q);
    s->S = dqdk::queue_events(s->q) * 16u;
    const size_t slot_bytes = (size_t)s->P * s->S;
    hipError_t e = hipSuccess;
    if (slot_bytes) {
        if ((e = hipHostMalloc(&s->h_stage, slot_bytes * s->nslots, hipHostMallocDefault)) != hipSuccess ||
            (e = hipMalloc(&s->d_stage, slot_bytes)) != hipSuccess)
            return (dqdk::set_hip_error("frame processor staging", e), -ENOMEM);
    }
    if ((e = hipHostMalloc(&s->h_len, (size_t)s->P * s->nslots * sizeof(uint32_t), hipHostMallocDefault)) != hipSuccess ||
        (e = hipMalloc(&s->d_len, (size_t)s->P * sizeof(uint32_t))) != hipSuccess)
        return (dqdk::set_hip_error("frame processor staging", e), -ENOMEM);
    for (uint32_t k = 0; k < s->nslots; k++)
        if ((e = hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming)) != hipSuccess)
            return dqdk::set_hip_error("hipEventCreate", e);
    return 0;
}

int next_device()
{
    const int nd = g_cfg.ndevices;
    return g_cfg.device_first + (int)(g_rr++ % (uint32_t)nd);
}

// The worker's state, created on first sight (under g_mu); null + *rc on failure.
FpWorker* find_or_open(const void* key, int device, int* rc)
{
    *rc = 0;
    for (auto& w : g_workers)
        if (w->key == key)
            return w.get();
    auto w = std::make_unique<FpWorker>();
    w->key = key;
    w->device = device >= 0 ? device : next_device();
    if ((*rc = fp_open(w.get())) != 0) {
        (void)fp_close(w.get());
        return nullptr;
    }
    g_workers.push_back(std::move(w));
    return g_workers.back().get();
}

FpWorker* lookup(const void* key, int* rc)
{
    const uint64_t gen = g_gen.load(std::memory_order_acquire);
    if (t_cache.key == key && t_cache.gen == gen && t_cache.s)
        return t_cache.s;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_init) {
        *rc = dqdk::set_error(-EINVAL, "frame processor: dqdk_gpu_fp_init was not called");
        return nullptr;
    }
    FpWorker* s = find_or_open(key, -1, rc);
    if (s)
        t_cache = Cache{key, s, gen};
    return s;
}

// Hand the current slot to the GPU (its H2D copy, then the batch), move to
// the next slot and wait until that one's previous copy has landed.
int submit(FpWorker* s)
{
    if (s->err)
        return s->err;
    const uint32_t n = s->fill;
    if (!n)
        return 0;
    DevScope g(s->device);
    hipError_t e = g.e;
    const uint32_t k = s->cur;
    if (e == hipSuccess && s->S)
        e = hipMemcpyAsync(s->d_stage, s->h_stage + (size_t)k * s->P * s->S, (size_t)n * s->S,
                           hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(s->d_len, s->h_len + (size_t)k * s->P, (size_t)n * sizeof(uint32_t),
                           hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess)
        e = hipEventRecord(s->ev[k], s->stream);
    if (e != hipSuccess)
        return s->err = dqdk::set_hip_error("frame processor: staging copy", e);
    int rc = dqdk::queue_launch_payloads(s->q, s->d_stage, s->d_len, n);
    if (rc)
        return s->err = rc;
    s->cur = (k + 1) % s->nslots;
    s->fill = 0;
    // (an event never recorded completes at once)
    if ((e = hipEventSynchronize(s->ev[s->cur])) != hipSuccess)
        return s->err = dqdk::set_hip_error("frame processor: slot wait", e);
    return 0;
}

}  // namespace

extern "C" {

int dqdk_gpu_fp_init(const dqdk_gpu_fp_cfg_t* cfg)
{
    if (!cfg)
        return dqdk::set_error(-EINVAL, "fp_init: null cfg");
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_init)
        return dqdk::set_error(-EBUSY, "fp_init: already set up (dqdk_gpu_fp_fini first)");
    dqdk_gpu_fp_cfg_t c = *cfg;
    if (c.cfg.mode > DQDK_MODE_ENERGYHISTO)
        return dqdk::set_error(-EINVAL, "fp_init: bad mode");
    if (!c.slot_payloads)
        c.slot_payloads = 8192;
    if (!c.nslots)
        c.nslots = 4;
    if (c.nslots < 2 || c.nslots > kFpMaxSlots)
        return dqdk::set_error(-EINVAL, "fp_init: nslots must be in [2, 64]");
    const int ndev = dqdk_gpu_device_count();
    if (c.ndevices == 0)
        c.ndevices = ndev - c.device_first;
    if (ndev <= 0 || c.device_first < 0 || c.ndevices <= 0 || c.device_first + c.ndevices > ndev)
        return dqdk::set_error(-ENODEV, "fp_init: no such HIP device range");
    g_cfg = c;
    g_rr = 0;
    const char* pm = getenv("DQDK_GPU_FP_PEER_MERGE");
    g_peer_merge = pm && !strcmp(pm, "1");
    g_init = true;
    return 0;
}

int dqdk_gpu_fp_bind(struct dqdk_worker* worker, int device, const void* umem, uint64_t umem_size)
{
    if (!worker || (!umem && umem_size))
        return dqdk::set_error(-EINVAL, "fp_bind: bad argument");
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_init)
        return dqdk::set_error(-EINVAL, "fp_bind: dqdk_gpu_fp_init was not called");
    if (device >= g_cfg.device_first + g_cfg.ndevices || (device >= 0 && device < g_cfg.device_first))
        return dqdk::set_error(-ENODEV, "fp_bind: device outside the configured range");
    int rc = 0;
    FpWorker* s = find_or_open(worker, device, &rc);
    if (!s)
        return rc;
    if (device >= 0 && s->device != device)
        return dqdk::set_error(-EBUSY, "fp_bind: the worker is already bound to another device");
    s->umem_lo = (const uint8_t*)umem;
    s->umem_hi = umem ? (const uint8_t*)umem + umem_size : nullptr;
    return 0;
}

int dqdk_gpu_frame_processor(struct dqdk_worker* worker, uint8_t* data, uint32_t datalen)
{
    int rc = 0;
    FpWorker* s = lookup(worker, &rc);
    if (!s)
        return rc;
    if (s->err)
        return s->err;
    const uint32_t i = s->fill;
    const uint32_t S = s->S;
    if (S) {
        // the bytes process_events_unrolled16 reads: E * 16 from the payload
        // start whatever datalen says (src/tristan.c:311-315)
        uint8_t* dst = s->h_stage + ((size_t)s->cur * s->P + i) * S;
        const uint8_t* src = data;
        if (s->umem_hi && src >= s->umem_lo && src < s->umem_hi && (uint64_t)(s->umem_hi - src) < S) {
            const size_t room = (size_t)(s->umem_hi - src);
            memcpy(dst, src, room);
            memset(dst + room, 0, S - room);
        } else {
            memcpy(dst, src, S);
        }
    }
    s->h_len[(size_t)s->cur * s->P + i] = datalen;
    if (++s->fill == s->P)
        return submit(s);
    return 0;  // tristan_process's result without a raw file (src/tristan.c:329)
}

int dqdk_gpu_fp_flush(struct dqdk_worker* worker)
{
    if (!worker)
        return -EINVAL;
    FpWorker* s = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto& w : g_workers)
            if (w->key == worker)
                s = w.get();
    }
    return s ? submit(s) : 0;
}

int dqdk_gpu_fp_fini(uint32_t* host_hist, int csv_fd, dqdk_gpu_counters_t* totals)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_init)
        return dqdk::set_error(-EINVAL, "fp_fini: dqdk_gpu_fp_init was not called");
    int rc = 0;
    for (auto& w : g_workers) {
        const int r = submit(w.get());
        rc = rc ? rc : r;
    }
    dqdk_gpu_counters_t sum;
    memset(&sum, 0, sizeof(sum));
    for (auto& w : g_workers) {
        if (rc)
            break;
        dqdk_gpu_counters_t c;
        if ((rc = dqdk_gpu_counters_get(w->q, &c)) != 0)
            break;
        sum.rcvd_frames += c.rcvd_frames;
        sum.rcvd_pkts += c.rcvd_pkts;
        sum.rcvd_bytes += c.rcvd_bytes;
        sum.invalid_ip_pkts += c.invalid_ip_pkts;
        sum.invalid_udp_pkts += c.invalid_udp_pkts;
        sum.failing_batches += c.failing_batches;
        sum.total_events += c.total_events;
        sum.total_bytes += c.total_bytes;
        sum.oob_events += c.oob_events;
        sum.empty_pkts += c.empty_pkts;
        sum.filtered_frames += c.filtered_frames;
    }
    if (!rc && totals)
        *totals = sum;
    const bool histo = !g_workers.empty() && dqdk::queue_events(g_workers[0]->q) != 0;
    // tristan_t::histo += every worker's table (before the CSV merge below
    // adds the other tables into the first worker's)
    for (auto& w : g_workers) {
        if (rc || !host_hist || !histo)
            break;
        rc = dqdk_gpu_histogram_accumulate(w->q, host_hist);
    }
    if (!rc && csv_fd >= 0) {
        if (!histo) {
            static const char header[] = "Channel,Histo,Energy,Freq\n";  // src/tristan.c:198
            if (write(csv_fd, header, sizeof(header) - 1) != (ssize_t)(sizeof(header) - 1))
                rc = dqdk::set_error(-EIO, "fp_fini: CSV header write");
        } else {
            FpWorker* w0 = g_workers[0].get();
            const size_t bytes = (size_t)DQDK_TRISTAN_HISTO_ENTRIES * sizeof(uint32_t);
            uint32_t* tmp = nullptr;
            for (size_t k = 1; !rc && k < g_workers.size(); k++) {
                FpWorker* w = g_workers[k].get();
                if (!tmp) {
                    DevScope g(w0->device);
                    if (hipMalloc(&tmp, bytes) != hipSuccess) {
                        tmp = nullptr;
                        rc = dqdk::set_error(-ENOMEM, "fp_fini: merge buffer");
                        break;
                    }
                }
                if (w->device == w0->device && !g_peer_merge) {
                    if (!(rc = dqdk_gpu_histogram_copy(w->q, tmp)))
                        rc = dqdk_gpu_queue_sync(w->q);
                } else {  // another GPU: its table copied there, then peer-copied over
                    uint32_t* tk = nullptr;
                    DevScope g(w->device);
                    if (hipMalloc(&tk, bytes) != hipSuccess) {
                        rc = dqdk::set_error(-ENOMEM, "fp_fini: merge buffer");
                        break;
                    }
                    if (!(rc = dqdk_gpu_histogram_copy(w->q, tk)) && !(rc = dqdk_gpu_queue_sync(w->q))) {
                        hipError_t e = hipMemcpyPeer(tmp, w0->device, tk, w->device, bytes);
                        if (e != hipSuccess)
                            rc = dqdk::set_hip_error("fp_fini: hipMemcpyPeer", e);
                    }
                    (void)hipFree(tk);
                }
                if (!rc && !(rc = dqdk_gpu_histogram_add(w0->q, tmp)))
                    rc = dqdk_gpu_queue_sync(w0->q);
            }
            if (tmp) {
                DevScope g(w0->device);
                (void)hipFree(tmp);
            }
            if (!rc)
                rc = dqdk_gpu_histogram_write_csv(w0->q, csv_fd, nullptr);
        }
    }
    for (auto& w : g_workers) {
        const int crc = fp_close(w.get());
        if (!rc)
            rc = crc;
    }
    g_workers.clear();
    g_init = false;
    g_gen.fetch_add(1, std::memory_order_acq_rel);
    return rc;
}

}  // extern "C"
