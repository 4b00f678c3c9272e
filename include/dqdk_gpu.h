/*
 * dqdk_gpu.h -- C ABI of the MI355X receive-path engine (libdqdk_gpu.so).
 *
 * Drop-in boundary for DQDK's per-frame receive hot path.  The reference
 * runs, per RX descriptor, on one worker pthread per queue:
 *
 *   fetch_xsk            src/dqdk.c:252-322   (per-descriptor loop :291-298)
 *     process_frame      src/dqdk.c:231-250
 *       get_udp_payload  src/dqdk.c:185-207   -> ip4_audit  src/tcpip/ipv4.c:13-20
 *                                             -> udp_audit  src/tcpip/udp.c:22-31
 *       frame_processor  src/dqdk.h:84-85  == process_unbuffered_frame src/tristan.c:377-381
 *         tristan_process            src/tristan.c:308-330
 *           process_events_unrolled16 src/tristan.c:247-304
 *             histogram_event         src/tristan.c:233-245
 *
 * dqdk_gpu_rx_batch() replaces the loop at src/dqdk.c:291-298 for a whole
 * peeked batch (the ring ops around it are unchanged) and runs
 * get_udp_payload + the TRISTAN sync frame processor on the GPU.  The
 * optional checksum configuration (ip4_audit_checksum src/tcpip/ipv4.c:6-11,
 * udp_audit_checksum src/tcpip/udp.c:10-20, both commented out of the audit
 * in the shipped code at ipv4.c:16 / udp.c:26) and the XDP forwarder's
 * predicate (src/bpf/forwarder.bpf.c:38-96) are selectable per queue.
 *
 * Plain C types only; every pointer is either a host pointer or a device
 * pointer as each function states.  Errors are negative errno values like
 * the reference (-EINVAL, -ENOMEM, -ENODEV; HIP failures map to -EIO).
 * There is no CPU implementation behind any of these entry points: without
 * a usable gfx950 device, dqdk_gpu_queue_create() returns -ENODEV.
 */
#ifndef DQDK_GPU_H
#define DQDK_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQDK_GPU_ABI_VERSION 1

/* struct xdp_desc from linux/if_xdp.h: frame = umem + addr (src/dqdk.c:293) */
typedef struct dqdk_gpu_desc {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
} dqdk_gpu_desc_t;

/* Per-frame verdict.  OK is the only status for which the reference calls
 * the frame processor; every other in-batch status makes process_frame
 * return -ENOBUFS (src/dqdk.c:243-249). */
enum dqdk_gpu_status {
    DQDK_RX_OK = 0,
    DQDK_RX_INVALID_IP = 1,       /* ip4_audit: ntohs(tot_len) != (u16)(len-14)   */
    DQDK_RX_INVALID_UDP = 2,      /* udp_audit: ntohs(udp->len) != (u16)udplen    */
    DQDK_RX_EMPTY = 3,            /* valid headers but datalen == 0               */
    DQDK_RX_INVALID_IP_CSUM = 4,  /* checksum config: ip4_audit_checksum failed   */
    DQDK_RX_INVALID_UDP_CSUM = 5, /* checksum config: udp_audit_checksum failed   */
    DQDK_RX_FILTER_DROP = 6,      /* prefilter: forwarder would XDP_DROP          */
    DQDK_RX_FILTER_PASS = 7,      /* prefilter: forwarder would XDP_PASS          */
};

/* 8-B per-frame record (the `datalen` out-param + payload pointer of
 * get_udp_payload, plus the verdict). */
typedef struct dqdk_gpu_rx_result {
    uint32_t datalen;     /* udplen - 8 in u32, may wrap (src/dqdk.c:205) */
    uint8_t status;       /* enum dqdk_gpu_status                          */
    uint8_t payload_off;  /* payload = umem + addr + payload_off (OK/EMPTY) */
    uint16_t oob_events;  /* events histogram_event rejected (saturating)  */
} dqdk_gpu_rx_result_t;

/* Counters: the dqdk_stats_t fields this path touches (src/dqdk.h:52-68)
 * plus the tristan_t atomics (src/tristan.h:81-82) and a few diagnostics. */
typedef struct dqdk_gpu_counters {
    uint64_t rcvd_frames;      /* dqdk.c:289                               */
    uint64_t rcvd_pkts;        /* dqdk.c:189                               */
    uint64_t rcvd_bytes;       /* dqdk.c:246                               */
    uint64_t invalid_ip_pkts;  /* dqdk.c:192                               */
    uint64_t invalid_udp_pkts; /* dqdk.c:201                               */
    uint64_t failing_batches;  /* dqdk.c:319                               */
    uint64_t total_events;     /* tristan.c:328                            */
    uint64_t total_bytes;      /* tristan.c:327                            */
    uint64_t oob_events;       /* tristan.c:236-240 (logged there)         */
    uint64_t empty_pkts;       /* datalen == 0 frames                      */
    uint64_t filtered_frames;  /* prefilter non-REDIRECT frames            */
    uint64_t first_abort_idx;  /* last batch: first failing index, or n    */
} dqdk_gpu_counters_t;

/* tristan_mode_t (src/tristan.h:62-67) */
enum dqdk_gpu_mode {
    DQDK_MODE_WAVEFORM = 0,
    DQDK_MODE_LISTWAVE = 1,
    DQDK_MODE_LISTMODE = 2,
    DQDK_MODE_ENERGYHISTO = 3,
};

enum dqdk_gpu_flags {
    DQDK_GPU_F_CSUM = 1u << 0,           /* verify IPv4 + UDP checksums                 */
    DQDK_GPU_F_BATCH_ABORT = 1u << 1,    /* account like fetch_xsk: stop at 1st failure */
    DQDK_GPU_F_PREFILTER = 1u << 2,      /* apply the XDP forwarder predicate first     */
    DQDK_GPU_F_NO_HISTO = 1u << 3,       /* decode only, no histogram accumulation      */
    DQDK_GPU_F_CSUM_WRITEBACK = 1u << 4, /* zero udp->check in UMEM like udp.c:17       */
    /* Histogram accumulation strategy (same table either way; default picks
     * per batch by event count): */
    DQDK_GPU_F_HISTO_ATOMIC = 1u << 5,      /* one device atomic per event              */
    DQDK_GPU_F_HISTO_PARTITIONED = 1u << 6, /* bucket -> slice -> LDS histogram + RMW   */
    DQDK_GPU_F_HISTO_EAGER = 1u << 7,       /* partitioned: slice pass after every batch */
    DQDK_GPU_F_HISTO_UNFUSED = 1u << 8,     /* partitioned: decode to frame-order records, then
                                               bucket them (default: the decode buckets its keys
                                               itself when no record buffer is passed and the
                                               accounting is per-packet) */
};

typedef struct dqdk_gpu_cfg {
    uint32_t payloadsz;  /* -s (src/tristan.c:419): events per frame = payloadsz/16 */
    uint32_t mode;       /* enum dqdk_gpu_mode                                        */
    uint32_t flags;      /* enum dqdk_gpu_flags                                       */
    uint16_t port_start; /* prefilter source-port range (dqdk_for_ports_range)        */
    uint16_t port_end;
} dqdk_gpu_cfg_t;

/* Histogram geometry (src/tristan.h:55-60): u32[1512][6][65536]. */
#define DQDK_TRISTAN_CHANNELS 1512u
#define DQDK_TRISTAN_HISTS 6u
#define DQDK_TRISTAN_BINS 65536u
#define DQDK_TRISTAN_HISTO_ENTRIES ((uint64_t)DQDK_TRISTAN_CHANNELS * DQDK_TRISTAN_HISTS * DQDK_TRISTAN_BINS)
#define DQDK_KEY_NONE 0xFFFFFFFFu /* decoded record of an out-of-bounds event */

typedef struct dqdk_gpu_queue dqdk_gpu_queue_t;

/* ---- lifecycle ----------------------------------------------------------- */
int dqdk_gpu_abi_version(void);
int dqdk_gpu_device_count(void);
/* One queue per RX queue / worker thread (src/dqdk.c:517-620).  Allocates
 * the queue's device histogram (2.38 GB, zeroed) unless the mode has none.
 *
 * HBM per queue with a histogram (max_batch = 1M frames, E = payloadsz/16):
 *                                         1M x 1500 B (E 91)   1M x 9000 B (E 559)
 *   table: u32 base + u8 low plane          2.97 GB              2.97 GB
 *   fused pieces (key triples, 1.25x)       0.34 GB              1.97 GB
 *   overflow regions + list (2 x 256 x      0.13 GB              0.59 GB
 *     max(64K, 1/8 of a block's keys))
 *   slice staging, per staged batch         0.22 GB              1.20 GB
 *     x batches per pass                    x 32 = 7.0 GB        x 21 = 25.2 GB
 *   descriptors, results, scratch           0.03 GB              0.03 GB
 *   total                                   ~10.5 GB             ~30.8 GB
 * The staging takes at most 24 GiB or a quarter of the device memory free at
 * creation, and halves while its allocation fails (down to one batch per
 * pass).  The records path (frame-order keys: BATCH_ABORT, HISTO_UNFUSED, or
 * batches too small to partition) adds n * E * 8 B (keys + their grouped copy)
 * on its first batch -- allocated at creation when the flags force it. */
int dqdk_gpu_queue_create(int device, const dqdk_gpu_cfg_t* cfg, uint32_t max_batch, dqdk_gpu_queue_t** out);
/* destroy waits for the queue's work, releases everything it holds whatever
 * fails, and returns 0 or the first failure (-EIO, dqdk_gpu_last_error names
 * the call): a device fault left by the queue's last kernels or copies is
 * reported by the destroy, not by the caller's next HIP call. */
int dqdk_gpu_queue_destroy(dqdk_gpu_queue_t* q);
/* Queues start on a stream of their own (hipStreamNonBlocking).  Run the
 * queue's work on the caller's hipStream_t instead -- verbatim, so NULL is
 * the legacy default stream -- to order it after the caller's producers.
 * Work already enqueued on the current stream is ordered before the new
 * one's (an event is recorded on it), so the current stream must still be
 * alive at the switch: switch away before destroying a caller stream.
 * No entry point changes the calling thread's current HIP device. */
int dqdk_gpu_queue_set_stream(dqdk_gpu_queue_t* q, void* hip_stream);
void* dqdk_gpu_queue_stream(dqdk_gpu_queue_t* q);     /* current stream     */
void* dqdk_gpu_queue_own_stream(dqdk_gpu_queue_t* q); /* the queue's own one */

/* Device memory for a UMEM image or frame staging slots in HBM (the
 * device-resident and PCIe-inclusive forms).  Physically contiguous when the
 * driver allows (hipDeviceMallocContiguous; else plain device memory).  The
 * 9000 B decode runs 2.12 or 2.35 ms per 1M frames depending on where the
 * driver placed the image relative to the queue's staging (DESIGN.md
 * section 5: a placement interaction, not a property of the box); images
 * from this call ran in the fast state more often than torch's allocator's.
 * Returns 0 (contiguous), 1 (the driver had no contiguous range: plain
 * device memory) or a negative errno.  Allocate large images early:
 * contiguous ranges fragment.  (The queue's own table and staging are plain
 * device memory unless DQDK_GPU_ALLOC = contig | auto: contiguous staging,
 * auto from 128 events per frame.) */
int dqdk_gpu_device_alloc(int device, uint64_t size, void** d_out);
int dqdk_gpu_device_free(int device, void* d_ptr);

/* ---- device-resident batch (async on the queue stream) ------------------- */
/* d_umem/d_desc/d_results/d_keys are DEVICE pointers.  d_keys (nullable)
 * receives n*E u32 decoded records: key = (channel*6 + hist_class)*65536 +
 * (energy>>8), DQDK_KEY_NONE for out-of-bounds events; records of frames
 * whose status is not OK are unspecified.  Counters accumulate on device. */
int dqdk_gpu_rx_batch_device(dqdk_gpu_queue_t* q, const uint8_t* d_umem, uint64_t umem_size,
                             const dqdk_gpu_desc_t* d_desc, uint32_t n, dqdk_gpu_rx_result_t* d_results,
                             uint32_t* d_keys);
int dqdk_gpu_queue_sync(dqdk_gpu_queue_t* q);

/* ---- host drop-in for the fetch_xsk loop (synchronous) ------------------- */
/* umem: host UMEM (pinned once through dqdk_gpu_umem_register for best
 * rate); d, per_pkt, delta: host pointers.  Copies the batch's frames in,
 * runs the batch, copies per-frame results and this batch's counter delta
 * out.  Returns 0, or the negative errno of the first failure.
 * dqdk_gpu_umem_register is a no-op for an address already registered with
 * at least `size` bytes; with fewer, the old registration is replaced (the
 * queue's stream drained first).  rx_batch registers a UMEM no registration
 * covers.  A registered UMEM must be unregistered (or its queue destroyed)
 * BEFORE its memory is freed or unmapped: a registration outlives nothing it
 * maps, and a new buffer placed at a freed one's address would otherwise be
 * read through the old registration's pages (the reference's UMEM lives
 * for the worker's lifetime: created at src/dqdk.c:562, unmapped by
 * umem_info_free at :476-479 (:74-80) in the worker's cleanup, so this is its
 * order too).
 * Registrations are process-wide and reference-counted: queues (on any GPU)
 * over one host buffer (the reference gives each worker its own UMEM,
 * src/dqdk.c:562, but a caller may share one) or over views inside it
 * share one mapping, and the last queue to unregister or be destroyed
 * releases it.  Replacing a registration another queue still holds fails
 * with -EBUSY. */
int dqdk_gpu_umem_register(dqdk_gpu_queue_t* q, void* umem, uint64_t size);
int dqdk_gpu_umem_unregister(dqdk_gpu_queue_t* q, void* umem);
int dqdk_gpu_rx_batch(dqdk_gpu_queue_t* q, const uint8_t* umem, uint64_t umem_size, const dqdk_gpu_desc_t* d,
                      uint32_t n, dqdk_gpu_rx_result_t* per_pkt, dqdk_gpu_counters_t* delta);

/* ---- frame-processor plugin (dqdk_frame_processor_t, src/dqdk.h:84-85) ---- */
/* The reference's own operator API for this path: process_frame
 * (src/dqdk.c:231-250) calls worker->frame_processor(worker, payload,
 * datalen) once per frame whose get_udp_payload succeeded with datalen != 0,
 * on that worker's pthread; TRISTAN registers process_unbuffered_frame
 * (src/tristan.c:377-381, at :589-590), i.e. tristan_process(payload,
 * datalen, 1) (:308-330): the E = payloadsz/16 events at the payload into
 * the shared histogram, total_bytes += datalen, total_events += E, return 0.
 *
 * dqdk_gpu_frame_processor has exactly that signature and result, so an
 * unmodified dqdk.c drives the GPU: register it as `proc` in dqdk_ctx_init
 * (src/tristan.c:589-590) after dqdk_gpu_fp_init, and call dqdk_gpu_fp_fini
 * before tristan_fini.  Per worker -- keyed by the worker
 * pointer, never by worker->private (the shared tristan_t) -- each call
 * copies the E * 16 bytes tristan_process reads (the copy post_async makes
 * into its ring, src/dqdk.c:220-229) into a pinned staging slot and returns
 * 0; a full slot is copied to the worker's GPU and decoded there
 * asynchronously (the worker reuses the slot once that copy has landed).
 * Returns 0, or -EIO / -ENOMEM / -ENODEV once the worker's GPU queue has
 * failed (process_frame then aborts the batch like any processor error). */
struct dqdk_worker; /* the reference's dqdk_worker_t (src/dqdk.h:87-105), opaque here */

typedef struct dqdk_gpu_fp_cfg {
    dqdk_gpu_cfg_t cfg;     /* payloadsz / mode as -s / -m; flags: histogram strategy only
                               (the header checks stay in the caller's get_udp_payload) */
    uint32_t slot_payloads; /* calls staged per GPU batch (0: 8192)                        */
    uint32_t nslots;        /* pinned staging slots per worker, >= 2 (0: 4)                */
    int device_first;       /* workers are spread round robin over devices                */
    int ndevices;           /*   [device_first, device_first + ndevices) (0: all devices)   */
} dqdk_gpu_fp_cfg_t;

/* Before the workers start (tristan_init's place).  -EBUSY if already set up. */
int dqdk_gpu_fp_init(const dqdk_gpu_fp_cfg_t* cfg);
/* Optional, before the worker's first frame (e.g. after dqdk_ctx_init): give
 * the worker its GPU now (device < 0: round robin) instead of at its first
 * call, and its UMEM (nullable): event bytes a call would read at or past
 * umem + umem_size are then taken as zeros, as the batch entry points do. */
int dqdk_gpu_fp_bind(struct dqdk_worker* worker, int device, const void* umem, uint64_t umem_size);
/* The dqdk_frame_processor_t (src/dqdk.h:85). */
int dqdk_gpu_frame_processor(struct dqdk_worker* worker, uint8_t* data, uint32_t datalen);
/* Optional: hand the worker's partly filled slot to the GPU now (e.g. when
 * its RX ring runs empty).  Call on the worker's thread or after it stopped. */
int dqdk_gpu_fp_flush(struct dqdk_worker* worker);
/* After the workers have stopped (dqdk_waitall), before tristan_fini: every
 * worker's staged calls are decoded, then
 *   host_hist (nullable): every worker's table added (u32 wrap) into it --
 *     tristan_t::histo, so tristan_fini's own CSV loop (:197-216) and JSON
 *     summary run unchanged;
 *   csv_fd >= 0: the merged table written as tristan_fini's CSV, formatted
 *     on the GPU (dqdk_gpu_histogram_write_csv);
 *   totals (nullable): the workers' counters summed -- total_events /
 *     total_bytes are what tristan_process added to tristan_t (:327-328),
 *     rcvd_pkts the calls, oob_events the events histogram_event rejected.
 * Then every worker's queue is released and the plugin can be set up again. */
int dqdk_gpu_fp_fini(uint32_t* host_hist, int csv_fd, dqdk_gpu_counters_t* totals);

/* ---- raw payload stream (tristan_process write(), src/tristan.c:318-324) -- */
/* The concatenation, in descriptor order, of payload[0, datalen) of every
 * frame the batch hands to the frame processor (accounted OK frames; in
 * BATCH_ABORT mode those before the first failure) -- what the reference
 * writes to its raw file when rawdata_fd >= 0 (waveform mode always).
 * Frames whose u32-wrapped datalen runs past the UMEM contribute nothing.
 * Device form: call after dqdk_gpu_rx_batch_device on the same queue stream
 * with the same d_desc/d_results; writes min(total, out_cap) bytes to d_out
 * (NULL with out_cap 0 = size query).  total (host, nullable) = the stream's
 * full length, which makes the call synchronous.  Host form: with a raw fd
 * set, dqdk_gpu_rx_batch appends each batch's stream to it.  By default, as
 * tristan_process does (src/tristan.c:318-324), the stream is gathered,
 * copied and write()n before the call returns, and a failed write() is that
 * call's -errno (returned after the batch's results and delta are
 * delivered).  Opt-in (dqdk_gpu_queue_set_raw_deferred(q, 1)): the GPU
 * gathers the stream before the call returns (the frames are valid only
 * until the descriptors are released, src/dqdk.c:300), its D2H copy runs on
 * a side stream into one of two pinned buffers, and its write() happens
 * during the next dqdk_gpu_rx_batch call while that batch's kernels run -- or
 * at dqdk_gpu_queue_sync, dqdk_gpu_queue_set_raw_fd, set_raw_deferred(q, 0)
 * and dqdk_gpu_queue_destroy, which drain it.  A failed deferred write() is
 * returned by the call that makes it (destroy also reports it on stderr): the
 * caller keeps the fd open until one of those has run. */
int dqdk_gpu_raw_compact_device(dqdk_gpu_queue_t* q, const uint8_t* d_umem, uint64_t umem_size,
                                const dqdk_gpu_desc_t* d_desc, uint32_t n, const dqdk_gpu_rx_result_t* d_results,
                                uint8_t* d_out, uint64_t out_cap, uint64_t* total);
int dqdk_gpu_queue_set_raw_fd(dqdk_gpu_queue_t* q, int fd); /* -1 = off (default); drains first */
int dqdk_gpu_queue_set_raw_deferred(dqdk_gpu_queue_t* q, int on); /* 0 = synchronous write() (default) */

/* ---- async consumer (async_processor, src/tristan.c:332-375) --------------- */
/* The raw/async modes hand each payload to post_async (src/dqdk.c:220-229):
 * a ring of elements of payloadsz bytes; one consumer thread fetches them in
 * bursts of `ret` <= 16 elements (dqdk_async_processor_nfetch) and calls
 * tristan_process(buffer, len, ret) with len = strip_wfm ? 16 : payloadsz
 * (:343).  d_ring (DEVICE) holds nelem such elements back to back (e.g. the
 * batch's raw stream when datalen == payloadsz); bursts[nbursts] (HOST) are
 * the fetch sizes in order.  Reproduces that call exactly, quirks included:
 * the histogram counts the FIRST payload of each burst ret times
 * (:314-315), total_events grows by E once per burst, total_bytes by
 * len * ret (:327-328), oob_events by ret per rejected event, and the raw
 * stream receives the first len * ret bytes of each burst (:319) -- written
 * to d_out (DEVICE, nullable; min(total, out_cap) bytes).  *total (nullable)
 * = the raw stream's full length.  payloadsz must be a multiple of 4 (the
 * reference ring's element rule, src/ds/cne_ring.c:41).  Synchronous. */
int dqdk_gpu_async_process_device(dqdk_gpu_queue_t* q, const uint8_t* d_ring, uint64_t nelem, const uint32_t* bursts,
                                  uint32_t nbursts, int strip_wfm, uint8_t* d_out, uint64_t out_cap, uint64_t* total);

/* ---- counters / histogram egress ----------------------------------------- */
int dqdk_gpu_counters_get(dqdk_gpu_queue_t* q, dqdk_gpu_counters_t* out); /* cumulative */
int dqdk_gpu_counters_reset(dqdk_gpu_queue_t* q);
/* Copy the queue's u32[DQDK_TRISTAN_HISTO_ENTRIES] histogram to host memory. */
int dqdk_gpu_histogram_get(dqdk_gpu_queue_t* q, uint32_t* host_hist);
/* Add (u32 wrap) the queue's histogram into host_hist: the end-of-run merge
 * of per-GPU partials into the one tristan_histo_t (src/tristan.c:97). */
int dqdk_gpu_histogram_accumulate(dqdk_gpu_queue_t* q, uint32_t* host_hist);
int dqdk_gpu_histogram_reset(dqdk_gpu_queue_t* q);
/* The device table is held as two planes (u32 base + low byte, value = sum
 * mod 2^32; the partitioned path sweeps only the 0.6 GB low plane per
 * batch).  device_ptr materialises the u32 table into a queue-owned device
 * buffer (synchronous) and returns it, valid until the next call or queue
 * destroy; NULL if the queue has no histogram. */
uint32_t* dqdk_gpu_histogram_device_ptr(dqdk_gpu_queue_t* q);
/* Partitioned batches stage their slice-sorted events and the slice pass
 * (the sweep of the table's low-byte plane) runs once per
 * batches_per_pass staged batches (up to 32, as many as the staging budget
 * above holds: 32 at 1M x 1500 B, 21 at 1M x 9000 B; DQDK_GPU_F_HISTO_EAGER:
 * 1).  Every histogram reader above and below flushes first; flush runs
 * the pending slice pass now (async on the queue stream). */
int dqdk_gpu_histogram_flush(dqdk_gpu_queue_t* q);
int dqdk_gpu_histogram_batches_per_pass(dqdk_gpu_queue_t* q);

/* ---- end-of-run egress (tristan_fini, src/tristan.c:162-233) ------------- */
/* Merge helpers for per-GPU partial tables.  d_dst / d_src are device
 * pointers to DQDK_TRISTAN_HISTO_ENTRIES u32 (16-B aligned) reachable from
 * the queue's device; both run async on the queue stream.  copy: d_dst =
 * the u32 table (e.g. into an RCCL reduce buffer); add: table += d_src (u32
 * wrap). */
int dqdk_gpu_histogram_copy(dqdk_gpu_queue_t* q, uint32_t* d_dst);
int dqdk_gpu_histogram_add(dqdk_gpu_queue_t* q, const uint32_t* d_src);
/* Number of non-zero bins (synchronous). */
int dqdk_gpu_histogram_nonzero(dqdk_gpu_queue_t* q, uint64_t* count);
/* Write the histogram file of tristan_fini (src/tristan.c:197-216) to fd:
 * the header "Channel,Histo,Energy,Freq\n" then "%d,%d,%u,%u\n" (channel,
 * histogram, energy bin, count) for every non-zero bin in table order.  The
 * text is formatted on the GPU chunk by chunk; only the text is copied to
 * the host.  *bytes_written (nullable) = bytes written to fd. */
int dqdk_gpu_histogram_write_csv(dqdk_gpu_queue_t* q, int fd, uint64_t* bytes_written);
/* The JSON status line tristan_fini sends to the controller
 * (src/tristan.c:171-189): events/bytes summed over the queues' counters,
 * packets = sum of rcvd_pkts, runtime = max of runtime_ns[k] (nullable)
 * in ms with 2 decimals.  Returns the snprintf length (truncates to bufsz). */
int dqdk_gpu_tristan_summary(const dqdk_gpu_counters_t* const* per_queue, int nqueues, const uint64_t* runtime_ns,
                             const char* directory, char* buf, uint64_t bufsz);

/* ---- measurement helpers (membench.hip; not on the receive path) --------- */
/* Streaming read of [d_buf, d_buf+bytes) (16-B aligned) on `stream`, and
 * one relaxed device atomic increment of d_table[d_keys[i]] per key (keys
 * >= entries skipped): iters timed passes after one warm-up, mean ms/pass. */
int dqdk_gpu_membench_read(const void* d_buf, uint64_t bytes, void* stream, int iters, double* ms_per_pass);
int dqdk_gpu_membench_atomic(uint32_t* d_table, uint64_t entries, const uint32_t* d_keys, uint64_t nkeys, void* stream,
                             int iters, double* ms_per_pass);
/* The receive path's memory traffic without its arithmetic: n frames at
 * `stride` in d_umem, frame_bytes (multiple of 16) read from each and
 * out_bytes_per_frame written per frame to d_out (16-B aligned; nullable:
 * read only).  flat = 0: one wave per frame, a frame at a time (the shape
 * of a per-frame loop); flat = 1: a flat grid-stride walk over all chunks
 * with four loads in flight per lane and the stores interleaved; flat = 2:
 * as 0 with 16-B record stores (4 words per lane) instead of 4-B ones;
 * flat = 3: no frames, n * stride bytes read contiguously and a quarter of
 * that written (d_out must hold n * stride / 4 bytes); flat = 4: a plain
 * 1:1 copy of n * stride bytes into d_out; flat = 5: write calibration, no
 * frames (d_umem ignored): n wave instructions of 4-B-per-lane stores, each
 * 64 aligned dwords (out_bytes_per_frame = 0) or a run of
 * out_bytes_per_frame / 4 (< 64) dwords at an unaligned offset, runs of one
 * wave adjacent (d_out 256-B aligned, sized by the caller for
 * n * 256 + 64 K bytes). */
int dqdk_gpu_membench_frames(const void* d_umem, uint64_t stride, uint32_t frame_bytes, uint32_t n, void* d_out,
                             uint32_t out_bytes_per_frame, int flat, void* stream, int iters, double* ms_per_pass);

/* ---- stage timing (HIP events on the queue stream) ------------------------ */
/* When enabled, every kernel launch of every batch is bracketed by its own
 * pair of hipEvents on the queue stream; stage k is one kernel, named by
 * dqdk_gpu_timing_stage_name(k):
 *   0 rx_decode (or the fused decode)  1 rx_abort  2 rx_count  3 rx_histo_atomic
 *   4 rx_part1   5 (unused)  6 rx_part2  7 rx_slice_histo  8 (unused)
 *   9 rx_fixup (fused path: the rx_part1 launch that takes the decode's piece
 *     sizes, its decoded frames whose final status is not OK and its overflow list)
 * timing_read adds up the completed pairs (after syncing the queue stream),
 * writes stage_ms[k] / counts[k] (launches) for k < nstages and clears them. */
#define DQDK_GPU_TIMING_STAGES 10
int dqdk_gpu_timing_enable(dqdk_gpu_queue_t* q, int on);
/* Restrict the bracketing to the stages whose bit is set in stage_mask
 * (default: all); the others launch without events in between. */
int dqdk_gpu_timing_stages(dqdk_gpu_queue_t* q, uint32_t stage_mask);
int dqdk_gpu_timing_read(dqdk_gpu_queue_t* q, double* stage_ms, uint64_t* counts, int nstages);
const char* dqdk_gpu_timing_stage_name(int stage); /* NULL when out of range */

/* ---- staging placement probe (no reference counterpart) ------------------- */
/* The fused decode's rate depends on where its piece buffer lands physically
 * relative to the UMEM image it reads.  A queue's first
 * fused batches of at least 65536 frames run on DQDK_GPU_PROBE_CANDS candidate
 * piece buffers in turn (each candidate's first batch untimed, then two more
 * batches each, in order and then in reverse order, their decodes timed by
 * HIP events: 3 x DQDK_GPU_PROBE_CANDS batches); at the next such batch the
 * fastest mean is kept, the others freed (DQDK_GPU_STAGING_PROBE=0 at queue
 * creation: off).  This reads the outcome: *chosen = the kept candidate (-1:
 * not decided yet, -2: off), ns_per_frame[k] = candidate k's mean decode
 * time per frame (0: untimed), k < ncand.
 * Returns the number of candidates. */
#define DQDK_GPU_PROBE_CANDS 8  /* (5 until round 6: one fast placement in five was common at 9000 B) */
int dqdk_gpu_queue_staging_probe(dqdk_gpu_queue_t* q, int* chosen, float* ns_per_frame, int ncand);

const char* dqdk_gpu_last_error(void);

/* ---- synthetic UMEM generator (bench/test input only; host C) ------------ */
typedef struct dqdk_synth_cfg {
    uint64_t seed;      /* counter-based PRNG seed (20261015) */
    uint32_t queue;     /* RX queue id: UDP source port 5000+queue           */
    uint32_t frame_len; /* L; 0 = seeded 50/50 mix of 1500 and 9000 B        */
    uint32_t stride;    /* UMEM bytes per frame slot (4096, 9216, ...)       */
    uint32_t faulty;    /* bit 0: inject header/checksum/event faults;       */
                        /* bit 1 (DQDK_SYNTH_PEAKED): skewed spectrum         */
} dqdk_synth_cfg_t;
#define DQDK_SYNTH_PEAKED 2u

uint64_t dqdk_synth_umem_size(const dqdk_synth_cfg_t* c, uint32_t n);
uint32_t dqdk_synth_frame_len(const dqdk_synth_cfg_t* c, uint64_t frame_index);
/* Fill umem[0, n*stride) with frames first..first+n-1 and their descriptors. */
int dqdk_synth_frames(const dqdk_synth_cfg_t* c, uint64_t first, uint32_t n, uint8_t* umem, uint64_t umem_size,
                      dqdk_gpu_desc_t* d, int threads);

#ifdef __cplusplus
}
#endif
#endif
