/*
 * dqdk_oracle.h -- CPU restatement of the DQDK receive hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the HIP path is compared
 * against.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; nothing under dqdk_amd/ links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - src/tcpip (ip4_audit, udp_audit, *_audit_checksum, udp_csum, inet_csum
 *     family) is PINNED: tests/test_oracle_ref.py compares every function
 *     here with the reference's own src/tcpip/{ipv4,udp,inet_csum}.c compiled verbatim into
 *     oracle/_ref/ (oracle/Makefile), and tests/golden/ holds fixtures made
 *     from that build (tests/golden/gen_golden.py: F1, F2).
 *   - the TRISTAN decode (histogram_event, process_events_unrolled16,
 *     tristan_process incl. its burst form, get_energy_events_count, the
 *     energy_evt / tristan_histo_t layout; src/tristan.{c,h}) is PINNED:
 *     oracle/ref_tristan.py compiles those functions extracted verbatim into
 *     oracle/_ref/libref_tristan.so, tests/golden/gen_tristan.py records
 *     F3 (events, frame cases, async bursts) and F4 (a 1024-frame batch
 *     under both accountings) from it, and test_golden.py / test_oracle_ref.py
 *     check this restatement against them.
 *   - the get_udp_payload / process_frame / fetch_xsk glue (src/dqdk.c:185-322)
 *     stays a restatement: dqdk.c's only type, dqdk_worker_t, embeds libxdp
 *     ring structs absent from this image, so its text cannot be compiled
 *     without stand-ins.  Every verdict it composes is a pinned tcpip call,
 *     and F4's expected counters are built by the same composition around
 *     the reference's own calls.
 *
 * All citations are path:line relative to the reference checkout.
 */
#ifndef DQDK_ORACLE_H
#define DQDK_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- src/tcpip/inet_csum.c ------------------------------------------- */
uint16_t or_from32to16(uint32_t x);                               /* :43-50  */
uint32_t or_from64to32(uint64_t x);                               /* :56-63  */
uint32_t or_inet_csum(const uint8_t* buff, int len);              /* :69-123 */
uint16_t or_inet_fast_csum(const void* data, unsigned size);      /* :125-128 */
uint16_t or_ip_fast_csum(const void* iph, unsigned ihl);          /* :136-139 */
uint32_t or_csum_tcpudp_nofold(uint32_t saddr, uint32_t daddr,
                               uint32_t len, uint8_t proto, uint32_t sum); /* :145-158 */
uint16_t or_csum_fold(uint32_t csum);                             /* :165-172 */
uint16_t or_csum_tcpudp_magic(uint32_t saddr, uint32_t daddr, uint32_t len,
                              uint8_t proto, uint32_t sum);       /* :178-182 */
uint16_t or_udp_csum(uint32_t saddr, uint32_t daddr, uint32_t len,
                     uint8_t proto, const uint8_t* udp_pkt);      /* :184-216 */

/* ---- src/tcpip/ipv4.c, udp.c ----------------------------------------- */
int or_ip4_audit(const uint8_t* iph, uint16_t actual_pkt_len);    /* ipv4.c:13-20 */
int or_ip4_audit_checksum(const uint8_t* iph);                    /* ipv4.c:6-11  */
int or_udp_audit(const uint8_t* udp, uint32_t saddr, uint32_t daddr,
                 uint16_t udplen);                                /* udp.c:22-31  */
/* writeback != 0 reproduces the in-place `udp->check = 0` (udp.c:17). */
int or_udp_audit_checksum(uint8_t* udp, uint32_t saddr, uint32_t daddr,
                          uint16_t udplen, int writeback);        /* udp.c:10-20  */

/* ---- batch path: src/dqdk.c:185-322 + src/tristan.c:72-85,233-330 ----- */

/* struct xdp_desc (linux/if_xdp.h) */
typedef struct {
    uint64_t addr;
    uint32_t len;
    uint32_t options;
} or_desc_t;

/* Per-frame verdicts.  Numbering shared with include/dqdk_gpu.h. */
enum {
    OR_RX_OK = 0,              /* frame_processor called                     */
    OR_RX_INVALID_IP = 1,      /* ip4_audit length check failed              */
    OR_RX_INVALID_UDP = 2,     /* udp_audit length check failed              */
    OR_RX_EMPTY = 3,           /* datalen == 0 -> -ENOBUFS (dqdk.c:247-248)  */
    OR_RX_INVALID_IP_CSUM = 4, /* checksum config: ip4_audit_checksum failed */
    OR_RX_INVALID_UDP_CSUM = 5,/* checksum config: udp_audit_checksum failed */
    OR_RX_FILTER_DROP = 6,     /* prefilter (forwarder.bpf.c) -> XDP_DROP    */
    OR_RX_FILTER_PASS = 7,     /* prefilter -> XDP_PASS (not for this XSK)   */
};

typedef struct {
    uint32_t datalen;     /* u32 as in get_udp_payload (may wrap)            */
    uint8_t status;
    uint8_t payload_off;  /* 14 + ihl*4 + 8 (valid for OK / EMPTY)           */
    uint16_t oob_events;  /* events skipped by histogram_event (saturating)  */
} or_result_t;

typedef struct {
    uint64_t rcvd_frames, rcvd_pkts, rcvd_bytes;
    uint64_t invalid_ip_pkts, invalid_udp_pkts, failing_batches;
    uint64_t total_events, total_bytes, oob_events;
    uint64_t empty_pkts, filtered_frames;
    uint64_t first_abort_idx; /* index into the batch; n when no abort       */
} or_counters_t;

/* tristan_mode_t (src/tristan.h:62-67) */
enum { OR_MODE_WAVEFORM = 0, OR_MODE_LISTWAVE = 1, OR_MODE_LISTMODE = 2, OR_MODE_ENERGYHISTO = 3 };

enum {
    OR_F_CSUM = 1u << 0,        /* ip4/udp checksum verify (commented-out config) */
    OR_F_BATCH_ABORT = 1u << 1, /* fetch_xsk stops at first failing frame         */
    OR_F_PREFILTER = 1u << 2,   /* apply dqdk_forwarder predicate first           */
    OR_F_NO_HISTO = 1u << 3,    /* do not accumulate the histogram                */
    OR_F_CSUM_WRITEBACK = 1u << 4, /* zero udp->check in UMEM like udp.c:17      */
};

typedef struct {
    uint32_t payloadsz;
    uint32_t mode;
    uint32_t flags;
    uint16_t port_start, port_end;
} or_cfg_t;

#define OR_CHNLS_COUNT 1512u      /* tristan.h:57-59 */
#define OR_CHANNELHISTO_COUNT 6u  /* tristan.h:56    */
#define OR_HISTO_BINS 65536u      /* tristan.h:55    */
#define OR_HISTO_ENTRIES ((uint64_t)OR_CHNLS_COUNT * OR_CHANNELHISTO_COUNT * OR_HISTO_BINS)
#define OR_KEY_NONE 0xFFFFFFFFu

uint32_t or_events_per_payload(uint32_t mode, uint32_t payloadsz); /* tristan.c:72-85 */

/* histogram_event (tristan.c:233-245) as a key: the flat index
 * (ch*6 + hc)*65536 + (energy >> 8) it increments, or OR_KEY_NONE when it
 * rejects the event as out of bounds. */
uint32_t or_event_key(const uint8_t* evt);

/* dqdk_forwarder predicate (src/bpf/forwarder.bpf.c:38-96): 0 DROP, 1 PASS, 2 REDIRECT */
int or_prefilter(const uint8_t* frame, uint32_t len, uint16_t start, uint16_t end);

/*
 * One fetch_xsk batch (dqdk.c:252-322) with the sync frame processor
 * process_unbuffered_frame (tristan.c:377-381).
 *   umem/umem_size : the UMEM image; bytes at or past umem_size read as 0
 *   res[n]         : per-frame verdict (always filled for every frame)
 *   cnt            : counters are ADDED to (like xsk->stats / tristan_t)
 *   hist           : OR_HISTO_ENTRIES u32 table or NULL
 *   keys           : n*E u32 flat bin indices (OR_KEY_NONE for OOB events),
 *                    written only for frames whose status is OK, or NULL
 */
int or_rx_batch(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n,
                const or_cfg_t* cfg, or_result_t* res, or_counters_t* cnt,
                uint32_t* hist, uint32_t* keys);

/* Multi-threaded driver for the CPU baseline: T threads, each one queue
 * (one contiguous slice of the descriptors), shared histogram like the
 * reference's shared tristan_t (relaxed atomics, tristan.c:243).  Returns
 * elapsed seconds. */
double or_rx_batch_threads(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n,
                           const or_cfg_t* cfg, or_result_t* res, or_counters_t* cnt,
                           uint32_t* hist, int threads);

/* or_rx_batch's exact outputs (results, keys, counters, histogram) for
 * large batches, computed by T threads over contiguous slices of the
 * descriptors and merged (counters summed, failing_batches = any failure,
 * first_abort_idx = the first failing index).  Per-packet accounting only:
 * with OR_F_BATCH_ABORT or OR_F_CSUM_WRITEBACK (or T <= 1) it runs
 * or_rx_batch itself.  Test infrastructure for full-size parity checks. */
int or_rx_batch_mt(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n, const or_cfg_t* cfg,
                   or_result_t* res, or_counters_t* cnt, uint32_t* hist, uint32_t* keys, int threads);

/*
 * The async consumer (async_processor, tristan.c:332-375) over a ring of
 * nelem elements of payloadsz bytes (post_async's elements, dqdk.c:220-229),
 * fetched in bursts of bursts[k] elements (the `ret` of each
 * dqdk_async_processor_nfetch): tristan_process(buffer, len, ret) with
 * len = strip_wfm ? 16 : payloadsz (:343).  Adds to cnt->total_events /
 * total_bytes / oob_events, to hist (may be NULL), and appends the bytes
 * write() would receive to raw_out (up to raw_cap; *raw_total = full length).
 * Returns -1 if the bursts overrun the ring.
 */
int or_async_process(const uint8_t* ring, uint64_t nelem, const uint32_t* bursts, uint32_t nbursts,
                     const or_cfg_t* cfg, int strip_wfm, or_counters_t* cnt, uint32_t* hist,
                     uint8_t* raw_out, uint64_t raw_cap, uint64_t* raw_total);

#ifdef __cplusplus
}
#endif
#endif
