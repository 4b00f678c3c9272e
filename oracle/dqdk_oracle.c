/*
 * dqdk_oracle.c -- CPU restatement of the DQDK receive hot path.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the product): see the header
 * comment of dqdk_oracle.h for who may call this and how it is pinned.
 *
 * Every function restates the reference function named in its comment,
 * file:line relative to the reference checkout.  The restatement keeps the
 * reference's integer widths (u16 truncations, u32 wraps) because the GPU
 * path must reproduce them bit for bit.
 */
#define _GNU_SOURCE
#include "dqdk_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static inline uint16_t ld16le(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint16_t ld16be(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t ld32le(const uint8_t* p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* ---------------------------------------------------------------------- */
/* src/tcpip/inet_csum.c                                                   */
/* ---------------------------------------------------------------------- */

/* inet_csum.c:43-50 */
uint16_t or_from32to16(uint32_t x)
{
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return (uint16_t)x;
}

/* inet_csum.c:56-63 */
uint32_t or_from64to32(uint64_t x)
{
    x = (x & 0xffffffffull) + (x >> 32);
    x = (x & 0xffffffffull) + (x >> 32);
    return (uint32_t)x;
}

/* inet_csum.c:69-123 -- Linux lib/checksum.c do_csum: the head handling
 * depends on the ADDRESS parity of buff, so this is restated on the real
 * pointer.  Byte-order branches: inet_csum.c's translation unit includes
 * only <linux/types.h> and ctypes.h, which do NOT define __LITTLE_ENDIAN
 * (glibc's <endian.h> does, but it is not included there), so the reference
 * build takes the `#else` arms at :80-82 and :115-116 even on x86.  Pinned by
 * tests/golden/f2_csum.npz.  (The hot path only calls this on a 4-aligned
 * copy with a multiple-of-4 length, where neither arm runs.) */
uint32_t or_inet_csum(const uint8_t* buff, int len)
{
    uint32_t result = 0;
    int odd;

    if (len <= 0)
        return 0;
    odd = 1 & (uintptr_t)buff;
    if (odd) {
        result = *buff; /* :81 (#else arm, see above) */
        len--;
        buff++;
    }
    if (len >= 2) {
        if (2 & (uintptr_t)buff) {
            result += ld16le(buff);
            len -= 2;
            buff += 2;
        }
        if (len >= 4) {
            const uint8_t* end = buff + ((unsigned int)len & ~3u);
            uint32_t carry = 0;
            do {
                uint32_t w = ld32le(buff);
                buff += 4;
                result += carry;
                result += w;
                carry = (w > result);
            } while (buff < end);
            result += carry;
            result = (result & 0xffff) + (result >> 16);
        }
        if (len & 2) {
            result += ld16le(buff);
            buff += 2;
        }
    }
    if (len & 1)
        result += (uint32_t)(*buff << 8); /* :116 (#else arm) */
    result = or_from32to16(result);
    if (odd)
        result = ((result >> 8) & 0xff) | ((result & 0xff) << 8);
    return result;
}

/* inet_csum.c:125-128 */
uint16_t or_inet_fast_csum(const void* data, unsigned size)
{
    return (uint16_t)~or_inet_csum((const uint8_t*)data, (int)size);
}

/* inet_csum.c:136-139 */
uint16_t or_ip_fast_csum(const void* iph, unsigned ihl)
{
    return or_inet_fast_csum(iph, ihl * 4);
}

/* inet_csum.c:145-158 (little-endian branch: (proto + len) << 8) */
uint32_t or_csum_tcpudp_nofold(uint32_t saddr, uint32_t daddr, uint32_t len, uint8_t proto, uint32_t sum)
{
    unsigned long long s = (uint32_t)sum;
    s += (uint32_t)saddr;
    s += (uint32_t)daddr;
    s += (uint32_t)((proto + len) << 8);
    return or_from64to32(s);
}

/* inet_csum.c:165-172 */
uint16_t or_csum_fold(uint32_t csum)
{
    uint32_t sum = csum;
    sum = (sum & 0xffff) + (sum >> 16);
    sum = (sum & 0xffff) + (sum >> 16);
    return (uint16_t)~sum;
}

/* inet_csum.c:178-182 */
uint16_t or_csum_tcpudp_magic(uint32_t saddr, uint32_t daddr, uint32_t len, uint8_t proto, uint32_t sum)
{
    return or_csum_fold(or_csum_tcpudp_nofold(saddr, daddr, len, proto, sum));
}

/* inet_csum.c:184-216, USE_SIMD undefined (src/dqdk.c:2 commented, src/Makefile:13):
 * u32 sum of the LE u16 words at udp_pkt[0 .. len) step 2.  For odd len the
 * last word's high byte is the byte AT udp_pkt[len]. */
uint16_t or_udp_csum(uint32_t saddr, uint32_t daddr, uint32_t len, uint8_t proto, const uint8_t* udp_pkt)
{
    uint32_t sum = 0;
    for (uint32_t cnt = 0; cnt < len; cnt += 2)
        sum += ld16le(udp_pkt + cnt);
    return or_csum_tcpudp_magic(saddr, daddr, len, proto, sum);
}

/* ---------------------------------------------------------------------- */
/* src/tcpip/ipv4.c, src/tcpip/udp.c                                       */
/* ---------------------------------------------------------------------- */

/* ipv4.c:13-20: only `ntohs(tot_len) == actual_pkt_len` is live; the
 * checksum term is commented out at :16. */
int or_ip4_audit(const uint8_t* iph, uint16_t actual_pkt_len)
{
    uint16_t len = ld16be(iph + 2);
    return len == actual_pkt_len;
}

/* ipv4.c:6-11: copy the 20-B struct iphdr, zero .check, compare
 * ip_fast_csum(copy, ihl) with the original .check.  For ihl > 5 the
 * reference reads past its 20-B stack copy (undefined); here the extra
 * words come from the real header, which is the only reproducible choice
 * (the GPU path does the same; fixtures restrict to ihl <= 5). */
int or_ip4_audit_checksum(const uint8_t* iph)
{
    uint32_t copy32[16];
    uint8_t* copy = (uint8_t*)copy32; /* 4-aligned like struct iphdr */
    unsigned ihl = iph[0] & 0x0f;
    unsigned n = ihl * 4 > 20 ? ihl * 4 : 20;
    memcpy(copy, iph, n);
    copy[10] = copy[11] = 0;
    uint16_t check = ld16le(iph + 10);
    return or_ip_fast_csum(copy, ihl) == check;
}

/* udp.c:22-31: only `ntohs(udp->len) == udplen` is live (checksum commented :26). */
int or_udp_audit(const uint8_t* udp, uint32_t saddr, uint32_t daddr, uint16_t udplen)
{
    (void)saddr;
    (void)daddr;
    return ld16be(udp + 4) == udplen;
}

/* udp.c:10-20: check == 0 -> valid; otherwise zero udp->check IN PLACE
 * (never restored), recompute with udp_csum and compare.  No 0 -> 0xFFFF
 * mapping. */
int or_udp_audit_checksum(uint8_t* udp, uint32_t saddr, uint32_t daddr, uint16_t udplen, int writeback)
{
    uint16_t rcvd = ld16le(udp + 6);
    if (rcvd == 0)
        return 1;
    uint8_t c6 = udp[6], c7 = udp[7];
    udp[6] = udp[7] = 0;
    uint16_t calc = or_udp_csum(saddr, daddr, udplen, 17 /* IPPROTO_UDP */, udp);
    if (!writeback) {
        udp[6] = c6;
        udp[7] = c7;
    }
    return calc == rcvd;
}

/* ---------------------------------------------------------------------- */
/* src/bpf/forwarder.bpf.c:38-96 -- optional pre-filter (row a-0)           */
/* ---------------------------------------------------------------------- */
int or_prefilter(const uint8_t* f, uint32_t len, uint16_t start, uint16_t end)
{
    if (len <= 14) /* :44-52 data >= end, data + ETH_HLEN >= end */
        return 0;
    if (!(f[12] == 0x08 && f[13] == 0x00)) /* :60-63 h_proto != ETH_P_IP */
        return 1;
    if (len <= 34) /* :66-69 PAYLOAD(ip) >= end (ip assumed 20 B) */
        return 0;
    if (f[23] != 17) /* :71-74 protocol != UDP */
        return 1;
    if (len <= 42) /* :77-80 PAYLOAD(udp) >= end (udp at +34, ihl ignored) */
        return 0;
    uint16_t sport = ld16be(f + 34); /* :32-36 check_in_range */
    if (!(sport <= end && sport >= start))
        return 1;
    return 2;
}

/* ---------------------------------------------------------------------- */
/* src/tristan.c                                                           */
/* ---------------------------------------------------------------------- */

/* tristan.c:72-85 */
uint32_t or_events_per_payload(uint32_t mode, uint32_t payloadsz)
{
    switch (mode) {
    case OR_MODE_LISTMODE:
    case OR_MODE_ENERGYHISTO:
        return payloadsz / 16; /* TRISTAN_HISTO_EVT_SZ, tristan.h:53 */
    case OR_MODE_LISTWAVE:
    case OR_MODE_WAVEFORM:
        return 1;
    default:
        return 0;
    }
}

/* tristan.c:65-70 is_store_histo -> histo_fd > 0 in tristan_init (:135-150) */
static int histo_enabled(const or_cfg_t* cfg)
{
    if (cfg->flags & OR_F_NO_HISTO)
        return 0;
    return cfg->mode == OR_MODE_LISTWAVE || cfg->mode == OR_MODE_LISTMODE || cfg->mode == OR_MODE_ENERGYHISTO;
}

/* struct energy_evt (tristan.h:13-25), packed little-endian:
 *   [0:2] id  [2:4] channel  [4:7] energy:24  [7] trigger_flags
 *   [8] hist_class:3 | reserved:5  [9] multiplicity  [10:16] timestamp:48
 * histogram_event (tristan.c:233-245): bin = energy >> 8 (bytes 5,6 LE);
 * channel >= CHNLS_COUNT or hist_class >= CHANNELHISTO_COUNT is skipped
 * (the bin >= HISTO_MAXVAL test can never fire); otherwise
 * histo->channels[ch].histograms[hc][bin]++ (relaxed atomic). */
static inline uint32_t evt_key(const uint8_t* e)
{
    uint32_t ch = ld16le(e + 2);
    uint32_t energy = (uint32_t)e[4] | ((uint32_t)e[5] << 8) | ((uint32_t)e[6] << 16);
    uint32_t hc = e[8] & 7;
    uint32_t bin = energy >> 8;
    if (ch >= OR_CHNLS_COUNT || hc >= OR_CHANNELHISTO_COUNT)
        return OR_KEY_NONE;
    return (ch * OR_CHANNELHISTO_COUNT + hc) * OR_HISTO_BINS + bin;
}

uint32_t or_event_key(const uint8_t* evt) { return evt_key(evt); }

/* tristan_process (tristan.c:308-330) with burst = ret, as async_processor
 * calls it (:343-349): the histogram loop runs `burst` times over the SAME
 * buffer base (:314-315), the raw write is len * burst bytes from the buffer
 * start (:319), total_bytes += len * burst (u32 product, :327) and
 * total_events += E once (:328). */
int or_async_process(const uint8_t* ring, uint64_t nelem, const uint32_t* bursts, uint32_t nbursts,
                     const or_cfg_t* cfg, int strip_wfm, or_counters_t* c, uint32_t* hist,
                     uint8_t* raw_out, uint64_t raw_cap, uint64_t* raw_total)
{
    const uint32_t E = or_events_per_payload(cfg->mode, cfg->payloadsz);
    const int histo = histo_enabled(cfg);
    const uint32_t len = strip_wfm ? 16u : cfg->payloadsz; /* :343 TRISTAN_HISTO_EVT_SZ */
    uint64_t e0 = 0, out = 0;
    for (uint32_t k = 0; k < nbursts; k++) {
        const uint32_t burst = bursts[k];
        if (e0 + burst > nelem)
            return -1;
        const uint8_t* buf = ring + e0 * cfg->payloadsz;
        if (histo) {
            uint32_t oob = 0;
            for (uint32_t e = 0; e < E; e++) {
                uint32_t key = evt_key(buf + 16 * (size_t)e);
                if (key == OR_KEY_NONE)
                    oob++;
                else if (hist)
                    hist[key] += burst;
            }
            c->oob_events += (uint64_t)oob * burst;
        }
        const uint32_t wlen = len * burst; /* u32, as write()'s count is computed */
        for (uint32_t b = 0; b < wlen; b++, out++)
            if (raw_out && out < raw_cap)
                raw_out[out] = buf[b];
        c->total_bytes += wlen;
        c->total_events += E;
        e0 += burst;
    }
    if (raw_total)
        *raw_total = out;
    return 0;
}

/* ---------------------------------------------------------------------- */
/* src/dqdk.c -- get_udp_payload / process_frame / fetch_xsk                */
/* ---------------------------------------------------------------------- */

typedef struct {
    uint8_t status;
    uint8_t payload_off;
    uint32_t datalen;
} frame_verdict_t;

/* get_udp_payload (dqdk.c:185-207) + the checksum configuration, on a
 * frame whose bytes [0, need) are all addressable. */
static frame_verdict_t parse_frame(uint8_t* f, uint32_t len, uint32_t flags)
{
    frame_verdict_t v = { 0, 0, 0 };
    uint8_t* iph = f + 14;                                        /* :187 */
    int ip_ok = or_ip4_audit(iph, (uint16_t)(len - 14));          /* :191 */
    if (ip_ok && (flags & OR_F_CSUM) && !or_ip4_audit_checksum(iph)) {
        v.status = OR_RX_INVALID_IP_CSUM;                         /* ipv4.c:16 */
        return v;
    }
    if (!ip_ok) {
        v.status = OR_RX_INVALID_IP;
        return v;
    }
    uint32_t iphdrsz = (uint32_t)(iph[0] & 0x0f) * 4;             /* :196 */
    uint32_t udplen = (uint32_t)ld16be(iph + 2) - iphdrsz;        /* :197 u32 wrap */
    uint8_t* udp = iph + iphdrsz;                                 /* :198 */
    uint32_t saddr = ld32le(iph + 12), daddr = ld32le(iph + 16);
    int udp_ok = or_udp_audit(udp, saddr, daddr, (uint16_t)udplen); /* :200 */
    if (udp_ok && (flags & OR_F_CSUM)
        && !or_udp_audit_checksum(udp, saddr, daddr, (uint16_t)udplen, (flags & OR_F_CSUM_WRITEBACK) != 0)) {
        v.status = OR_RX_INVALID_UDP_CSUM;                        /* udp.c:26 */
        return v;
    }
    if (!udp_ok) {
        v.status = OR_RX_INVALID_UDP;
        return v;
    }
    v.datalen = udplen - 8;                                       /* :205 */
    v.payload_off = (uint8_t)(14 + iphdrsz + 8);                  /* :206 */
    v.status = v.datalen ? OR_RX_OK : OR_RX_EMPTY;                /* :243-248 */
    return v;
}

/* Per-thread scratch for frames whose reads run past the UMEM end. */
typedef struct {
    uint8_t* buf;
    size_t cap;
} scratch_t;

static uint8_t* scratch_get(scratch_t* s, size_t need)
{
    if (s->cap < need) {
        free(s->buf);
        s->cap = need + 4096;
        s->buf = (uint8_t*)malloc(s->cap);
    }
    return s->buf;
}

/* Bytes of the frame that any stage may touch: headers (<= 82 B), the UDP
 * checksum range (udp + u16 udplen + 1 odd over-read) and the E*16-B decode
 * range from the payload start. */
static uint64_t frame_extent(uint32_t E, uint32_t flags)
{
    uint64_t ext = 14 + 60 + 8 + 16;
    if (flags & OR_F_CSUM)
        ext = 14 + 60 + 65536 + 2;
    uint64_t dec = 14 + 60 + 8 + (uint64_t)E * 16;
    return dec > ext ? dec : ext;
}

static void process_one(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, const or_cfg_t* cfg,
                        uint32_t E, int histo, or_result_t* r, uint32_t* keys_out, scratch_t* sc)
{
    uint64_t ext = frame_extent(E, cfg->flags);
    uint8_t* f;
    int copied = 0;
    if (d->addr <= umem_size && umem_size - d->addr >= ext) {
        f = umem + d->addr;
    } else {
        /* bytes at or past umem_size read as zero (defined here and on the
         * GPU; the reference would read whatever follows its mapping) */
        f = scratch_get(sc, ext);
        memset(f, 0, ext);
        if (d->addr < umem_size)
            memcpy(f, umem + d->addr, umem_size - d->addr);
        copied = 1;
    }

    r->datalen = 0;
    r->payload_off = 0;
    r->oob_events = 0;

    if (cfg->flags & OR_F_PREFILTER) {
        int pf = or_prefilter(f, d->len, cfg->port_start, cfg->port_end);
        if (pf != 2) {
            r->status = pf == 0 ? OR_RX_FILTER_DROP : OR_RX_FILTER_PASS;
            return;
        }
    }

    frame_verdict_t v = parse_frame(f, d->len, cfg->flags);
    r->status = v.status;
    if (v.status == OR_RX_OK || v.status == OR_RX_EMPTY) {
        r->datalen = v.datalen;
        r->payload_off = v.payload_off;
    }
    if (copied && (cfg->flags & OR_F_CSUM_WRITEBACK) && d->addr < umem_size)
        memcpy(umem + d->addr, f, umem_size - d->addr);

    if (v.status != OR_RX_OK || (!keys_out && !histo))
        return;
    /* process_events_unrolled16 (tristan.c:247-304) reads E events from the
     * payload start regardless of datalen (tristan.c:311, :315).  The OOB
     * count is histogram_event's: 0 when the mode keeps no histogram
     * (histo_fd < 0, tristan.c:312), whatever the frame's position in an
     * aborted batch (a per-frame property; the counter sums accounted frames). */
    const uint8_t* ev = f + v.payload_off;
    uint32_t oob = 0;
    for (uint32_t e = 0; e < E; e++) {
        uint32_t k = evt_key(ev + 16 * (size_t)e);
        oob += (k == OR_KEY_NONE);
        if (keys_out)
            keys_out[e] = k;
    }
    if (histo)
        r->oob_events = (uint16_t)(oob > 0xffff ? 0xffff : oob);
}

/* Accounting for one frame that fetch_xsk actually processed
 * (process_frame dqdk.c:231-250 -> process_unbuffered_frame tristan.c:377
 * -> tristan_process tristan.c:308-330 with burst = 1). */
static void account_one(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, const or_cfg_t* cfg, uint32_t E,
                        or_result_t* r, or_counters_t* c, uint32_t* hist, int histo)
{
    c->rcvd_pkts++; /* dqdk.c:189 */
    switch (r->status) {
    case OR_RX_INVALID_IP:
    case OR_RX_INVALID_IP_CSUM:
        c->invalid_ip_pkts++; /* :192 */
        return;
    case OR_RX_INVALID_UDP:
    case OR_RX_INVALID_UDP_CSUM:
        c->invalid_udp_pkts++; /* :201 */
        return;
    case OR_RX_EMPTY:
        c->empty_pkts++;
        return;
    default:
        break;
    }
    if (histo) {
        const uint8_t* ev = NULL;
        uint8_t* tmp = NULL;
        uint64_t need = (uint64_t)r->payload_off + (uint64_t)E * 16;
        if (d->addr <= umem_size && umem_size - d->addr >= need) {
            ev = umem + d->addr + r->payload_off;
        } else {
            tmp = (uint8_t*)calloc(need + 16, 1);
            if (d->addr < umem_size)
                memcpy(tmp, umem + d->addr, umem_size - d->addr);
            ev = tmp + r->payload_off;
        }
        uint32_t oob = 0;
        for (uint32_t e = 0; e < E; e++) {
            uint32_t k = evt_key(ev + 16 * (size_t)e);
            if (k == OR_KEY_NONE) {
                oob++;
                continue;
            }
            if (hist)
                __atomic_fetch_add(&hist[k], 1u, __ATOMIC_RELAXED); /* tristan.c:243 */
        }
        c->oob_events += oob;
        r->oob_events = (uint16_t)(oob > 0xffff ? 0xffff : oob);
        free(tmp);
    }
    c->total_bytes += (uint32_t)(r->datalen * 1u); /* tristan.c:327, len * burst */
    c->total_events += E;                          /* tristan.c:328 */
    c->rcvd_bytes += r->datalen;                   /* dqdk.c:245-246 */
}

int or_rx_batch(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n, const or_cfg_t* cfg,
                or_result_t* res, or_counters_t* c, uint32_t* hist, uint32_t* keys)
{
    uint32_t E = or_events_per_payload(cfg->mode, cfg->payloadsz);
    int histo = histo_enabled(cfg);
    scratch_t sc = { NULL, 0 };
    uint64_t abort_idx = n;
    int failed = 0;

    /* one pass in descriptor order, like the loop at dqdk.c:291-298 */
    for (uint32_t i = 0; i < n; i++) {
        or_result_t* r = &res[i];
        process_one(umem, umem_size, &d[i], cfg, E, histo, r, keys ? keys + (size_t)i * E : NULL, &sc);
        if (r->status == OR_RX_FILTER_DROP || r->status == OR_RX_FILTER_PASS) {
            c->filtered_frames++; /* never reaches the XSK ring */
            continue;
        }
        c->rcvd_frames++; /* dqdk.c:289 counts the whole peeked batch */
        if ((cfg->flags & OR_F_BATCH_ABORT) && failed)
            continue; /* dqdk.c:294-296: the rest of the batch is not processed */
        account_one(umem, umem_size, &d[i], cfg, E, r, c, hist, histo);
        if (r->status != OR_RX_OK && !failed) {
            failed = 1;
            abort_idx = i;
        }
    }
    free(sc.buf);
    if (failed)
        c->failing_batches++; /* dqdk.c:317-319 */
    c->first_abort_idx = abort_idx;
    return 0;
}

/* ---------------------------------------------------------------------- */
/* CPU-baseline driver: one thread per RX queue (dqdk.c:491-515), shared  */
/* histogram through relaxed atomics (tristan.c:243).                      */
/* ---------------------------------------------------------------------- */

typedef struct {
    uint8_t* umem;
    uint64_t umem_size;
    const or_desc_t* d;
    uint32_t n;
    const or_cfg_t* cfg;
    or_result_t* res;
    or_counters_t c;
    uint32_t* hist;
} thr_arg_t;

static void* thr_main(void* p)
{
    thr_arg_t* a = (thr_arg_t*)p;
    memset(&a->c, 0, sizeof(a->c));
    or_rx_batch(a->umem, a->umem_size, a->d, a->n, a->cfg, a->res, &a->c, a->hist, NULL);
    return NULL;
}

double or_rx_batch_threads(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n, const or_cfg_t* cfg,
                           or_result_t* res, or_counters_t* c, uint32_t* hist, int threads)
{
    if (threads < 1)
        threads = 1;
    thr_arg_t* args = (thr_arg_t*)calloc((size_t)threads, sizeof(thr_arg_t));
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; t++) {
        uint32_t lo = (uint32_t)t * per;
        uint32_t hi = lo + per > n ? n : lo + per;
        if (lo > n)
            lo = n;
        args[t] = (thr_arg_t){ umem, umem_size, d + lo, hi - lo, cfg, res + lo, { 0 }, hist };
        pthread_create(&tid[t], NULL, thr_main, &args[t]);
    }
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        c->rcvd_frames += args[t].c.rcvd_frames;
        c->rcvd_pkts += args[t].c.rcvd_pkts;
        c->rcvd_bytes += args[t].c.rcvd_bytes;
        c->invalid_ip_pkts += args[t].c.invalid_ip_pkts;
        c->invalid_udp_pkts += args[t].c.invalid_udp_pkts;
        c->failing_batches += args[t].c.failing_batches;
        c->total_events += args[t].c.total_events;
        c->total_bytes += args[t].c.total_bytes;
        c->oob_events += args[t].c.oob_events;
        c->empty_pkts += args[t].c.empty_pkts;
        c->filtered_frames += args[t].c.filtered_frames;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(args);
    free(tid);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------------- */
/* or_rx_batch over T threads with identical outputs (full-size checks).   */
/* ---------------------------------------------------------------------- */

typedef struct {
    uint8_t* umem;
    uint64_t umem_size;
    const or_desc_t* d;
    uint32_t lo, n;
    const or_cfg_t* cfg;
    or_result_t* res;
    or_counters_t c;
    uint32_t* hist;
    uint32_t* keys;
} mt_arg_t;

static void* mt_main(void* p)
{
    mt_arg_t* a = (mt_arg_t*)p;
    memset(&a->c, 0, sizeof(a->c));
    uint32_t E = or_events_per_payload(a->cfg->mode, a->cfg->payloadsz);
    or_rx_batch(a->umem, a->umem_size, a->d + a->lo, a->n, a->cfg, a->res + a->lo, &a->c, a->hist,
                a->keys ? a->keys + (size_t)a->lo * E : NULL);
    return NULL;
}

int or_rx_batch_mt(uint8_t* umem, uint64_t umem_size, const or_desc_t* d, uint32_t n, const or_cfg_t* cfg,
                   or_result_t* res, or_counters_t* c, uint32_t* hist, uint32_t* keys, int threads)
{
    if (threads <= 1 || n < 2 * (uint32_t)threads || (cfg->flags & (OR_F_BATCH_ABORT | OR_F_CSUM_WRITEBACK)))
        return or_rx_batch(umem, umem_size, d, n, cfg, res, c, hist, keys);
    if (threads > 64)
        threads = 64;
    mt_arg_t args[64];
    pthread_t tid[64];
    uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int t = 0; t < threads; t++) {
        uint32_t lo = (uint32_t)t * per;
        uint32_t hi = lo + per > n ? n : lo + per;
        if (lo > n)
            lo = n;
        args[t] = (mt_arg_t){ umem, umem_size, d, lo, hi - lo, cfg, res, { 0 }, hist, keys };
        pthread_create(&tid[t], NULL, mt_main, &args[t]);
    }
    uint64_t first = n;
    uint64_t failed = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        const or_counters_t* x = &args[t].c;
        c->rcvd_frames += x->rcvd_frames;
        c->rcvd_pkts += x->rcvd_pkts;
        c->rcvd_bytes += x->rcvd_bytes;
        c->invalid_ip_pkts += x->invalid_ip_pkts;
        c->invalid_udp_pkts += x->invalid_udp_pkts;
        c->total_events += x->total_events;
        c->total_bytes += x->total_bytes;
        c->oob_events += x->oob_events;
        c->empty_pkts += x->empty_pkts;
        c->filtered_frames += x->filtered_frames;
        if (x->failing_batches) {
            failed = 1;
            if (args[t].lo + x->first_abort_idx < first)
                first = args[t].lo + x->first_abort_idx;
        }
    }
    c->failing_batches += failed; /* dqdk.c:317-319: once per batch */
    c->first_abort_idx = first;
    return 0;
}
