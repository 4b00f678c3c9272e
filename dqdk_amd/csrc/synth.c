/*
 * synth.c -- deterministic synthetic UMEM generator (bench / test input).
 *
 * Writes TRISTAN-over-UDP frames the way SURVEY.md §8(d) specifies them:
 * counter-based PRNG (splitmix64 of seed, queue, frame, word), Ethernet type
 * 0x0800, IPv4 ihl=5 with a valid header checksum, UDP 5000+q -> 5000 with a
 * checksum valid under the reference's udp_csum rule
 * (src/tcpip/inet_csum.c:184-216), and 16-B energy events
 * (src/tristan.h:13-25) with channel U[0,1512), energy U[0,2^24),
 * hist_class U[0,6) -- the distribution of tests/structgenerator.py:12-16,
 * seeded.  The "faulty" variant injects, per frame at 1/256 each: bad
 * tot_len, bad udp.len, bad UDP checksum, ihl=6 (4 B of IP options), a
 * 42-B frame (datalen 0), a 40-B frame (udplen 6 < 8 -> datalen wraps); and
 * per event at 1/128 each: channel >= 1512, hist_class in {6,7}.  Bit 1 of
 * `faulty` (DQDK_SYNTH_PEAKED) piles 3 of every 8 events onto four hot bins
 * (three L1 buckets): the skewed spectra of real detectors, which overflow
 * the fused decode's LDS stages and per-block pieces.  Checksums are computed
 * after the events are written, so a peaked frame is still valid.
 *
 * This is input generation only.  It is not on the hot path and computes
 * nothing the GPU path returns.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "../../include/dqdk_gpu.h"

static inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t frame_base(const dqdk_synth_cfg_t* c, uint64_t g)
{
    return mix64(c->seed ^ ((uint64_t)c->queue << 40) ^ g);
}

static inline uint64_t rnd(uint64_t base, uint64_t w) { return mix64(base + w * 0xD1B54A32D192ED03ull); }

static inline void st16be(uint8_t* p, uint16_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
static inline void st16le(uint8_t* p, uint16_t v)
{
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}

enum { F_TOTLEN = 1, F_UDPLEN = 2, F_CSUM = 4, F_OPTS = 8, F_EMPTY = 16, F_SHORT = 32 };

static uint32_t frame_faults(const dqdk_synth_cfg_t* c, uint64_t rf)
{
    if (!(c->faulty & 1u))
        return 0;
    uint32_t f = 0;
    if ((rf & 0xff) == 0)
        f |= F_TOTLEN;
    if (((rf >> 8) & 0xff) == 1)
        f |= F_UDPLEN;
    if (((rf >> 16) & 0xff) == 2)
        f |= F_CSUM;
    if (((rf >> 24) & 0xff) == 3)
        f |= F_OPTS;
    if (((rf >> 32) & 0xff) == 4)
        f |= F_EMPTY;
    else if (((rf >> 40) & 0xff) == 5)
        f |= F_SHORT;
    return f;
}

uint32_t dqdk_synth_frame_len(const dqdk_synth_cfg_t* c, uint64_t g)
{
    uint64_t b = frame_base(c, g);
    uint64_t rf = rnd(b, 0);
    uint32_t f = frame_faults(c, rf);
    if (f & F_EMPTY)
        return 42;
    if (f & F_SHORT)
        return 40;
    if (c->frame_len)
        return c->frame_len;
    return (rnd(b, 1ull << 40) & 1) ? 9000u : 1500u; /* mixed 1500/9000 (config 4) */
}

/* pass 1: everything but the two checksum fields */
static void write_frame(const dqdk_synth_cfg_t* c, uint64_t g, uint8_t* f, uint32_t L)
{
    uint64_t b = frame_base(c, g);
    uint64_t rf = rnd(b, 0);
    uint32_t flt = frame_faults(c, rf);
    uint32_t ihl = (flt & F_OPTS) ? 6 : 5, hs = ihl * 4;
    uint32_t q = c->queue;
    static const uint8_t mac[12] = { 2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2 };
    uint32_t hdr_end = 14 + hs + 8;
    memcpy(f, mac, 12);
    f[12] = 0x08;
    f[13] = 0x00;
    uint8_t* ip = f + 14;
    ip[0] = (uint8_t)(0x40 | ihl);
    uint16_t tot = (uint16_t)(L - 14);
    if (flt & F_TOTLEN)
        tot = (uint16_t)(tot + 1 + ((rf >> 48) & 7));
    st16be(ip + 2, tot);
    st16be(ip + 4, (uint16_t)g);
    ip[8] = 64;
    ip[9] = 17;
    ip[12] = 192; ip[13] = 168; ip[14] = 10; ip[15] = 103; /* udp.c:76 */
    ip[16] = 192; ip[17] = 168; ip[18] = 10; ip[19] = 1;   /* udp.c:77 */
    if (ihl == 6)
        memset(ip + 20, 1, 4); /* IPOPT_NOP x4 */
    uint8_t* udp = ip + hs;
    st16be(udp + 0, (uint16_t)(5000 + q));
    st16be(udp + 2, 5000);
    uint16_t ulen = (uint16_t)(L - 14 - hs);
    if (flt & F_UDPLEN)
        ulen = (uint16_t)(ulen + 2);
    st16be(udp + 4, ulen);
    if (L <= hdr_end)
        return;
    uint8_t* pl = udp + 8;
    uint32_t E = (L - hdr_end) / 16;
    for (uint32_t e = 0; e < E; e++) {
        uint8_t* ev = pl + 16 * (size_t)e;
        uint64_t r = rnd(b, e + 1);
        uint64_t r2 = mix64(r);
        uint64_t seq = g * 4096u + e;
        uint32_t ch = (uint32_t)(((r & 0xffffffffull) * 1512u) >> 32);
        uint32_t energy = (uint32_t)((r >> 32) & 0xffffff);
        uint32_t hc = (uint32_t)((((r >> 56) & 0xff) * 6u) >> 8);
        if (c->faulty & 2u) {
            /* hot bins: (ch, hc, energy >> 8) */
            static const uint32_t hot[4][3] = { { 3, 1, 0x1234 }, { 3, 1, 0x1235 }, { 700, 4, 0xffff }, { 1511, 5, 0 } };
            const uint32_t pick = (uint32_t)(r2 >> 56) & 7u;
            if (pick < 3) {
                const uint32_t* h = hot[((r2 >> 52) & 3u)];
                ch = h[0];
                hc = h[1];
                energy = (h[2] << 8) | (energy & 0xffu);
            }
        }
        if (c->faulty & 1u) {
            if (((r2 >> 32) & 127) == 0)
                ch = 0xffffu - (uint32_t)((r2 >> 40) & 0xff);
            if (((r2 >> 39) & 127) == 1)
                hc = 6 + (uint32_t)((r2 >> 48) & 1);
        }
        st16le(ev + 0, (uint16_t)seq);
        st16le(ev + 2, (uint16_t)ch);
        ev[4] = (uint8_t)energy;
        ev[5] = (uint8_t)(energy >> 8);
        ev[6] = (uint8_t)(energy >> 16);
        ev[7] = (uint8_t)r2;                 /* trigger_flags */
        ev[8] = (uint8_t)(hc & 7);           /* hist_class:3, reserved:5 = 0 */
        ev[9] = (uint8_t)(r2 >> 8);          /* multiplicity */
        uint64_t ts = seq * 8u;              /* increasing 48-bit timestamp */
        for (int k = 0; k < 6; k++)
            ev[10 + k] = (uint8_t)(ts >> (8 * k));
    }
}

static inline uint16_t ld16le(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

/* Linux-style one's-complement helpers (same arithmetic as
 * src/tcpip/inet_csum.c:43-182) used to make the frames valid. */
static uint16_t fold16(uint64_t s)
{
    s = (s & 0xffffffffull) + (s >> 32);
    s = (s & 0xffffffffull) + (s >> 32);
    uint32_t x = (uint32_t)s;
    x = (x & 0xffff) + (x >> 16);
    x = (x & 0xffff) + (x >> 16);
    return (uint16_t)~x;
}

/* pass 2: IP header checksum and UDP checksum (reads the byte after an
 * odd-length datagram from the image, as the verifier does) */
static void write_checksums(const dqdk_synth_cfg_t* c, uint64_t g, uint8_t* f, uint32_t L, const uint8_t* img_end)
{
    uint64_t b = frame_base(c, g);
    uint64_t rf = rnd(b, 0);
    uint32_t flt = frame_faults(c, rf);
    uint32_t ihl = (flt & F_OPTS) ? 6 : 5, hs = ihl * 4;
    uint8_t* ip = f + 14;
    uint64_t s = 0;
    for (uint32_t k = 0; k < hs; k += 2)
        s += ld16le(ip + k);
    st16le(ip + 10, fold16(s));
    if (L < 14 + hs + 8)
        return;
    uint8_t* udp = ip + hs;
    uint32_t len = L - 14 - hs;
    uint64_t sum = 0;
    for (uint32_t k = 0; k + 1 < len; k += 2)
        sum += ld16le(udp + k);
    if (len & 1)
        sum += udp[len - 1] | ((udp + len < img_end ? udp[len] : 0) << 8);
    uint32_t saddr = (uint32_t)ip[12] | ((uint32_t)ip[13] << 8) | ((uint32_t)ip[14] << 16) | ((uint32_t)ip[15] << 24);
    uint32_t daddr = (uint32_t)ip[16] | ((uint32_t)ip[17] << 8) | ((uint32_t)ip[18] << 16) | ((uint32_t)ip[19] << 24);
    uint64_t t = (uint32_t)sum;
    t += saddr;
    t += daddr;
    t += (uint32_t)((17 + len) << 8);
    uint16_t ck = fold16(t);
    if (flt & F_CSUM)
        ck = (uint16_t)(ck ^ 0x5a5a) ? (uint16_t)(ck ^ 0x5a5a) : 0x5a5a;
    st16le(udp + 6, ck);
}

typedef struct {
    const dqdk_synth_cfg_t* c;
    uint64_t first;
    uint32_t lo, hi;
    uint8_t* umem;
    uint64_t umem_size;
    dqdk_gpu_desc_t* d;
    int pass;
} job_t;

static void* worker(void* p)
{
    job_t* j = (job_t*)p;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        uint64_t g = j->first + i;
        uint64_t addr = (uint64_t)i * j->c->stride;
        uint32_t L = dqdk_synth_frame_len(j->c, g);
        if (j->pass == 0) {
            j->d[i].addr = addr;
            j->d[i].len = L;
            j->d[i].options = 0;
            memset(j->umem + addr, 0, j->c->stride);
            write_frame(j->c, g, j->umem + addr, L);
        } else {
            write_checksums(j->c, g, j->umem + addr, L, j->umem + j->umem_size);
        }
    }
    return NULL;
}

uint64_t dqdk_synth_umem_size(const dqdk_synth_cfg_t* c, uint32_t n) { return (uint64_t)n * c->stride; }

int dqdk_synth_frames(const dqdk_synth_cfg_t* c, uint64_t first, uint32_t n, uint8_t* umem, uint64_t umem_size,
                      dqdk_gpu_desc_t* d, int threads)
{
    if (!c || !umem || !d || c->stride < 128 || (uint64_t)n * c->stride > umem_size)
        return -22;
    uint32_t maxL = c->frame_len ? c->frame_len : 9000u;
    if (maxL > c->stride)
        return -22;
    if (threads < 1)
        threads = 1;
    if (threads > 64)
        threads = 64;
    memset(umem + (uint64_t)n * c->stride, 0, umem_size - (uint64_t)n * c->stride);
    pthread_t tid[64];
    job_t jobs[64];
    uint32_t per = (n + (uint32_t)threads - 1) / (uint32_t)threads;
    for (int pass = 0; pass < 2; pass++) {
        for (int t = 0; t < threads; t++) {
            uint32_t lo = (uint32_t)t * per, hi = lo + per;
            if (lo > n)
                lo = n;
            if (hi > n)
                hi = n;
            jobs[t] = (job_t){ c, first, lo, hi, umem, umem_size, d, pass };
            pthread_create(&tid[t], NULL, worker, &jobs[t]);
        }
        for (int t = 0; t < threads; t++)
            pthread_join(tid[t], NULL);
    }
    return 0;
}
