/*
 * fetch_xsk_harness.c -- a C consumer of include/dqdk_gpu.h driving
 * libdqdk_gpu.so the two ways DQDK can (src/dqdk.c:252-322), with the AF_XDP
 * pieces DQDK wraps around the receive loop modelled in plain C (libxdp is
 * not in this image):
 *
 *   UMEM       one per worker, as umem_info_create makes it for each
 *              (src/dqdk.c:562, :57-72): mmap(MAP_HUGETLB when available,
 *              src/dqdk-mem.c:12-28) + mlock, the frames of an input image
 *              copied in (DQDK_HARNESS_SHARED_UMEM=1: one UMEM for every
 *              worker's queue, a layout the library also serves)
 *   RX ring    power-of-two descriptor ring with producer / consumer
 *              indices and a cached consumer (xsk_ring_cons__peek advances
 *              it, __release publishes it); a producer ("the NIC") refills
 *              it between batches, so batches wrap around the ring end
 *   fill ring  fq_ring_configure's one-time slot addresses
 *              (src/dqdk.c:109-127), reserved and submitted per batch
 *              without rewriting (src/dqdk.c:278-301)
 *
 * proc = batch: INTEGRATION.md's fetch_xsk patch -- the per-descriptor loop
 *   replaced by one dqdk_gpu_rx_batch over the UMEM registered once, the
 *   counter delta folded into the worker stats, batch abort from
 *   first_abort_idx.
 * proc = fp: fetch_xsk, process_frame and get_udp_payload as the reference
 *   has them (src/dqdk.c:185-207, :231-250, :252-322; ip4_audit / udp_audit
 *   src/tcpip/ipv4.c:13-20, udp.c:22-31), unpatched, with
 *   dqdk_gpu_frame_processor registered as the worker's frame_processor the
 *   way src/tristan.c:589-590 registers process_unbuffered_frame; at the end
 *   dqdk_gpu_fp_fini hands back tristan_t's totals, its histogram (host
 *   table) and the CSV.  `workers` threads each run the loop over the
 *   descriptor stream with their own rings and stats (one worker per RX
 *   queue, src/dqdk.c:491-515).
 *
 * Per batch: peek <= batch_size descriptors, rcvd_frames += rcvd (:289),
 * process them, and on a batch abort failing_batches++ with no release /
 * submit (:294-296, :317-321).  Each fetch_xsk call is timed (CLOCK_MONOTONIC).
 *
 * usage: fetch_xsk_harness <umem.bin | synth:N:LEN:STRIDE[:faulty]> <desc.bin | ->
 *                          <batch_size> <ring_size> <ring_start> <repeat>
 *                          <payloadsz> <mode> <flags> <csv_out | -> [batch|fp [workers [slot_payloads]]]
 * prints "name value" lines: worker stats, GPU counters, histogram bins, timing.
 * Test / measurement program only (tests/test_c_harness.py, tools/); not part
 * of the library.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "dqdk_gpu.h"

#define FRAME_SIZE 4096u /* XSK_UMEM__DEFAULT_FRAME_SIZE */
#define ETH_HLEN 14u

typedef struct {
    uint64_t rcvd_frames, rcvd_pkts, rcvd_bytes, invalid_ip_pkts, invalid_udp_pkts, failing_batches;
} stats_t; /* the dqdk_stats_t fields of this path (src/dqdk.h:52-68) */

typedef struct {
    dqdk_gpu_desc_t* ring;
    uint32_t size, mask;
    uint32_t producer;     /* written by "the NIC"          */
    uint32_t consumer;     /* published by release          */
    uint32_t cached_cons;  /* advanced by peek              */
} rx_ring_t;

typedef struct {
    uint64_t* addr;
    uint32_t size, mask, producer, cached_prod;
} fill_ring_t;

/* The dqdk_worker_t members the receive loop touches (src/dqdk.h:87-105);
 * the plugin sees only the pointer. */
struct dqdk_worker {
    stats_t stats;
    uint8_t debug_flags;
    int (*frame_processor)(struct dqdk_worker*, uint8_t*, uint32_t);
    uint8_t* umem;
    uint64_t umem_len;
    uint32_t batch_size;
    rx_ring_t rx;
    fill_ring_t fq;
    /* harness-only */
    int index;
    dqdk_gpu_queue_t* q; /* proc = batch */
    dqdk_gpu_desc_t* gdesc;
    dqdk_gpu_rx_result_t* gres;
    uint32_t flags;
    uint64_t batches, wrapped, fed, total;
    const dqdk_gpu_desc_t* descs;
    uint32_t ndesc;
    uint64_t* lat_ns; /* per fetch_xsk call */
    uint64_t nlat, caplat;
    int err;
};
typedef struct dqdk_worker dqdk_worker_t;

static uint64_t now_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

static uint32_t rx_peek(rx_ring_t* r, uint32_t nb, uint32_t* idx)
{
    uint32_t avail = r->producer - r->cached_cons;
    uint32_t n = avail < nb ? avail : nb;
    *idx = r->cached_cons;
    r->cached_cons += n;
    return n;
}

static void rx_release(rx_ring_t* r, uint32_t n) { r->consumer += n; }

/* ---- the reference's per-frame path, unpatched (src/dqdk.c:185-250) ------ */
static uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

static int ip4_audit(const uint8_t* iph, uint16_t actual_len) /* src/tcpip/ipv4.c:13-20 */
{
    return be16(iph + 2) == actual_len;
}

static int udp_audit(const uint8_t* udp, uint16_t udplen) /* src/tcpip/udp.c:22-31 (checksum commented out) */
{
    return be16(udp + 4) == udplen;
}

static uint8_t* get_udp_payload(dqdk_worker_t* xsk, uint8_t* buffer, uint32_t len, uint32_t* datalen)
{
    uint8_t* packet = buffer + ETH_HLEN;
    ++xsk->stats.rcvd_pkts;
    if (!ip4_audit(packet, (uint16_t)(len - ETH_HLEN))) {
        ++xsk->stats.invalid_ip_pkts;
        return NULL;
    }
    uint32_t iphdrsz = (uint32_t)(packet[0] & 0xf) * 4u; /* ip4_get_header_size, ipv4.h:9 */
    uint32_t udplen = (uint32_t)be16(packet + 2) - iphdrsz;
    uint8_t* udp = packet + iphdrsz;
    if (!udp_audit(udp, (uint16_t)udplen)) {
        xsk->stats.invalid_udp_pkts++;
        return NULL;
    }
    *datalen = udplen - 8u;
    return udp + 8;
}

static int process_frame(dqdk_worker_t* xsk, uint8_t* frame, uint32_t len)
{
    int ret = 0;
    uint32_t datalen = 0;
    uint8_t* data = get_udp_payload(xsk, frame, len, &datalen);
    if (datalen) {
        ret = xsk->frame_processor(xsk, data, datalen); /* (post_async when NULL: not this harness) */
        if (!ret)
            xsk->stats.rcvd_bytes += datalen;
    } else
        ret = -ENOBUFS;
    return ret;
}

/* one fetch_xsk call; returns 0 when the ring had nothing */
static int fetch_xsk(dqdk_worker_t* xsk, int fp)
{
    uint32_t idx = 0;
    const uint32_t rcvd = rx_peek(&xsk->rx, xsk->batch_size, &idx);
    if (!rcvd)
        return 0;
    /* xsk_ring_prod__reserve(fq, rcvd) (:278-287): slots only, no address writes */
    xsk->fq.cached_prod += rcvd;
    xsk->stats.rcvd_frames += rcvd; /* :289 */
    if ((idx & xsk->rx.mask) + rcvd > xsk->rx.size)
        xsk->wrapped++;
    xsk->batches++;
    int abort_batch = 0;
    if (fp) {
        for (uint32_t i = 0; i < rcvd; i++) { /* :291-298 */
            const dqdk_gpu_desc_t* desc = &xsk->rx.ring[idx++ & xsk->rx.mask];
            uint8_t* frame = xsk->umem + desc->addr;
            if (process_frame(xsk, frame, desc->len) < 0) {
                abort_batch = 1;
                break;
            }
        }
    } else {
        for (uint32_t i = 0; i < rcvd; i++) /* the RX ring wraps: gather the peeked descriptors */
            xsk->gdesc[i] = xsk->rx.ring[idx++ & xsk->rx.mask];
        dqdk_gpu_counters_t d;
        int rc = dqdk_gpu_rx_batch(xsk->q, xsk->umem, xsk->umem_len, xsk->gdesc, rcvd, xsk->gres, &d);
        if (rc < 0) {
            fprintf(stderr, "rx_batch: %d %s\n", rc, dqdk_gpu_last_error());
            xsk->err = rc;
            return -1;
        }
        xsk->stats.rcvd_pkts += d.rcvd_pkts;
        xsk->stats.invalid_ip_pkts += d.invalid_ip_pkts;
        xsk->stats.invalid_udp_pkts += d.invalid_udp_pkts;
        xsk->stats.rcvd_bytes += d.rcvd_bytes;
        /* batch-abort accounting (the reference's): process_frame() < 0 at
         * first_abort_idx (:294-296); per-packet accounting releases every batch */
        abort_batch = (xsk->flags & DQDK_GPU_F_BATCH_ABORT) && d.first_abort_idx < (uint64_t)rcvd;
    }
    if (abort_batch) {
        xsk->stats.failing_batches++; /* :317-319, no release / submit */
        /* the peeked slots stay unreleased; the consumer catches up so the
         * model ring can refill (the kernel side would eventually stall) */
        xsk->rx.consumer = xsk->rx.cached_cons;
        return 1;
    }
    rx_release(&xsk->rx, rcvd);            /* :300 */
    xsk->fq.producer = xsk->fq.cached_prod; /* :301 xsk_ring_prod__submit */
    return 1;
}

static int g_fp;

static void* worker_loop(void* arg)
{
    dqdk_worker_t* xsk = arg;
    while (xsk->fed < xsk->total || xsk->rx.producer != xsk->rx.cached_cons) {
        /* the NIC fills free ring slots with the next descriptors */
        while (xsk->fed < xsk->total && xsk->rx.producer - xsk->rx.consumer < xsk->rx.size &&
               xsk->rx.producer - xsk->rx.cached_cons < xsk->rx.size)
            xsk->rx.ring[xsk->rx.producer++ & xsk->rx.mask] = xsk->descs[xsk->fed++ % xsk->ndesc];
        const uint64_t t0 = now_ns();
        const int r = fetch_xsk(xsk, g_fp);
        if (r < 0)
            break;
        if (r > 0 && xsk->nlat < xsk->caplat)
            xsk->lat_ns[xsk->nlat++] = now_ns() - t0;
    }
    return NULL;
}

static void* read_file(const char* path, size_t* len)
{
    int fd = open(path, O_RDONLY);
    if (fd < 0)
        return NULL;
    struct stat st;
    fstat(fd, &st);
    void* p = malloc((size_t)st.st_size + 1);
    size_t got = 0;
    while (got < (size_t)st.st_size) {
        ssize_t r = read(fd, (char*)p + got, (size_t)st.st_size - got);
        if (r <= 0)
            break;
        got += (size_t)r;
    }
    close(fd);
    *len = got;
    return p;
}

/* a UMEM: hugepage mapping when the host has them, else 4-KiB pages; mlock'ed */
static uint8_t* map_umem(size_t size, const uint8_t* image, size_t len, int* hugetlb, int* locked)
{
    *hugetlb = 1;
    uint8_t* u = mmap(NULL, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_HUGETLB, -1, 0);
    if (u == MAP_FAILED) {
        *hugetlb = 0;
        u = mmap(NULL, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    }
    if (u == MAP_FAILED)
        return NULL;
    *locked = mlock(u, size) == 0;
    memcpy(u, image, len);
    return u;
}

static int cmp_u64(const void* a, const void* b)
{
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char** argv)
{
    if (argc < 11 || argc > 14) {
        fprintf(stderr,
                "usage: %s umem.bin|synth:N:LEN:STRIDE[:faulty] desc.bin|- batch ring_size ring_start repeat "
                "payloadsz mode flags csv|- [batch|fp [workers [slot_payloads]]]\n",
                argv[0]);
        return 2;
    }
    const int fp = argc > 11 && !strcmp(argv[11], "fp");
    const int nworkers = argc > 12 ? atoi(argv[12]) : 1;
    const uint32_t slot_payloads = argc > 13 ? (uint32_t)atoi(argv[13]) : 0;
    g_fp = fp;
    size_t umem_len = 0, desc_len = 0;
    uint8_t* image = NULL;
    dqdk_gpu_desc_t* descs = NULL;
    if (!strncmp(argv[1], "synth:", 6)) { /* synthetic frames (dqdk_synth_frames) */
        unsigned n = 0, flen = 0, stride = 0, faulty = 0;
        if (sscanf(argv[1] + 6, "%u:%u:%u:%u", &n, &flen, &stride, &faulty) < 3 || !n) {
            fprintf(stderr, "bad synth spec\n");
            return 2;
        }
        dqdk_synth_cfg_t sc = { .seed = 20261015u, .queue = 0, .frame_len = flen, .stride = stride, .faulty = faulty };
        umem_len = (size_t)((dqdk_synth_umem_size(&sc, n) + 15) / 16 * 16);
        image = calloc(1, umem_len);
        descs = calloc(n, sizeof(*descs));
        if (!image || !descs || dqdk_synth_frames(&sc, 0, n, image, umem_len, descs, 8) != 0) {
            fprintf(stderr, "synth failed\n");
            return 1;
        }
        desc_len = (size_t)n * sizeof(*descs);
    } else {
        image = read_file(argv[1], &umem_len);
        descs = read_file(argv[2], &desc_len);
    }
    const uint32_t batch = (uint32_t)atoi(argv[3]);
    const uint32_t ring_size = (uint32_t)atoi(argv[4]);
    const uint32_t ring_start = (uint32_t)atoi(argv[5]);
    const uint32_t repeat = (uint32_t)atoi(argv[6]);
    if (!image || !descs || !batch || !ring_size || (ring_size & (ring_size - 1)) || nworkers < 1 || nworkers > 16) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    const uint32_t ndesc = (uint32_t)(desc_len / sizeof(dqdk_gpu_desc_t));

    /* UMEMs: one per worker (src/dqdk.c:562), or one shared */
    const size_t huge = 2u << 20;
    const size_t size = (umem_len + huge - 1) / huge * huge;
    const char* sh = getenv("DQDK_HARNESS_SHARED_UMEM");
    const int shared = sh && atoi(sh) != 0;
    const int numem = shared ? 1 : nworkers;
    uint8_t** umems = calloc((size_t)numem, sizeof(uint8_t*));
    int hugetlb = 1, locked = 1;
    for (int k = 0; k < numem; k++) {
        int h = 0, l = 0;
        if (!(umems[k] = map_umem(size, image, umem_len, &h, &l))) {
            perror("mmap");
            return 1;
        }
        hugetlb &= h;
        locked &= l;
    }
    free(image);
    printf("umem_hugetlb %d\numem_mlocked %d\numem_count %d\n", hugetlb, locked, numem);

    dqdk_gpu_cfg_t cfg = { .payloadsz = (uint32_t)atoi(argv[7]), .mode = (uint32_t)atoi(argv[8]),
                           .flags = (uint32_t)strtoul(argv[9], NULL, 0) };
    int rc = 0;
    if (fp) { /* tristan.c:589-590: proc = process_unbuffered_frame -> the GPU plugin */
        dqdk_gpu_fp_cfg_t fc = { .cfg = cfg, .slot_payloads = slot_payloads };
        if ((rc = dqdk_gpu_fp_init(&fc)) != 0) {
            fprintf(stderr, "fp_init: %d %s\n", rc, dqdk_gpu_last_error());
            return 1;
        }
    }

    dqdk_worker_t* w = calloc((size_t)nworkers, sizeof(*w));
    const uint64_t total = (uint64_t)ndesc * repeat;
    for (int k = 0; k < nworkers; k++) {
        dqdk_worker_t* x = &w[k];
        uint8_t* const umem = umems[shared ? 0 : k];
        x->index = k;
        x->umem = umem;
        x->umem_len = umem_len;
        x->batch_size = batch;
        x->flags = cfg.flags;
        x->descs = descs;
        x->ndesc = ndesc;
        x->total = total;
        x->rx = (rx_ring_t){ calloc(ring_size, sizeof(dqdk_gpu_desc_t)), ring_size, ring_size - 1, ring_start,
                             ring_start, ring_start };
        x->fq = (fill_ring_t){ calloc(ring_size, sizeof(uint64_t)), ring_size, ring_size - 1, 0, 0 };
        for (uint32_t i = 0; i < ring_size; i++) /* fq_ring_configure: fixed addresses, never rewritten */
            x->fq.addr[i] = (uint64_t)i * FRAME_SIZE;
        x->caplat = total / batch + 16;
        x->lat_ns = calloc(x->caplat, sizeof(uint64_t));
        if (fp) {
            x->frame_processor = dqdk_gpu_frame_processor;
            /* optional: the worker's GPU and UMEM before its first frame (dqdk_worker_init's place) */
            if ((rc = dqdk_gpu_fp_bind(x, -1, umem, umem_len)) != 0) {
                fprintf(stderr, "fp_bind: %d %s\n", rc, dqdk_gpu_last_error());
                return 1;
            }
        } else {
            if ((rc = dqdk_gpu_queue_create(k % dqdk_gpu_device_count(), &cfg, batch, &x->q)) != 0) {
                fprintf(stderr, "queue_create: %d %s\n", rc, dqdk_gpu_last_error());
                return 1;
            }
            if ((rc = dqdk_gpu_umem_register(x->q, umem, size)) != 0) {
                fprintf(stderr, "umem_register: %d %s\n", rc, dqdk_gpu_last_error());
                return 1;
            }
            x->gdesc = calloc(batch, sizeof(*x->gdesc));
            x->gres = calloc(batch, sizeof(*x->gres));
        }
    }

    pthread_t* th = calloc((size_t)nworkers, sizeof(pthread_t));
    const uint64_t t0 = now_ns();
    for (int k = 0; k < nworkers; k++)
        pthread_create(&th[k], NULL, worker_loop, &w[k]);
    for (int k = 0; k < nworkers; k++)
        pthread_join(th[k], NULL);
    const uint64_t t_loop = now_ns() - t0;
    for (int k = 0; k < nworkers; k++)
        if (w[k].err)
            return 1;

    /* fini: tristan_fini's inputs (src/tristan.c:163-231) */
    const uint64_t tf0 = now_ns();
    const int want_csv = strcmp(argv[10], "-") != 0;
    int fd = want_csv ? open(argv[10], O_WRONLY | O_CREAT | O_TRUNC, 0644) : -1;
    if (want_csv && fd < 0) {
        perror("open csv");
        return 1;
    }
    dqdk_gpu_counters_t c;
    memset(&c, 0, sizeof(c));
    uint64_t nz = 0, csv_bytes = 0;
    if (fp) {
        /* tristan_t::histo (host) += the GPU tables; the CSV straight from the GPU */
        uint32_t* host_hist = want_csv ? calloc(DQDK_TRISTAN_HISTO_ENTRIES, sizeof(uint32_t)) : NULL;
        if (want_csv && !host_hist) {
            fprintf(stderr, "no memory for the host table\n");
            return 1;
        }
        if ((rc = dqdk_gpu_fp_fini(host_hist, fd, &c)) != 0) {
            fprintf(stderr, "fp_fini: %d %s\n", rc, dqdk_gpu_last_error());
            return 1;
        }
        if (host_hist)
            for (uint64_t i = 0; i < DQDK_TRISTAN_HISTO_ENTRIES; i++)
                nz += host_hist[i] != 0;
        free(host_hist);
        if (fd >= 0)
            csv_bytes = (uint64_t)lseek(fd, 0, SEEK_CUR);
    } else {
        /* per-queue partials summed (one queue per worker; merged on GPU 0 when all share it) */
        for (int k = 0; k < nworkers; k++) {
            dqdk_gpu_counters_t ck;
            dqdk_gpu_counters_get(w[k].q, &ck);
            c.total_events += ck.total_events;
            c.total_bytes += ck.total_bytes;
            c.oob_events += ck.oob_events;
            c.empty_pkts += ck.empty_pkts;
        }
        if (want_csv) {
            if (nworkers != 1) {
                fprintf(stderr, "batch mode writes the CSV of one worker only\n");
                return 2;
            }
            dqdk_gpu_histogram_nonzero(w[0].q, &nz);
            if (dqdk_gpu_histogram_write_csv(w[0].q, fd, &csv_bytes) != 0) {
                fprintf(stderr, "write_csv: %s\n", dqdk_gpu_last_error());
                return 1;
            }
        }
    }
    if (fd >= 0)
        close(fd);
    const uint64_t t_fini = now_ns() - tf0;

    stats_t s;
    memset(&s, 0, sizeof(s));
    uint64_t batches = 0, wrapped = 0, fill = 0, nlat = 0;
    for (int k = 0; k < nworkers; k++) {
        s.rcvd_frames += w[k].stats.rcvd_frames;
        s.rcvd_pkts += w[k].stats.rcvd_pkts;
        s.rcvd_bytes += w[k].stats.rcvd_bytes;
        s.invalid_ip_pkts += w[k].stats.invalid_ip_pkts;
        s.invalid_udp_pkts += w[k].stats.invalid_udp_pkts;
        s.failing_batches += w[k].stats.failing_batches;
        batches += w[k].batches;
        wrapped += w[k].wrapped;
        fill += w[k].fq.producer;
        nlat += w[k].nlat;
    }
    uint64_t* lat = calloc(nlat + 1, sizeof(uint64_t));
    for (int k = 0, o = 0; k < nworkers; k++) {
        memcpy(lat + o, w[k].lat_ns, w[k].nlat * sizeof(uint64_t));
        o += (int)w[k].nlat;
    }
    qsort(lat, nlat, sizeof(uint64_t), cmp_u64);
    printf("batches %" PRIu64 "\nwrapped_batches %" PRIu64 "\nfill_submitted %" PRIu64 "\n", batches, wrapped, fill);
    printf("rcvd_frames %" PRIu64 "\nrcvd_pkts %" PRIu64 "\nrcvd_bytes %" PRIu64 "\ninvalid_ip_pkts %" PRIu64
           "\ninvalid_udp_pkts %" PRIu64 "\nfailing_batches %" PRIu64 "\n",
           s.rcvd_frames, s.rcvd_pkts, s.rcvd_bytes, s.invalid_ip_pkts, s.invalid_udp_pkts, s.failing_batches);
    printf("total_events %" PRIu64 "\ntotal_bytes %" PRIu64 "\noob_events %" PRIu64 "\nempty_pkts %" PRIu64
           "\nhisto_nonzero %" PRIu64 "\ncsv_bytes %" PRIu64 "\n",
           c.total_events, c.total_bytes, c.oob_events, c.empty_pkts, nz, csv_bytes);
    if (fp)
        printf("fp_calls %" PRIu64 "\n", c.rcvd_pkts);
    /* timing: the receive loop (all workers, wall clock) and each fetch_xsk call */
    printf("workers %d\nloop_ns %" PRIu64 "\nfini_ns %" PRIu64 "\n", nworkers, t_loop, t_fini);
    if (nlat) {
        printf("fetch_p50_ns %" PRIu64 "\nfetch_p99_ns %" PRIu64 "\nfetch_max_ns %" PRIu64 "\n", lat[nlat / 2],
               lat[(nlat * 99) / 100], lat[nlat - 1]);
    }
    free(lat);
    int bad = 0;
    for (int k = 0; k < nworkers; k++) {
        if (!fp) {
            /* a UMEM is unregistered before it is freed (include/dqdk_gpu.h) */
            if (dqdk_gpu_umem_unregister(w[k].q, w[k].umem) || dqdk_gpu_queue_destroy(w[k].q)) {
                fprintf(stderr, "teardown: %s\n", dqdk_gpu_last_error());
                bad = 1;
            }
        }
    }
    for (int k = 0; k < numem; k++) {
        munlock(umems[k], size);
        munmap(umems[k], size);
    }
    free(umems);
    return bad;
}
