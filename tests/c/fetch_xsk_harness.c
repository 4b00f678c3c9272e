/*
 * fetch_xsk_harness.c -- a C consumer of include/dqdk_gpu.h running the
 * INTEGRATION.md fetch_xsk patch shape (src/dqdk.c:252-322) against
 * libdqdk_gpu.so, with the AF_XDP pieces DQDK wraps around the loop modelled
 * in plain C (libxdp is not in this image):
 *
 *   UMEM       mmap(MAP_HUGETLB when available, src/dqdk-mem.c:12-28) +
 *              mlock, the frames of an input image copied in, registered
 *              with the GPU once (dqdk_gpu_umem_register)
 *   RX ring    power-of-two descriptor ring with producer / consumer
 *              indices and a cached consumer (xsk_ring_cons__peek advances
 *              it, __release publishes it); a producer ("the NIC") refills
 *              it between batches, so batches wrap around the ring end
 *   fill ring  fq_ring_configure's one-time slot addresses
 *              (src/dqdk.c:109-127), reserved and submitted per batch
 *              without rewriting (src/dqdk.c:278-301)
 *
 * Per batch: peek <= batch_size descriptors, rcvd_frames += rcvd (:289),
 * gather the (wrapping) descriptors, dqdk_gpu_rx_batch, fold the counter
 * delta into the worker stats, and on a batch abort (first_abort_idx <
 * rcvd) failing_batches++ with no release / submit (:294-296, :317-321).
 *
 * usage: fetch_xsk_harness <umem.bin> <desc.bin> <batch_size> <ring_size>
 *                          <ring_start> <repeat> <payloadsz> <mode> <flags>
 *                          <csv_out>
 * prints "name value" lines: worker stats, GPU counters, histogram bins.
 * Test program only (tests/test_c_harness.py); not part of the library.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "dqdk_gpu.h"

#define FRAME_SIZE 4096u /* XSK_UMEM__DEFAULT_FRAME_SIZE */

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

static uint32_t rx_peek(rx_ring_t* r, uint32_t nb, uint32_t* idx)
{
    uint32_t avail = r->producer - r->cached_cons;
    uint32_t n = avail < nb ? avail : nb;
    *idx = r->cached_cons;
    r->cached_cons += n;
    return n;
}

static void rx_release(rx_ring_t* r, uint32_t n) { r->consumer += n; }

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

int main(int argc, char** argv)
{
    if (argc != 11) {
        fprintf(stderr, "usage: %s umem.bin desc.bin batch ring_size ring_start repeat payloadsz mode flags csv\n",
                argv[0]);
        return 2;
    }
    size_t umem_len = 0, desc_len = 0;
    uint8_t* image = read_file(argv[1], &umem_len);
    dqdk_gpu_desc_t* descs = read_file(argv[2], &desc_len);
    const uint32_t batch = (uint32_t)atoi(argv[3]);
    const uint32_t ring_size = (uint32_t)atoi(argv[4]);
    const uint32_t ring_start = (uint32_t)atoi(argv[5]);
    const uint32_t repeat = (uint32_t)atoi(argv[6]);
    if (!image || !descs || !batch || !ring_size || (ring_size & (ring_size - 1))) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    const uint32_t ndesc = (uint32_t)(desc_len / sizeof(dqdk_gpu_desc_t));

    /* UMEM: hugepage mapping when the host has them, else 4-KiB pages; mlock'ed */
    const size_t huge = 2u << 20;
    const size_t size = (umem_len + huge - 1) / huge * huge;
    int hugetlb = 1;
    uint8_t* umem = mmap(NULL, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_HUGETLB, -1, 0);
    if (umem == MAP_FAILED) {
        hugetlb = 0;
        umem = mmap(NULL, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    }
    if (umem == MAP_FAILED) {
        perror("mmap");
        return 1;
    }
    const int locked = mlock(umem, size) == 0;
    memcpy(umem, image, umem_len);
    printf("umem_hugetlb %d\numem_mlocked %d\n", hugetlb, locked);

    dqdk_gpu_cfg_t cfg = { .payloadsz = (uint32_t)atoi(argv[7]), .mode = (uint32_t)atoi(argv[8]),
                           .flags = (uint32_t)strtoul(argv[9], NULL, 0) };
    dqdk_gpu_queue_t* q = NULL;
    int rc = dqdk_gpu_queue_create(0, &cfg, batch, &q);
    if (rc) {
        fprintf(stderr, "queue_create: %d %s\n", rc, dqdk_gpu_last_error());
        return 1;
    }
    if ((rc = dqdk_gpu_umem_register(q, umem, size)) != 0) {
        fprintf(stderr, "umem_register: %d %s\n", rc, dqdk_gpu_last_error());
        return 1;
    }

    rx_ring_t rx = { calloc(ring_size, sizeof(dqdk_gpu_desc_t)), ring_size, ring_size - 1, ring_start, ring_start,
                     ring_start };
    fill_ring_t fq = { calloc(ring_size, sizeof(uint64_t)), ring_size, ring_size - 1, 0, 0 };
    for (uint32_t i = 0; i < ring_size; i++) /* fq_ring_configure: fixed addresses, never rewritten */
        fq.addr[i] = (uint64_t)i * FRAME_SIZE;
    dqdk_gpu_desc_t* gdesc = calloc(batch, sizeof(*gdesc));
    dqdk_gpu_rx_result_t* gres = calloc(batch, sizeof(*gres));

    stats_t stats = { 0 };
    uint64_t fed = 0, batches = 0, wrapped = 0;
    const uint64_t total = (uint64_t)ndesc * repeat;
    while (fed < total || rx.producer != rx.cached_cons) {
        /* the NIC fills free ring slots with the next descriptors */
        while (fed < total && rx.producer - rx.consumer < rx.size && rx.producer - rx.cached_cons < rx.size)
            rx.ring[rx.producer++ & rx.mask] = descs[fed++ % ndesc];
        uint32_t idx = 0;
        const uint32_t rcvd = rx_peek(&rx, batch, &idx);
        if (!rcvd)
            continue;
        /* xsk_ring_prod__reserve(fq, rcvd) (:278-287): slots only, no address writes */
        fq.cached_prod += rcvd;
        stats.rcvd_frames += rcvd; /* :289 */
        if ((idx & rx.mask) + rcvd > rx.size)
            wrapped++;
        for (uint32_t i = 0; i < rcvd; i++) /* the RX ring wraps: gather the peeked descriptors */
            gdesc[i] = rx.ring[idx++ & rx.mask];
        dqdk_gpu_counters_t d;
        rc = dqdk_gpu_rx_batch(q, umem, umem_len, gdesc, rcvd, gres, &d);
        if (rc < 0) {
            fprintf(stderr, "rx_batch: %d %s\n", rc, dqdk_gpu_last_error());
            return 1;
        }
        stats.rcvd_pkts += d.rcvd_pkts;
        stats.invalid_ip_pkts += d.invalid_ip_pkts;
        stats.invalid_udp_pkts += d.invalid_udp_pkts;
        stats.rcvd_bytes += d.rcvd_bytes;
        batches++;
        /* batch-abort accounting (the reference's): process_frame() < 0 at
         * first_abort_idx (:294-296); per-packet accounting releases every batch */
        if ((cfg.flags & DQDK_GPU_F_BATCH_ABORT) && d.first_abort_idx < (uint64_t)rcvd) {
            stats.failing_batches++;              /* :317-319, no release / submit */
            /* the peeked slots stay unreleased; the consumer catches up so the
             * model ring can refill (the kernel side would eventually stall) */
            rx.consumer = rx.cached_cons;
            continue;
        }
        rx_release(&rx, rcvd);        /* :300 */
        fq.producer = fq.cached_prod; /* :301 xsk_ring_prod__submit */
    }

    dqdk_gpu_counters_t c;
    dqdk_gpu_counters_get(q, &c);
    uint64_t nz = 0;
    dqdk_gpu_histogram_nonzero(q, &nz);
    int fd = open(argv[10], O_WRONLY | O_CREAT | O_TRUNC, 0644);
    uint64_t csv_bytes = 0;
    if (fd < 0 || dqdk_gpu_histogram_write_csv(q, fd, &csv_bytes) != 0) {
        fprintf(stderr, "write_csv: %s\n", dqdk_gpu_last_error());
        return 1;
    }
    close(fd);
    printf("batches %" PRIu64 "\nwrapped_batches %" PRIu64 "\nfill_submitted %" PRIu32 "\n", batches, wrapped,
           fq.producer);
    printf("rcvd_frames %" PRIu64 "\nrcvd_pkts %" PRIu64 "\nrcvd_bytes %" PRIu64 "\ninvalid_ip_pkts %" PRIu64
           "\ninvalid_udp_pkts %" PRIu64 "\nfailing_batches %" PRIu64 "\n",
           stats.rcvd_frames, stats.rcvd_pkts, stats.rcvd_bytes, stats.invalid_ip_pkts, stats.invalid_udp_pkts,
           stats.failing_batches);
    printf("total_events %" PRIu64 "\ntotal_bytes %" PRIu64 "\noob_events %" PRIu64 "\nempty_pkts %" PRIu64
           "\nhisto_nonzero %" PRIu64 "\ncsv_bytes %" PRIu64 "\n",
           c.total_events, c.total_bytes, c.oob_events, c.empty_pkts, nz, csv_bytes);
    dqdk_gpu_umem_unregister(q, umem);
    dqdk_gpu_queue_destroy(q);
    munlock(umem, size);
    munmap(umem, size);
    return 0;
}
