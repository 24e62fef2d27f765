/*
 * rxqueues.c — host-UMEM throughput of Q independent RX queues, the way an AF_XDP deployment scales: one socket,
 * one UMEM and one RX loop thread per NIC queue (the reference's client binds one socket to one queue,
 * src/lib/xsk_utils.c:129-158, and runs handle_receive_packets() on it, src/lib/xsk_receive.c:192-237), here each
 * with its own xsk_gpu_ctx on the same GPU.  Every thread replays its UMEM of 4096 ICMP echo requests (one per 4 KiB
 * chunk at a 256-B headroom, BASELINE config 1's shape) in batches of B descriptors through xsk_gpu_process(); after
 * each pass over its UMEM it restores the request headers from a pristine copy (untimed) and checks that every call
 * of the pass answered every frame (TX_REPLY).
 *
 *   rxqueues <queues> <batch> <lowlat|zerocopy|staged> <seconds> [len=64]
 *
 * Prints one JSON line: aggregate Mframes/s (frames of all queues / the slowest queue's busy time), per-queue us per
 * call and the mode each context runs in (xsk_gpu_ctx_mode: LOWLAT requests beyond XSK_GPU_LOWLAT_PER_DEVICE run as
 * ZEROCOPY), verification.  Tool only (not the product): it builds its own frames and links only libxsknet_amd.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/xsk_gpu.h"

#define NFRAMES 4096u
#define CHUNK 4096u
#define HEADROOM 256u

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static uint16_t csum16(const uint8_t* p, size_t n) { /* RFC 1071 over network-order bytes */
    uint32_t s = 0;
    for (size_t i = 0; i + 1 < n; i += 2) s += (uint32_t)p[i] << 8 | p[i + 1];
    if (n & 1) s += (uint32_t)p[n - 1] << 8;
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)~s;
}

/* One ICMP echo request of `len` bytes (>= 42) at p: Ethernet / IPv4 (20 B) / ICMP, valid checksums. */
static void make_request(uint8_t* p, uint32_t len, uint32_t q, uint32_t i) {
    memset(p, 0, len);
    const uint8_t dst[6] = {0x02, 0, 0, 0, (uint8_t)q, 1}, src[6] = {0x02, 0, 0, 0, (uint8_t)q, 2};
    memcpy(p, dst, 6);
    memcpy(p + 6, src, 6);
    p[12] = 0x08;
    p[13] = 0x00;
    uint8_t* ip = p + 14;
    ip[0] = 0x45;
    ip[2] = (uint8_t)((len - 14) >> 8);
    ip[3] = (uint8_t)(len - 14);
    ip[4] = (uint8_t)(i >> 8);
    ip[5] = (uint8_t)i;
    ip[8] = 64;
    ip[9] = 1;
    ip[12] = 10, ip[13] = 0, ip[14] = (uint8_t)q, ip[15] = 2;
    ip[16] = 10, ip[17] = 0, ip[18] = (uint8_t)q, ip[19] = 1;
    const uint16_t ic = csum16(ip, 20);
    ip[10] = (uint8_t)(ic >> 8);
    ip[11] = (uint8_t)ic;
    uint8_t* icmp = p + 34;
    icmp[0] = 8;
    icmp[4] = 0x12, icmp[5] = 0x34;
    icmp[6] = (uint8_t)(i >> 8), icmp[7] = (uint8_t)i;
    for (uint32_t k = 42; k < len; k++) p[k] = (uint8_t)(k * 7 + i);
    const uint16_t cc = csum16(icmp, len - 34);
    icmp[2] = (uint8_t)(cc >> 8);
    icmp[3] = (uint8_t)cc;
}

struct queue {
    uint32_t q, batch, len;
    int mode;
    double seconds;
    xsk_gpu_ctx* ctx;
    uint8_t *umem, *pristine;
    struct xsk_gpu_desc descs[NFRAMES];
    /* results */
    double busy;
    uint64_t calls, frames, bad;
    int rc;
};

static pthread_barrier_t g_start;

static void* run_queue(void* arg) {
    struct queue* Q = (struct queue*)arg;
    uint8_t verd[XSK_GPU_LOWLAT_MAX];
    struct xsk_gpu_stats st;
    memset(&st, 0, sizeof st);
    /* warm-up pass: starts the device side (resident kernel / first launch) */
    for (uint32_t i0 = 0; i0 < NFRAMES && !Q->rc; i0 += Q->batch)
        Q->rc = xsk_gpu_process(Q->ctx, Q->descs + i0, Q->batch, verd, NULL, &st);
    memcpy(Q->umem, Q->pristine, (size_t)NFRAMES * CHUNK);
    pthread_barrier_wait(&g_start);
    const double t_end = now_s() + Q->seconds;
    while (!Q->rc && now_s() < t_end) {
        const double t0 = now_s();
        for (uint32_t i0 = 0; i0 < NFRAMES; i0 += Q->batch) {
            Q->rc = xsk_gpu_process(Q->ctx, Q->descs + i0, Q->batch, verd, NULL, &st);
            if (Q->rc) break;
            for (uint32_t k = 0; k < Q->batch; k++) Q->bad += verd[k] != XSK_GPU_TX_REPLY;
            Q->calls++;
            Q->frames += Q->batch;
        }
        Q->busy += now_s() - t0;
        for (uint32_t i = 0; i < NFRAMES; i++) /* untimed: the requests again */
            memcpy(Q->umem + (size_t)i * CHUNK + HEADROOM, Q->pristine + (size_t)i * CHUNK + HEADROOM, 64);
    }
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <queues> <batch> <lowlat|zerocopy|staged> <seconds> [len=64]\n", argv[0]);
        return 2;
    }
    const uint32_t nq = (uint32_t)atoi(argv[1]), batch = (uint32_t)atoi(argv[2]);
    const int mode = !strcmp(argv[3], "lowlat") ? XSK_GPU_MODE_LOWLAT
                     : !strcmp(argv[3], "staged") ? XSK_GPU_MODE_STAGED : XSK_GPU_MODE_ZEROCOPY;
    const double seconds = atof(argv[4]);
    uint32_t len = 64;
    for (int a = 5; a < argc; a++)
        if (!strncmp(argv[a], "len=", 4)) len = (uint32_t)atoi(argv[a] + 4);
    if (nq < 1 || nq > 16 || batch < 1 || batch > XSK_GPU_LOWLAT_MAX || NFRAMES % batch || len < 42 ||
        len > CHUNK - HEADROOM) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    struct queue* qs = (struct queue*)calloc(nq, sizeof *qs);
    pthread_t* th = (pthread_t*)calloc(nq, sizeof *th);
    if (!qs || !th) return 1;
    for (uint32_t q = 0; q < nq; q++) {
        struct queue* Q = &qs[q];
        Q->q = q;
        Q->batch = batch;
        Q->len = len;
        Q->mode = mode;
        Q->seconds = seconds;
        if (posix_memalign((void**)&Q->umem, 4096, (size_t)NFRAMES * CHUNK) ||
            posix_memalign((void**)&Q->pristine, 4096, (size_t)NFRAMES * CHUNK))
            return 1;
        memset(Q->pristine, 0, (size_t)NFRAMES * CHUNK);
        for (uint32_t i = 0; i < NFRAMES; i++) {
            make_request(Q->pristine + (size_t)i * CHUNK + HEADROOM, len, q, i);
            Q->descs[i].addr = (uint64_t)i * CHUNK + HEADROOM;
            Q->descs[i].len = len;
            Q->descs[i].options = 0;
        }
        memcpy(Q->umem, Q->pristine, (size_t)NFRAMES * CHUNK);
        const int rc = xsk_gpu_init(&Q->ctx, 0, Q->umem, (uint64_t)NFRAMES * CHUNK, batch, mode);
        if (rc) {
            fprintf(stderr, "xsk_gpu_init(queue %u): %d (%s)\n", q, rc, xsk_gpu_last_error());
            return 1;
        }
    }
    pthread_barrier_init(&g_start, NULL, nq);
    for (uint32_t q = 0; q < nq; q++) pthread_create(&th[q], NULL, run_queue, &qs[q]);
    for (uint32_t q = 0; q < nq; q++) pthread_join(th[q], NULL);
    double busy_max = 0;
    uint64_t frames = 0, bad = 0;
    int rc = 0;
    printf("{\"queues\": %u, \"batch\": %u, \"mode\": \"%s\", \"frame_len\": %u, \"per_queue_us_per_call\": [", nq, batch,
           argv[3], len);
    for (uint32_t q = 0; q < nq; q++) {
        const struct queue* Q = &qs[q];
        if (Q->busy > busy_max) busy_max = Q->busy;
        frames += Q->frames;
        bad += Q->bad;
        if (Q->rc && !rc) rc = Q->rc;
        printf("%s%.2f", q ? ", " : "", Q->calls ? Q->busy * 1e6 / (double)Q->calls : 0.0);
    }
    printf("], \"modes\": [");
    for (uint32_t q = 0; q < nq; q++) printf("%s%d", q ? ", " : "", xsk_gpu_ctx_mode(qs[q].ctx));
    printf("], \"mframes_s\": %.3f, \"frames\": %llu, \"not_replied\": %llu, \"rc\": %d}\n",
           busy_max > 0 ? (double)frames / busy_max / 1e6 : 0.0, (unsigned long long)frames, (unsigned long long)bad, rc);
    for (uint32_t q = 0; q < nq; q++) xsk_gpu_fini(qs[q].ctx);
    return rc || bad ? 1 : 0;
}
