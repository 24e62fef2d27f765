/*
 * rxring.c — RX-loop throughput per queue under a saturated RX ring: xsk_gpu_rx_step() against
 * a simulated kernel side of the AF_XDP rings, the loop of the reference's client (src/lib/xsk_receive.c:192-237 with
 * complete_tx() :77-99) with the transform on the GPU.
 *
 * Per queue (one UMEM, one context or pipelined loop, its four rings):
 *   - the simulated NIC, in a thread of its own like the hardware it stands for (nic=thread, the default): takes every
 *     TX descriptor, checks the frame is the exact echo reply of the request it delivered there (the header of every
 *     reply, every byte of every 16th), and posts its address on the completion ring; then receives a request into
 *     every frame the fill ring hands it (the chunk base + the 256-B XDP headroom, as the kernel does in aligned-chunk
 *     mode) until the RX ring is full -- the ring stays saturated.  nic=inline runs it between the steps on the
 *     application's thread, untimed (rounds 4-5's first method: it also hides GPU work a pipelined loop overlaps with it,
 *     so it is not used for pipe=D);
 *   - the application loop, on the queue's thread: xsk_gpu_tx_complete() (complete_tx minus the kick) and one
 *     xsk_gpu_rx_step() (or xsk_gpu_rx_pipe_step()) of up to <step> descriptors.  Throughput = frames / the loop's wall
 *     time (nic=thread) or / the summed step time (nic=inline).
 * huge=1: the UMEM from xsk_gpu_umem_alloc (transparent huge pages) instead of posix_memalign's 4 KiB pages.
 * nic=burst measures the application and the GPU alone: untimed, the NIC fills the RX ring with every frame (ring =
 * frames); timed, the application's steps until each of them is completed (replies on the TX ring); repeat.  One NIC
 * thread that touches every frame caps nic=thread at a few tens of Mframes/s, below a pipelined loop.
 * A step takes min(ring occupancy, step, XSK_GPU_RX_MAX_STEP) frames; the reference's RX_BATCH_SIZE (64,
 * src/lib/xsk_utils.h:8) is a constant of its CPU loop and changes no frame's result.
 *
 *   rxring <step> <lowlat|zerocopy|staged> <seconds> [len=64] [queues=1] [ring=4096] [frames=4096] [empty=0] [pipe=0] [nic=thread|inline|burst] [huge=0] [groups=0]
 *
 * groups=G: LOWLAT batches served by G workgroups (xsk_gpu__lowlat_tune; 0 = by size).  The line's `where` lists the
 * first failures of queue 0 as runs of consecutive slots of one step (step index, slot range, kind: 0 handed back
 * holding the request, 2 other bytes, 3 a transmitted reply that differs).
 *
 * pipe=D (1..XSK_GPU_RX_PIPE_MAX): the pipelined loop instead -- xsk_gpu_rx_pipe_step() with up to D batches in flight
 * (one context each), a flush at the end; frames count when their batch completes.
 * empty=1: the empty-ring latency instead -- the NIC delivers exactly <step> frames, the step serves them, repeat
 * (each call finds exactly its batch: the RX-loop latency of tools/hostlat.py, through the ring loop).
 * Prints one JSON line: Mframes/s per queue and in total (frames / the timed application time), us per step (mean,
 * p50, p99), frames checked, and the frames not answered by cause:
 *   tx_full      replies the step produced but dropped because the TX ring was full (xsk_receive.c:178-181's path;
 *                the NIC thread had not taken the earlier ones yet) -- not a wrong result;
 *   not_replied  frames handed back with a verdict other than TX_REPLY: every frame is an echo request, so a wrong
 *                verdict;
 *   wrong_reply  transmitted replies whose bytes differ from the exact echo reply (or whose length does);
 *   counters     1 if the step counters disagree with the frames completed (tx_packets must equal the replies sent);
 * failures = not_replied + wrong_reply + counters (the correctness failures only).  A dropped frame's header, read when
 * it comes back on the fill ring, is also sorted into request / reply / other (dropped_req_rep_other): a TX-full drop
 * holds the reply, a wrong verdict the request.  Tool only: it builds its own frames and links only libxsknet_amd.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>

#include "../include/xsk_gpu.h"

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

/* An ICMP echo request of `len` (>= 42) bytes, valid checksums, and its reply as the reference writes it
 * (xsk_receive.c:148-157: MACs and IPv4 addresses swapped, type 0, checksum by csum_replace2). */
static void make_pair(uint8_t* req, uint8_t* rep, uint32_t len, uint32_t q) {
    memset(req, 0, len);
    const uint8_t dst[6] = {0x02, 0, 0, 0, (uint8_t)q, 1}, src[6] = {0x02, 0, 0, 0, (uint8_t)q, 2};
    memcpy(req, dst, 6);
    memcpy(req + 6, src, 6);
    req[12] = 0x08;
    uint8_t* ip = req + 14;
    ip[0] = 0x45;
    ip[2] = (uint8_t)((len - 14) >> 8);
    ip[3] = (uint8_t)(len - 14);
    ip[8] = 64;
    ip[9] = 1;
    ip[12] = 10, ip[14] = (uint8_t)q, ip[15] = 2;
    ip[16] = 10, ip[18] = (uint8_t)q, ip[19] = 1;
    const uint16_t ic = csum16(ip, 20);
    ip[10] = (uint8_t)(ic >> 8), ip[11] = (uint8_t)ic;
    uint8_t* icmp = req + 34;
    icmp[0] = 8;
    for (uint32_t i = 8; i < len - 34; i++) icmp[i] = (uint8_t)(i * 7u + q);
    const uint16_t cc = csum16(icmp, len - 34);
    icmp[2] = (uint8_t)(cc >> 8), icmp[3] = (uint8_t)cc;
    memcpy(rep, req, len);
    memcpy(rep, src, 6);
    memcpy(rep + 6, dst, 6);
    memcpy(rep + 26, ip + 16, 4);
    memcpy(rep + 30, ip + 12, 4);
    rep[34] = 0;
    /* csum_replace2(&csum, 8, 0) on the little-endian-loaded field (xsk_receive.c:101-111) */
    uint32_t c = (uint32_t)req[36] | (uint32_t)req[37] << 8;
    c = (~c) & 0xFFFFu;
    c += (~8u) & 0xFFFFu;
    c = (c & 0xFFFFu) + (c >> 16);
    c = (~c) & 0xFFFFu;
    rep[36] = (uint8_t)c, rep[37] = (uint8_t)(c >> 8);
}

struct ring_mem { /* one ring: producer, consumer, flags words and the entries */
    uint32_t prod, cons, flags;
    void* ents;
};

static void ring_init(struct xsk_gpu_ring* r, struct ring_mem* m, uint32_t size, size_t esz, int producer_side) {
    memset(m, 0, sizeof *m);
    m->ents = calloc(size, esz);
    memset(r, 0, sizeof *r);
    r->mask = size - 1;
    r->size = size;
    r->producer = &m->prod;
    r->consumer = &m->cons;
    r->flags = &m->flags;
    r->ring = m->ents;
    if (producer_side) r->cached_cons = size; /* libxdp: a producer's cached consumer is consumer + size */
}

xsk_gpu_ctx* xsk_gpu__rx_pipe_ctx(xsk_gpu_rx_pipe* p, uint32_t i); /* (library hook: a pipe's context) */
int xsk_gpu__lowlat_tune(xsk_gpu_ctx* c, uint32_t tile_frames, uint32_t groups, uint32_t timeout_us); /* (hook) */
int xsk_gpu__lowlat_outcomes(const xsk_gpu_ctx* c, uint64_t out[4]); /* (library hook: LOWLAT call outcomes) */

struct queue {
    uint32_t q, step, len, ring, frames, empty, pipe, nic_thread, huge, groups;
    int mode, real_mode;
    double seconds;
    /* results */
    uint64_t frames_done, steps, checked, fail;
    uint64_t tx_full, not_replied, wrong_reply, counters; /* the unanswered frames by cause (fail = the last three) */
    uint64_t dropped[3]; /* frames handed back without a reply: header still the request / the reply / other */
    uint64_t outcomes[4]; /* LOWLAT batches past their timeout: all, completed partly served, failed, late (xsk_gpu__lowlat_outcomes) */
    double busy, wall;
    double* lat;
    uint64_t nlat;
    int rc;
    /* failure locations: each step's first RX sequence number and size, and the first failures' sequence numbers */
    uint64_t* step_seq;
    uint32_t* step_n;
    uint64_t nsteps_logged;
    uint64_t fail_seq[4096];
    uint8_t fail_kind[4096]; /* 0 handed back holding the request, 1 holding the reply, 2 other, 3 wrong reply on TX */
    uint32_t nfail_logged;
};

static int cmpd(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

/* The simulated NIC / kernel side of one queue: its own cursors over the shared index words. */
struct nic {
    struct queue* Q;
    uint8_t* umem;
    const uint8_t *req, *rep;
    struct ring_mem *mrx, *mfill, *mtx, *mcomp;
    uint32_t R, len, k_rx_prod, k_fill_cons, k_tx_cons, k_comp_prod;
    uint8_t* primed; /* per chunk: the full request was written once (later only its header is restored) */
    uint8_t* out;    /* per chunk: delivered on RX and not yet seen on TX */
    uint64_t* dseq;  /* per chunk: the RX sequence number of its last delivery */
    volatile int stop;
    uint64_t checked, fail;  /* fail: transmitted replies of the wrong length or bytes */
};

/* One pass: every reply on the TX ring completed, its frame checked against the exact echo reply of the request
 * delivered there (the header of every 4th reply, every byte of every 64th: the checks touch the frames, and a NIC
 * thread that touched every byte of every frame would be the bottleneck it stands in for); then a request received
 * into each frame the fill ring offers while the RX ring has room.  The transform rewrites only the header (bytes below
 * 38), so a recycled frame needs only its 64-B header restored -- with non-temporal stores, so the NIC thread does not
 * read the line it overwrites -- and frames ahead are prefetched. */
static void nic_pass(struct nic* N) {
    const uint32_t R = N->R, len = N->len, hdr = len < 64u ? len : 64u;
    const struct xsk_gpu_desc* txe = (const struct xsk_gpu_desc*)N->mtx->ents;
    const uint32_t tx_prod = __atomic_load_n(&N->mtx->prod, __ATOMIC_ACQUIRE);
    /* a TX descriptor is taken only while the completion ring has room for it, as the kernel does (round 5's tool
     * posted completions without looking: with thousands of replies per step it overwrote completions the application
     * had not read yet, handing the same frames back twice -- every "failure" of its pipelined 1024-frame runs) */
    const uint32_t comp_cons = __atomic_load_n(&N->mcomp->cons, __ATOMIC_ACQUIRE);
    uint32_t comp_room = R - (N->k_comp_prod - comp_cons);
    for (; N->k_tx_cons != tx_prod && comp_room; N->k_tx_cons++, comp_room--) {
        const struct xsk_gpu_desc* d = &txe[N->k_tx_cons & (R - 1)];
        if (tx_prod - N->k_tx_cons > 16u) __builtin_prefetch(N->umem + txe[(N->k_tx_cons + 16u) & (R - 1)].addr);
        N->out[d->addr / CHUNK] = 0;
        const uint64_t k = N->checked++;
        int bad = 0;
        if (d->len != len) bad = 1;
        else if ((k & 3u) == 0 && memcmp(N->umem + d->addr, N->rep, (k & 63u) ? hdr : len) != 0) bad = 1;
        if (bad) {
            N->fail++;
            if (N->Q->nfail_logged < 4096) {
                N->Q->fail_seq[N->Q->nfail_logged] = N->dseq[d->addr / CHUNK];
                N->Q->fail_kind[N->Q->nfail_logged++] = 3;
            }
        }
        ((uint64_t*)N->mcomp->ents)[N->k_comp_prod & (R - 1)] = d->addr;
        N->k_comp_prod++;
    }
    __atomic_store_n(&N->mtx->cons, N->k_tx_cons, __ATOMIC_RELEASE);
    __atomic_store_n(&N->mcomp->prod, N->k_comp_prod, __ATOMIC_RELEASE);
    const uint32_t fill_prod = __atomic_load_n(&N->mfill->prod, __ATOMIC_ACQUIRE);
    const uint32_t rx_cons = __atomic_load_n(&N->mrx->cons, __ATOMIC_ACQUIRE);
    uint32_t room = R - (N->k_rx_prod - rx_cons);
    if (N->Q->empty) {
        if (N->k_rx_prod != rx_cons) room = 0; /* exactly one batch per step: the previous one taken first */
        room = room < N->Q->step ? room : N->Q->step;
    }
    const __m128i* rq = (const __m128i*)N->req;
    const __m128i r0 = _mm_loadu_si128(rq), r1 = _mm_loadu_si128(rq + 1), r2 = _mm_loadu_si128(rq + 2),
                  r3 = _mm_loadu_si128(rq + 3);
    for (; room && N->k_fill_cons != fill_prod; room--, N->k_fill_cons++) {
        const uint64_t base = ((uint64_t*)N->mfill->ents)[N->k_fill_cons & (R - 1)] & ~(uint64_t)(CHUNK - 1);
        const uint64_t c = base / CHUNK;
        uint8_t* f = N->umem + base + HEADROOM;
        if (N->out[c]) { /* delivered, never transmitted, back on the fill ring: a frame the step did not answer */
            const int is_req = !memcmp(f, N->req, hdr), is_rep = !memcmp(f, N->rep, hdr);
            const int kind = is_req ? 0 : is_rep ? 1 : 2;
            N->Q->dropped[kind]++;
            if (kind != 1 && N->Q->nfail_logged < 4096) { /* (a reply handed back: the TX ring was full) */
                N->Q->fail_seq[N->Q->nfail_logged] = N->dseq[c];
                N->Q->fail_kind[N->Q->nfail_logged++] = (uint8_t)kind;
            }
        }
        N->out[c] = 1;
        N->dseq[c] = N->k_rx_prod;
        if (N->primed[c] && hdr == 64u) { /* 64-B aligned header, streamed */
            _mm_stream_si128((__m128i*)f, r0);
            _mm_stream_si128((__m128i*)f + 1, r1);
            _mm_stream_si128((__m128i*)f + 2, r2);
            _mm_stream_si128((__m128i*)f + 3, r3);
        } else {
            memcpy(f, N->req, N->primed[c] ? hdr : len);
        }
        N->primed[c] = 1;
        struct xsk_gpu_desc* d = &((struct xsk_gpu_desc*)N->mrx->ents)[N->k_rx_prod & (R - 1)];
        d->addr = base + HEADROOM;
        d->len = len;
        d->options = 0;
        N->k_rx_prod++;
    }
    _mm_sfence(); /* the streamed headers before the RX descriptors that hand them over */
    __atomic_store_n(&N->mfill->cons, N->k_fill_cons, __ATOMIC_RELEASE);
    __atomic_store_n(&N->mrx->prod, N->k_rx_prod, __ATOMIC_RELEASE);
}

static void* nic_main(void* arg) {
    struct nic* N = (struct nic*)arg;
    while (!N->stop) nic_pass(N);
    nic_pass(N); /* the last replies */
    return NULL;
}

static void* run_queue(void* arg) {
    struct queue* Q = (struct queue*)arg;
    const uint32_t R = Q->ring, F = Q->frames, len = Q->len;
    uint8_t* umem = NULL;
    if (Q->huge ? xsk_gpu_umem_alloc((void**)&umem, (uint64_t)F * CHUNK, NULL) != 0
                : posix_memalign((void**)&umem, 4096, (size_t)F * CHUNK) != 0) {
        Q->rc = -12;
        return NULL;
    }
    memset(umem, 0, (size_t)F * CHUNK);
    uint8_t req[4096], rep[4096];
    make_pair(req, rep, len, Q->q);
    struct ring_mem mrx, mfill, mtx, mcomp;
    struct xsk_gpu_ring rx, fill, tx, comp; /* the application's views */
    ring_init(&rx, &mrx, R, sizeof(struct xsk_gpu_desc), 0);
    ring_init(&fill, &mfill, R, 8, 1);
    ring_init(&tx, &mtx, R, sizeof(struct xsk_gpu_desc), 1);
    ring_init(&comp, &mcomp, R, 8, 0);
    struct xsk_gpu_frame_pool pool;
    pool.addr = (uint64_t*)malloc(sizeof(uint64_t) * F);
    pool.capacity = F;
    pool.n_free = 0;
    for (uint32_t i = 0; i < F; i++) pool.addr[pool.n_free++] = (uint64_t)(F - 1 - i) * CHUNK; /* xsk_utils.c:140-141 */
    xsk_gpu_ctx* ctx = NULL;
    xsk_gpu_rx_pipe* pipe = NULL;
    const uint32_t maxb = Q->step < XSK_GPU_RX_MAX_STEP ? Q->step : XSK_GPU_RX_MAX_STEP;
    if (Q->pipe) {
        Q->rc = xsk_gpu_rx_pipe_init(&pipe, 0, umem, (uint64_t)F * CHUNK, Q->pipe, Q->mode);
        if (Q->rc) return NULL;
        Q->real_mode = xsk_gpu_ctx_mode(xsk_gpu__rx_pipe_ctx(pipe, Q->pipe - 1)); /* (the last may have no slot) */
    } else {
        Q->rc = xsk_gpu_init(&ctx, 0, umem, (uint64_t)F * CHUNK, maxb, Q->mode);
        if (Q->rc) return NULL;
        Q->real_mode = xsk_gpu_ctx_mode(ctx);
    }
    struct nic N;
    memset(&N, 0, sizeof N);
    N.Q = Q;
    N.umem = umem;
    N.req = req;
    N.rep = rep;
    N.mrx = &mrx, N.mfill = &mfill, N.mtx = &mtx, N.mcomp = &mcomp;
    N.R = R;
    N.len = len;
    N.primed = (uint8_t*)calloc(F, 1);
    N.out = (uint8_t*)calloc(F, 1);
    N.dseq = (uint64_t*)calloc(F, sizeof(uint64_t));
    struct xsk_gpu_stats st;
    memset(&st, 0, sizeof st);
    const size_t cap = 1u << 22;
    Q->lat = (double*)malloc(sizeof(double) * cap);
    Q->step_seq = (uint64_t*)malloc(sizeof(uint64_t) * cap);
    Q->step_n = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    if (Q->groups) /* LOWLAT serving workgroups forced (diagnosis: slices vs whole batches) */
        for (uint32_t i = 0; i < (pipe ? Q->pipe : 1u); i++)
            (void)xsk_gpu__lowlat_tune(pipe ? xsk_gpu__rx_pipe_ctx(pipe, i) : ctx, 0, Q->groups, 0);
    /* prime the fill ring (the reference's init, xsk_utils.c:163-177) */
    {
        uint32_t idx = 0;
        const uint32_t n = F < R ? F : R;
        idx = fill.cached_prod;
        for (uint32_t i = 0; i < n; i++) ((uint64_t*)mfill.ents)[(idx + i) & (R - 1)] = pool.addr[--pool.n_free];
        fill.cached_prod += n;
        __atomic_store_n(&mfill.prod, mfill.prod + n, __ATOMIC_RELEASE);
    }
    pthread_t nth;
    if (Q->nic_thread == 1 && pthread_create(&nth, NULL, nic_main, &N) != 0) Q->nic_thread = 0;
    const double t_start = now_s(), t_end = t_start + Q->seconds;
    while (Q->nic_thread == 2 && now_s() < t_end && Q->nlat < cap) {
        /* burst: untimed, the NIC checks and completes the last burst's replies, the application returns them to the
         * fill ring, and the NIC receives a request into every frame (the RX ring holds them all); timed, the
         * application's steps until every received frame is completed */
        nic_pass(&N);
        xsk_gpu_tx_complete(&comp, &pool, R);
        {
            uint32_t n = pool.n_free, idx = fill.cached_prod;
            const uint32_t room = R - (fill.cached_prod - __atomic_load_n(&mfill.cons, __ATOMIC_ACQUIRE));
            n = n < room ? n : room;
            for (uint32_t i = 0; i < n; i++) ((uint64_t*)mfill.ents)[(idx + i) & (R - 1)] = pool.addr[--pool.n_free];
            fill.cached_prod += n;
            __atomic_store_n(&mfill.prod, fill.cached_prod, __ATOMIC_RELEASE);
        }
        nic_pass(&N);
        const uint32_t burst = N.k_rx_prod - __atomic_load_n(&mrx.cons, __ATOMIC_ACQUIRE);
        const double t0 = now_s();
        uint64_t done = 0;
        while (done < burst) {
            const double s0 = now_s();
            struct xsk_gpu_rx_result res;
            const uint32_t cons0 = mrx.cons;
            const int got = pipe ? xsk_gpu_rx_pipe_step(pipe, &rx, &fill, &tx, &pool, Q->step, &st, &res)
                                 : xsk_gpu_rx_step(ctx, &rx, &fill, &tx, &pool, Q->step, &st, &res);
            if (got >= 0 && res.received && Q->nsteps_logged < cap) {
                Q->step_seq[Q->nsteps_logged] = cons0;
                Q->step_n[Q->nsteps_logged++] = res.received;
            }
            if (got < 0) {
                Q->rc = got;
                break;
            }
            if (got == 0) continue;
            Q->tx_full += res.tx_full;
            Q->not_replied += (uint64_t)got - res.replied - res.tx_full;
            done += (uint64_t)got;
            Q->steps++;
            if (Q->nlat < cap) Q->lat[Q->nlat++] = now_s() - s0;
        }
        Q->busy += now_s() - t0;
        Q->frames_done += done;
        if (Q->rc) break;
    }
    while (Q->nic_thread != 2 && now_s() < t_end && Q->nlat < cap) {
        if (!Q->nic_thread) nic_pass(&N); /* the NIC between steps, untimed */
        /* ---- the application's loop ---- */
        const double t0 = now_s();
        xsk_gpu_tx_complete(&comp, &pool, R);
        struct xsk_gpu_rx_result res;
        const uint32_t cons0 = mrx.cons;
        const int got = pipe ? xsk_gpu_rx_pipe_step(pipe, &rx, &fill, &tx, &pool, Q->step, &st, &res)
                             : xsk_gpu_rx_step(ctx, &rx, &fill, &tx, &pool, Q->step, &st, &res);
        if (got >= 0 && res.received && Q->nsteps_logged < cap) {
            Q->step_seq[Q->nsteps_logged] = cons0;
            Q->step_n[Q->nsteps_logged++] = res.received;
        }
        const double dt = now_s() - t0;
        if (got < 0) {
            Q->rc = got;
            break;
        }
        Q->busy += dt;
        if (got == 0) continue;
        Q->tx_full += res.tx_full;
        Q->not_replied += (uint64_t)got - res.replied - res.tx_full;
        Q->frames_done += (uint64_t)got;
        Q->steps++;
        Q->lat[Q->nlat++] = dt;
    }
    if (pipe) { /* the batches still in flight (part of the run) */
        const double t0 = now_s();
        struct xsk_gpu_rx_result res;
        const int got = xsk_gpu_rx_pipe_flush(pipe, &tx, &pool, &st, &res);
        Q->busy += now_s() - t0;
        if (got < 0) {
            Q->rc = got;
        } else {
            Q->tx_full += res.tx_full;
            Q->not_replied += (uint64_t)got - res.replied - res.tx_full;
            Q->frames_done += (uint64_t)got;
        }
    }
    Q->wall = Q->nic_thread == 2 ? Q->busy : now_s() - t_start;
    if (Q->nic_thread == 1) {
        N.stop = 1;
        pthread_join(nth, NULL);
    } else {
        nic_pass(&N);
    }
    Q->checked = N.checked;
    Q->wrong_reply = N.fail;
    for (uint32_t i = 0; i < (pipe ? Q->pipe : 1u); i++) { /* LOWLAT outcomes, every context of the queue */
        uint64_t o[4];
        if (xsk_gpu__lowlat_outcomes(pipe ? xsk_gpu__rx_pipe_ctx(pipe, i) : ctx, o) == 0)
            for (int k = 0; k < 4; k++) Q->outcomes[k] += o[k];
    }
    if (pipe) xsk_gpu_rx_pipe_fini(pipe);
    xsk_gpu_fini(ctx);
    /* a reply dropped for a full TX ring is not counted as sent (xsk_receive.c:171-172 count successful sends) */
    if (st.rx_packets != Q->frames_done || st.tx_packets != Q->frames_done - Q->tx_full - Q->not_replied) Q->counters = 1;
    Q->fail = Q->not_replied + Q->wrong_reply + Q->counters;
    free(N.primed);
    free(N.out);
    free(N.dseq);
    if (Q->huge) xsk_gpu_umem_free(umem, (uint64_t)F * CHUNK);
    else free(umem);
    free(pool.addr);
    free(mrx.ents), free(mfill.ents), free(mtx.ents), free(mcomp.ents);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <step> <lowlat|zerocopy|staged> <seconds> [len=64] [queues=1] [ring=4096] "
                        "[frames=4096] [empty=0]\n", argv[0]);
        return 2;
    }
    const uint32_t step = (uint32_t)atoi(argv[1]);
    const int mode = !strcmp(argv[2], "lowlat") ? XSK_GPU_MODE_LOWLAT
                     : !strcmp(argv[2], "staged") ? XSK_GPU_MODE_STAGED : XSK_GPU_MODE_ZEROCOPY;
    const double seconds = atof(argv[3]);
    uint32_t len = 64, nq = 1, ring = 4096, frames = 4096, empty = 0, pipe = 0, nic = 1, huge = 0, groups = 0;
    for (int a = 4; a < argc; a++) {
        if (!strncmp(argv[a], "len=", 4)) len = (uint32_t)atoi(argv[a] + 4);
        else if (!strncmp(argv[a], "queues=", 7)) nq = (uint32_t)atoi(argv[a] + 7);
        else if (!strncmp(argv[a], "ring=", 5)) ring = (uint32_t)atoi(argv[a] + 5);
        else if (!strncmp(argv[a], "frames=", 7)) frames = (uint32_t)atoi(argv[a] + 7);
        else if (!strncmp(argv[a], "empty=", 6)) empty = (uint32_t)atoi(argv[a] + 6);
        else if (!strncmp(argv[a], "pipe=", 5)) pipe = (uint32_t)atoi(argv[a] + 5);
        else if (!strncmp(argv[a], "huge=", 5)) huge = (uint32_t)atoi(argv[a] + 5);
        else if (!strncmp(argv[a], "groups=", 7)) groups = (uint32_t)atoi(argv[a] + 7);
        else if (!strncmp(argv[a], "nic=", 4))
            nic = !strcmp(argv[a] + 4, "thread") ? 1u : !strcmp(argv[a] + 4, "burst") ? 2u : 0u;
    }
    if (len < 42 || len > CHUNK - HEADROOM || nq < 1 || nq > 16 || (ring & (ring - 1)) || ring < 64 || frames < ring ||
        step < 1 || pipe > XSK_GPU_RX_PIPE_MAX) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    struct queue Q[16];
    pthread_t th[16];
    memset(Q, 0, sizeof Q);
    for (uint32_t q = 0; q < nq; q++) {
        Q[q].q = q;
        Q[q].step = step;
        Q[q].len = len;
        Q[q].ring = ring;
        Q[q].frames = frames;
        Q[q].empty = empty;
        Q[q].pipe = pipe;
        Q[q].nic_thread = nic;
        Q[q].huge = huge;
        Q[q].groups = groups;
        Q[q].mode = mode;
        Q[q].seconds = seconds;
        pthread_create(&th[q], NULL, run_queue, &Q[q]);
    }
    uint64_t tot = 0, checked = 0, fail = 0, tx_full = 0;
    /* where the first failures of queue 0 sit: per failing step (by RX sequence), the slot ranges that failed */
    char where[8192];
    where[0] = 0;
    double t_max = 0.0;
    int rc = 0;
    printf("{\"tool\": \"rxring\", \"step\": %u, \"mode\": \"%s\", \"len\": %u, \"queues\": %u, \"ring\": %u, "
           "\"frames\": %u, \"empty\": %u, \"pipe\": %u, \"huge\": %u, \"timing\": \"%s\", \"per_queue\": [", step, argv[2],
           len, nq, ring, frames, empty, pipe, huge, nic == 2 ? "burst" : nic ? "wall" : "app");
    for (uint32_t q = 0; q < nq; q++) {
        pthread_join(th[q], NULL);
        struct queue* R = &Q[q];
        if (q == 0 && R->nfail_logged) {
            size_t w = 0;
            uint64_t prev_step = ~0ull;
            uint32_t run0 = 0, runlen = 0, kind0 = 0;
            int printed = 0;
            /* sort the logged failures by sequence number (insertion sort: at most 4096) */
            for (uint32_t i = 1; i < R->nfail_logged; i++)
                for (uint32_t j = i; j > 0 && R->fail_seq[j - 1] > R->fail_seq[j]; j--) {
                    uint64_t t = R->fail_seq[j];
                    R->fail_seq[j] = R->fail_seq[j - 1];
                    R->fail_seq[j - 1] = t;
                    uint8_t k = R->fail_kind[j];
                    R->fail_kind[j] = R->fail_kind[j - 1];
                    R->fail_kind[j - 1] = k;
                }
            for (uint32_t i = 0; i <= R->nfail_logged && printed < 40 && w < sizeof where - 200; i++) {
                uint64_t st_i = ~0ull;
                uint32_t slot = 0, sn = 0;
                if (i < R->nfail_logged) {
                    const uint64_t s32 = R->fail_seq[i] & 0xFFFFFFFFull; /* ring indices are u32 */
                    uint64_t lo = 0, hi = R->nsteps_logged;
                    while (lo < hi) { /* last step whose start <= seq (steps in RX order; u32 wrap ignored) */
                        const uint64_t mid = (lo + hi) / 2;
                        if (R->step_seq[mid] <= s32) lo = mid + 1;
                        else hi = mid;
                    }
                    if (lo) {
                        st_i = lo - 1;
                        slot = (uint32_t)(s32 - R->step_seq[st_i]);
                        sn = R->step_n[st_i];
                    }
                }
                const int cont = i < R->nfail_logged && st_i == prev_step && slot == run0 + runlen &&
                                 R->fail_kind[i] == kind0;
                if (cont) {
                    runlen++;
                    continue;
                }
                if (runlen)
                    w += (size_t)snprintf(where + w, sizeof where - w, "%s[step %llu: slots %u-%u kind %u]",
                                          printed++ ? ", " : "", (unsigned long long)prev_step, run0, run0 + runlen - 1,
                                          kind0);
                if (i == R->nfail_logged) break;
                prev_step = st_i;
                run0 = slot;
                runlen = 1;
                kind0 = R->fail_kind[i];
                (void)sn;
            }
        }
        if (R->rc) rc = R->rc;
        qsort(R->lat, R->nlat, sizeof(double), cmpd);
        const double p50 = R->nlat ? R->lat[R->nlat / 2] : 0.0, p99 = R->nlat ? R->lat[(R->nlat * 99) / 100] : 0.0;
        const double T = nic ? R->wall : R->busy; /* the NIC in a thread of its own: the loop's wall time */
        printf("%s{\"mode\": %d, \"mframes_s\": %.3f, \"us_per_step\": %.3f, \"p50_us\": %.3f, \"p99_us\": %.3f, "
               "\"frames_per_step\": %.1f, \"steps\": %llu, \"tx_full\": %llu, \"not_replied\": %llu, "
               "\"wrong_reply\": %llu, \"counters\": %llu, \"dropped_req_rep_other\": [%llu, %llu, %llu], "
               "\"lowlat_timeouts_all_partial_failed_late\": [%llu, %llu, %llu, %llu], \"rc\": %d}", q ? ", " : "", R->real_mode,
               T > 0 ? 1e-6 * (double)R->frames_done / T : 0.0, R->steps ? 1e6 * T / (double)R->steps : 0.0, 1e6 * p50,
               1e6 * p99,
               R->steps ? (double)R->frames_done / (double)R->steps : 0.0, (unsigned long long)R->steps,
               (unsigned long long)R->tx_full, (unsigned long long)R->not_replied, (unsigned long long)R->wrong_reply,
               (unsigned long long)R->counters, (unsigned long long)R->dropped[0], (unsigned long long)R->dropped[1], (unsigned long long)R->dropped[2],
               (unsigned long long)R->outcomes[0], (unsigned long long)R->outcomes[1],
               (unsigned long long)R->outcomes[2], (unsigned long long)R->outcomes[3], R->rc);
        tot += R->frames_done;
        checked += R->checked;
        fail += R->fail;
        tx_full += R->tx_full;
        if ((nic ? R->wall : R->busy) > t_max) t_max = nic ? R->wall : R->busy;
        free(R->lat);
        free(R->step_seq);
        free(R->step_n);
    }
    printf("], \"mframes_s_total\": %.3f, \"frames\": %llu, \"checked\": %llu, \"tx_full\": %llu, \"failures\": %llu, "
           "\"where\": \"%s\", \"rc\": %d}\n", t_max > 0 ? 1e-6 * (double)tot / t_max : 0.0, (unsigned long long)tot,
           (unsigned long long)checked, (unsigned long long)tx_full, (unsigned long long)fail, where, rc);
    return rc || fail ? 1 : 0;
}
