/* CPU unit test of the pipelined RX loop (xsknet_amd/csrc/xsk_gpu_pipe.c) and the RX-step helpers it shares with
 * xsk_gpu_rx_step (xsk_gpu_rx.c), against fake contexts: submit / complete / ready / process are simulated (a batch
 * completes after a random number of ready() polls; a completion or a submit can be made to fail), and a simulated
 * AF_XDP kernel side delivers bursts into the RX ring from the fill ring and takes replies off the TX ring.  Checked:
 * every frame transformed exactly once and handed on exactly once, in RX order (replies on the TX ring in RX order),
 * never more than `depth` batches in flight, a failed completion run again by the next step (its frames untouched
 * until then), a failed submit leaving its frames on the RX ring, the counters, and every frame accounted for at the
 * end.  A failure whose batch may be partly transformed (a partly served doorbell batch whose launch path failed, a
 * launch error: xsk_gpu__failed_untouched() == 0) drops the batch -- its frames back to the pool, none handed on, and
 * no frame ever transformed twice (the pipe used to run such a batch again).
 * Built and run by tests/test_rx_pipe.py. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_gpu_pipe.c"
#include "../../xsknet_amd/csrc/xsk_gpu_rx.c"

/* ---- the HIP calls xsk_gpu_pipe.c makes ---- */
hipError_t hipGetDeviceCount(int* n) {
    *n = 1;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidDevice; }
static int g_umem_refs; /* the pipe's references of the UMEM registration (xsk_gpu_host.c's table) */
int xsk_gpu__umem_ref(void* base, uint64_t size, void** reg_base) {
    (void)size;
    *reg_base = base;
    g_umem_refs++;
    return 0;
}
void xsk_gpu__umem_unref(void* reg_base) {
    if (!reg_base) return;
    assert(g_umem_refs > 0);
    g_umem_refs--;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
int xsk_gpu__dev_save(void) { return 0; }
void xsk_gpu__dev_restore(int d) { (void)d; }

/* ---- fake contexts ---- */
#define NFRAMES 4096u
#define RING 1024u
static uint32_t g_times[NFRAMES]; /* transformed, per frame */
static uint32_t g_pos[NFRAMES];   /* fifo position of the frame's latest delivery */
static uint8_t g_fifo_dropped[1u << 20], g_rep_dropped[1u << 20]; /* per delivery: its batch was dropped */
static uint32_t g_rpos[NFRAMES];  /* rep_fifo position of its latest delivery (replies) */
static uint64_t g_dropped, g_dropped_bytes, g_dropped_tx, g_dropped_tx_bytes, g_dropped_total;
static uint64_t g_seed = 0x1234567u;
static uint32_t rnd(uint32_t m) {
    g_seed = g_seed * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(g_seed >> 33) % m;
}

struct xsk_gpu_ctx {
    uint32_t pend_n, countdown, max_batch, opts;
    int fail_complete, fail_submit, mode;
    int fail_partial, fail_submit_partial, untouched; /* unknown-outcome failures; the last failure's kind */
    struct xsk_gpu_desc d[XSK_GPU_RX_MAX_STEP];
};
static struct xsk_gpu_ctx g_ctx[XSK_GPU_RX_PIPE_MAX];
static uint32_t g_nctx;
static int g_ll_left = 1000; /* the device's free resident-kernel slots (a LOWLAT request without one runs ZEROCOPY) */

static uint8_t verdict_of(const struct xsk_gpu_desc* d) {
    if (d->len < 20u) return XSK_GPU_DROP_SHORT;
    return (d->addr / 4096u) % 5u == 0 ? XSK_GPU_DROP_NOT_ECHO : XSK_GPU_TX_REPLY;
}
static void transform(const struct xsk_gpu_desc* d, uint32_t n, uint8_t* v) {
    for (uint32_t i = 0; i < n; i++) {
        assert(g_times[d[i].addr / 4096u] == 0); /* never twice per delivery */
        g_times[d[i].addr / 4096u]++;
        if (v) v[i] = verdict_of(&d[i]);
    }
}

/* the batch fails with part of it transformed: the pipe must drop it (frames back to the pool, none handed on) */
static void fail_partly(const struct xsk_gpu_desc* d, uint32_t n) {
    transform(d, (n + 1u) / 2u, NULL);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t f = (uint32_t)(d[i].addr / 4096u);
        g_times[f] = 0;
        g_fifo_dropped[g_pos[f]] = 1;
        g_dropped++;
        g_dropped_bytes += d[i].len;
        if (verdict_of(&d[i]) == XSK_GPU_TX_REPLY) {
            g_rep_dropped[g_rpos[f]] = 1;
            g_dropped_tx++;
            g_dropped_tx_bytes += d[i].len;
        }
    }
}

int xsk_gpu__init_prereg(xsk_gpu_ctx** out, int device, void* umem, uint64_t umem_size, uint32_t max_batch, int mode) {
    (void)device, (void)umem, (void)umem_size;
    struct xsk_gpu_ctx* c = &g_ctx[g_nctx++];
    memset(c, 0, sizeof *c);
    c->max_batch = max_batch;
    c->mode = mode;
    if (mode == XSK_GPU_MODE_LOWLAT) {
        if (g_ll_left > 0) g_ll_left--;
        else c->mode = XSK_GPU_MODE_ZEROCOPY;
    }
    *out = c;
    return 0;
}
void xsk_gpu_fini(xsk_gpu_ctx* c) {
    if (!c) return;
    assert(c->pend_n == 0); /* the test flushes first */
    if (c->mode == XSK_GPU_MODE_LOWLAT) g_ll_left++;
    c->mode = -1;
}
int xsk_gpu_ctx_mode(const xsk_gpu_ctx* c) { return c ? c->mode : -EINVAL; }
int xsk_gpu__submit(xsk_gpu_ctx* c, const struct xsk_gpu_desc* d, uint32_t n, int want_recs, int no_doorbell) {
    (void)want_recs, (void)no_doorbell;
    c->untouched = 1;
    if (c->pend_n) return -EBUSY;
    if (c->fail_submit) {
        c->fail_submit = 0;
        return -EIO;
    }
    assert(n >= 1 && n <= c->max_batch);
    if (c->fail_submit_partial) { /* e.g. a launch error after the first chunks ran */
        c->fail_submit_partial = 0;
        c->untouched = 0;
        fail_partly(d, n);
        return -EIO;
    }
    memcpy(c->d, d, n * sizeof *d);
    c->pend_n = n;
    c->countdown = rnd(4);
    return 0;
}
int xsk_gpu__ready(const xsk_gpu_ctx* cc) {
    struct xsk_gpu_ctx* c = (struct xsk_gpu_ctx*)cc;
    if (!c->pend_n) return 1;
    if (c->countdown) {
        c->countdown--;
        return 0;
    }
    return 1;
}
int xsk_gpu__complete(xsk_gpu_ctx* c, uint8_t* verdicts, struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    (void)recs, (void)stats;
    const uint32_t n = c->pend_n;
    if (!n) return 0;
    c->pend_n = 0;
    c->untouched = 0;
    if (c->fail_complete) { /* timed out with every frame untouched */
        c->fail_complete = 0;
        c->untouched = 1;
        return -ETIMEDOUT;
    }
    if (c->fail_partial) { /* part of the batch served, the rest's launch path failed */
        c->fail_partial = 0;
        fail_partly(c->d, n);
        return -EIO;
    }
    transform(c->d, n, verdicts);
    return 0;
}
int xsk_gpu_process(xsk_gpu_ctx* c, const struct xsk_gpu_desc* d, uint32_t n, uint8_t* verdicts,
                    struct xsk_gpu_rec* recs, struct xsk_gpu_stats* stats) {
    (void)recs, (void)stats;
    c->untouched = 1;
    if (c->pend_n) return -EBUSY;
    transform(d, n, verdicts);
    return 0;
}
int xsk_gpu__failed_untouched(const xsk_gpu_ctx* c) { return c->untouched; }
int xsk_gpu_set_options(xsk_gpu_ctx* c, uint32_t opts) {
    c->opts = opts;
    return 0;
}
uint32_t xsk_gpu__ctx_max_batch(const xsk_gpu_ctx* c) { return c->max_batch; }

/* ---- a ring pair: the application's view + the kernel side's cursors ---- */
struct kring {
    uint32_t prod, cons, flags;
    void* ents;
    struct xsk_gpu_ring view;
};
static void kring_init(struct kring* k, size_t esz, int app_produces) {
    memset(k, 0, sizeof *k);
    k->ents = calloc(RING, esz);
    k->view.mask = RING - 1;
    k->view.size = RING;
    k->view.producer = &k->prod;
    k->view.consumer = &k->cons;
    k->view.flags = &k->flags;
    k->view.ring = k->ents;
    if (app_produces) k->view.cached_cons = RING;
}

static void run(uint32_t depth, uint32_t step, int faults) {
    memset(g_times, 0, sizeof g_times);
    memset(g_fifo_dropped, 0, sizeof g_fifo_dropped);
    memset(g_rep_dropped, 0, sizeof g_rep_dropped);
    g_dropped = g_dropped_bytes = g_dropped_tx = g_dropped_tx_bytes = 0;
    g_nctx = 0;
    static uint8_t umem[4096] __attribute__((aligned(4096)));
    xsk_gpu_rx_pipe* p = NULL;
    assert(xsk_gpu_rx_pipe_init(&p, 0, umem, sizeof umem, depth, XSK_GPU_MODE_LOWLAT) == 0);
    struct kring rx, fq, tx, cq;
    kring_init(&rx, sizeof(struct xsk_gpu_desc), 0);
    kring_init(&fq, 8, 1);
    kring_init(&tx, sizeof(struct xsk_gpu_desc), 1);
    kring_init(&cq, 8, 0);
    uint64_t* stack = (uint64_t*)malloc(NFRAMES * sizeof(uint64_t));
    struct xsk_gpu_frame_pool pool = {stack, 0, NFRAMES};
    for (uint32_t i = 0; i < NFRAMES; i++) stack[pool.n_free++] = (uint64_t)(NFRAMES - 1 - i) * 4096u;
    /* prefill the fill ring with RING frames */
    for (uint32_t i = 0; i < RING; i++) ((uint64_t*)fq.ents)[i] = stack[--pool.n_free];
    fq.prod = RING;
    fq.view.cached_prod = RING;
    static uint64_t fifo[1u << 20]; /* delivered frames in RX order */
    static uint64_t rep_fifo[1u << 20]; /* delivered frames that are replies, in RX order */
    uint32_t f_head = 0, f_tail = 0, r_head = 0, r_tail = 0;
    uint64_t sent = 0, handed = 0, replies = 0;
    struct xsk_gpu_stats st;
    memset(&st, 0, sizeof st);
    uint64_t want_rx_bytes = 0, want_tx = 0, want_tx_bytes = 0;
    const uint64_t total = 60000;
    for (uint32_t it = 0; handed + g_dropped < total; it++) {
        assert(it < 10000000u);
        /* kernel: deliver a burst (sometimes nothing, so the ring runs empty) */
        uint32_t burst = rnd(5) == 0 ? 0 : 1 + rnd(200);
        while (burst && sent < total && fq.cons != fq.prod && rx.prod - rx.cons < RING) {
            const uint64_t a = ((uint64_t*)fq.ents)[fq.cons++ & (RING - 1)] & ~4095ull;
            struct xsk_gpu_desc* d = &((struct xsk_gpu_desc*)rx.ents)[rx.prod++ & (RING - 1)];
            d->addr = a;
            d->len = (uint32_t)(sent % 7u == 3u ? 10u : 60u + sent % 1400u);
            d->options = 0;
            want_rx_bytes += d->len;
            if (verdict_of(d) == XSK_GPU_TX_REPLY) {
                want_tx++;
                want_tx_bytes += d->len;
                g_rpos[a / 4096u] = r_tail;
                rep_fifo[r_tail++] = a;
            }
            assert(g_times[a / 4096u] == 0); /* not transformed since it was last handed on */
            g_pos[a / 4096u] = f_tail;
            fifo[f_tail++] = a;
            sent++;
            burst--;
        }
        /* faults: a completion that times out untouched, a submit that fails */
        if (faults && rnd(40) == 0) g_ctx[rnd(depth)].fail_complete = 1;
        if (faults && rnd(60) == 0) g_ctx[rnd(depth)].fail_submit = 1;
        if (faults == 2 && rnd(50) == 0) g_ctx[rnd(depth)].fail_partial = 1;
        if (faults == 2 && rnd(90) == 0) g_ctx[rnd(depth)].fail_submit_partial = 1;
        const uint32_t rx_cons0 = rx.cons, rx_prod0 = rx.prod;
        const uint64_t dropped0 = g_dropped;
        struct xsk_gpu_rx_result res;
        const int got = xsk_gpu_rx_pipe_step(p, &rx.view, &fq.view, &tx.view, &pool, step, &st, &res);
        assert(xsk_gpu_rx_pipe_inflight(p) <= depth);
        if (got < 0) {
            assert(got == -ETIMEDOUT || got == -EIO);
            if (got == -EIO && g_dropped == dropped0) /* an untouched submit failure: the frames stay on RX */
                assert(rx.cons == rx_cons0 && rx.view.cached_cons == rx_cons0);
            continue;
        }
        assert(res.received <= step && rx.cons - rx_cons0 == res.received && rx.prod == rx_prod0);
        /* every completed frame: transformed exactly once, handed on in RX order */
        for (int k = 0; k < got; k++) {
            while (g_fifo_dropped[f_head]) f_head++; /* a dropped batch's frames are never handed on */
            const uint64_t a = fifo[f_head++];
            assert(g_times[a / 4096u] == 1);
            g_times[a / 4096u] = 0; /* (the frame may be delivered again once it is back on the fill ring) */
        }
        if (xsk_gpu_rx_pipe_inflight(p)) assert(xsk_gpu_rx_pipe_set_options(p, 0) == -EBUSY);
        handed += (uint64_t)got;
        /* kernel: transmit in order, complete */
        while (tx.cons != tx.prod) {
            const struct xsk_gpu_desc* t = &((struct xsk_gpu_desc*)tx.ents)[tx.cons++ & (RING - 1)];
            while (g_rep_dropped[r_head]) r_head++;
            assert(r_head < r_tail && t->addr == rep_fifo[r_head]);
            r_head++;
            replies++;
            ((uint64_t*)cq.ents)[cq.prod++ & (RING - 1)] = t->addr;
        }
        xsk_gpu_tx_complete(&cq.view, &pool, RING);
        if (sent == total && rx.prod == rx.cons) {
            struct xsk_gpu_rx_result fr;
            int k = xsk_gpu_rx_pipe_flush(p, &tx.view, &pool, &st, &fr);
            if (k < 0) {
                assert(k == -ETIMEDOUT || k == -EIO);
                k = 0;
            }
            for (int j = 0; j < k; j++) {
                while (g_fifo_dropped[f_head]) f_head++;
                const uint64_t a = fifo[f_head++];
                assert(g_times[a / 4096u] == 1);
                g_times[a / 4096u] = 0;
            }
            handed += (uint64_t)k;
            while (tx.cons != tx.prod) {
                const struct xsk_gpu_desc* t = &((struct xsk_gpu_desc*)tx.ents)[tx.cons++ & (RING - 1)];
                while (g_rep_dropped[r_head]) r_head++;
                assert(t->addr == rep_fifo[r_head++]);
                replies++;
                ((uint64_t*)cq.ents)[cq.prod++ & (RING - 1)] = t->addr;
            }
            xsk_gpu_tx_complete(&cq.view, &pool, RING);
        }
    }
    while (f_head < f_tail && g_fifo_dropped[f_head]) f_head++;
    while (r_head < r_tail && g_rep_dropped[r_head]) r_head++;
    assert(handed + g_dropped == total && f_head == f_tail && r_head == r_tail && xsk_gpu_rx_pipe_inflight(p) == 0);
    if (faults < 2) assert(g_dropped == 0);
    g_dropped_total += g_dropped;
    for (uint32_t f = 0; f < NFRAMES; f++) assert(g_times[f] == 0); /* nothing transformed and not handed on */
    assert(st.rx_packets == total - g_dropped && st.rx_bytes == want_rx_bytes - g_dropped_bytes &&
           st.tx_packets == want_tx - g_dropped_tx && st.tx_bytes == want_tx_bytes - g_dropped_tx_bytes &&
           replies == want_tx - g_dropped_tx);
    /* every frame accounted for: free stack + fill ring (nothing in flight, nothing on RX / TX / completion) */
    assert(pool.n_free + (fq.prod - fq.cons) == NFRAMES);
    assert(xsk_gpu_rx_pipe_set_options(p, XSK_GPU_OPT_ALL) == 0);
    xsk_gpu_rx_pipe_fini(p);
    free(stack);
    free(rx.ents), free(fq.ents), free(tx.ents), free(cq.ents);
}

int main(void) {
    for (uint32_t depth = 1; depth <= XSK_GPU_RX_PIPE_MAX; depth++)
        for (int faults = 0; faults < 3; faults++)
            for (uint32_t step = 1; step <= 1024; step *= 8) run(depth, step, faults);
    assert(g_dropped_total > 0); /* the unknown-outcome failures did happen */
    /* argument checks */
    {
        g_nctx = 0;
        static uint8_t umem[4096] __attribute__((aligned(4096)));
        xsk_gpu_rx_pipe* p = NULL;
        assert(xsk_gpu_rx_pipe_init(&p, 0, umem, sizeof umem, 2, XSK_GPU_MODE_ZEROCOPY) == 0);
        assert(xsk_gpu_rx_pipe_depth(p) == 2 && xsk_gpu_rx_pipe_depth(NULL) == 0);
        xsk_gpu_rx_pipe_fini(p);
        assert(xsk_gpu_rx_pipe_init(&p, 0, umem, sizeof umem, XSK_GPU_RX_PIPE_MAX + 1, XSK_GPU_MODE_ZEROCOPY) == -EINVAL);
        assert(xsk_gpu_rx_pipe_init(&p, 1, umem, sizeof umem, 2, XSK_GPU_MODE_ZEROCOPY) == -ENODEV);
        xsk_gpu_rx_pipe_fini(p);
    }
    /* a LOWLAT pipe keeps doorbell contexts only: with 3 slots left a depth-8 request holds 3 LOWLAT contexts (the
     * fourth, downgraded, is let go); with none, all 8 run ZEROCOPY; ZEROCOPY pipes are never trimmed */
    {
        static uint8_t umem[4096] __attribute__((aligned(4096)));
        for (int left = 0; left <= 9; left += 3) {
            g_nctx = 0;
            g_ll_left = left;
            xsk_gpu_rx_pipe* p = NULL;
            assert(xsk_gpu_rx_pipe_init(&p, 0, umem, sizeof umem, 8, XSK_GPU_MODE_LOWLAT) == 0);
            const uint32_t want = left == 0 ? 8u : (left < 8 ? (uint32_t)left : 8u);
            assert(xsk_gpu_rx_pipe_depth(p) == want);
            for (uint32_t i = 0; i < want; i++)
                assert(xsk_gpu_ctx_mode(xsk_gpu__rx_pipe_ctx(p, i)) == (left ? XSK_GPU_MODE_LOWLAT : XSK_GPU_MODE_ZEROCOPY));
            assert(g_ll_left == (left > 8 ? left - 8 : 0)); /* the let-go context held no slot */
            xsk_gpu_rx_pipe_fini(p);
            assert(g_ll_left == left);
        }
        g_nctx = 0;
        g_ll_left = 1;
        xsk_gpu_rx_pipe* p = NULL;
        assert(xsk_gpu_rx_pipe_init(&p, 0, umem, sizeof umem, 6, XSK_GPU_MODE_ZEROCOPY) == 0);
        assert(xsk_gpu_rx_pipe_depth(p) == 6);
        xsk_gpu_rx_pipe_fini(p);
        g_ll_left = 1000;
    }
    assert(g_umem_refs == 0); /* every pipe gave its registration reference back */
    printf("rx pipe ok\n");
    return 0;
}
