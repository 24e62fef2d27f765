/*
 * xsk_gpu_pipe.c — the pipelined RX loop (include/xsk_gpu.h, xsk_gpu_rx_pipe_*): the reference's
 * handle_receive_packets() (src/lib/xsk_receive.c:192-237) as xsk_gpu_rx_step runs it, but with up to
 * XSK_GPU_RX_PIPE_MAX batches in flight, one per context.  A step of xsk_gpu_rx_step costs a PCIe round trip
 * (doorbell, frames, completion) whatever its size; here step k+1 is posted while step k is still being served, so a
 * queue's throughput at a small step is no longer one batch per round trip.  Batches complete in the order they were
 * received, and every frame's bytes, verdict and counters are exactly xsk_gpu_rx_step's.  Host code (C11).
 */
#define _GNU_SOURCE
#define __HIP_PLATFORM_AMD__ 1
#include <errno.h>
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include "xsk_gpu_internal.h"
#include "xsk_ring.h"

struct pipe_slot {
    xsk_gpu_ctx* ctx;
    uint32_t n;  /* frames of the batch this context holds (0: free) */
    int failed;  /* its completion failed with every frame untouched: the next step or flush runs it again through
                  * xsk_gpu_process */
    struct xsk_gpu_desc descs[XSK_GPU_RX_MAX_STEP]; /* the batch as received (the TX / free path needs them) */
    uint8_t verdict[XSK_GPU_RX_MAX_STEP];
};

struct xsk_gpu_rx_pipe {
    int device;
    uint8_t* umem;
    void* reg_base; /* the UMEM registration this object holds a reference of */
    uint32_t depth;
    uint32_t head;  /* slot of the oldest batch in flight */
    uint32_t count; /* batches in flight: slots head, head + 1, ... (mod depth) */
    struct pipe_slot s[XSK_GPU_RX_PIPE_MAX];
};

void xsk_gpu_rx_pipe_fini(xsk_gpu_rx_pipe* p) {
    if (!p) return;
    for (uint32_t i = 0; i < p->depth; i++) xsk_gpu_fini(p->s[i].ctx); /* (waits for a batch still in flight) */
    if (p->reg_base) {
        const int caller_dev = xsk_gpu__dev_save();
        (void)hipSetDevice(p->device);
        xsk_gpu__umem_unref(p->reg_base);
        xsk_gpu__dev_restore(caller_dev);
    }
    free(p);
}

int xsk_gpu_rx_pipe_init(xsk_gpu_rx_pipe** out, int device, void* umem, uint64_t umem_size, uint32_t depth, int mode) {
    if (!out || !umem || umem_size == 0 || !xsk_gpu__umem_aligned(umem) || (umem_size & 15u) || depth == 0 ||
        depth > XSK_GPU_RX_PIPE_MAX ||
        (mode != XSK_GPU_MODE_ZEROCOPY && mode != XSK_GPU_MODE_STAGED && mode != XSK_GPU_MODE_LOWLAT))
        return -EINVAL;
    *out = NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    xsk_gpu_rx_pipe* p = (xsk_gpu_rx_pipe*)calloc(1, sizeof *p);
    if (!p) return -ENOMEM;
    p->device = device;
    p->umem = (uint8_t*)umem;
    int rc = 0;
    /* one registration of the UMEM, mapped, for every context of the pipe */
    const int caller_dev = xsk_gpu__dev_save();
    /* (shared and counted with every other user of this UMEM: xsk_gpu__umem_ref) */
    rc = hipSetDevice(device) == hipSuccess ? xsk_gpu__umem_ref(umem, umem_size, &p->reg_base) : -EIO;
    xsk_gpu__dev_restore(caller_dev);
    if (rc) {
        free(p);
        return rc;
    }
    uint32_t kept = depth;
    for (uint32_t i = 0; i < depth; i++) {
        rc = xsk_gpu__init_prereg(&p->s[i].ctx, device, umem, umem_size, XSK_GPU_RX_MAX_STEP, mode);
        if (rc) {
            p->depth = i;
            xsk_gpu_rx_pipe_fini(p);
            return rc;
        }
        /* a LOWLAT pipe keeps doorbell contexts only: completion is in RX order, so a launched (ZEROCOPY) context
         * among them would hold every batch behind its own (include/xsk_gpu.h) */
        if (i > 0 && mode == XSK_GPU_MODE_LOWLAT && xsk_gpu_ctx_mode(p->s[i].ctx) != XSK_GPU_MODE_LOWLAT &&
            xsk_gpu_ctx_mode(p->s[0].ctx) == XSK_GPU_MODE_LOWLAT) {
            xsk_gpu_fini(p->s[i].ctx);
            p->s[i].ctx = NULL;
            kept = i;
            break;
        }
    }
    p->depth = kept;
    *out = p;
    return 0;
}

static void retire_oldest(xsk_gpu_rx_pipe* p) {
    struct pipe_slot* s = &p->s[p->head];
    s->n = 0;
    s->failed = 0;
    p->head = (p->head + 1u) % p->depth;
    p->count--;
}

/* Complete the oldest batch in flight and hand it on (xsk_gpu_rx_step's steps 4-5): the frames completed, or the
 * error.  A batch that failed with every frame untouched stays the oldest, marked to run again; one whose frames may
 * partly have been transformed (xsk_gpu__failed_untouched) is dropped -- its frames back to the pool, none transmitted
 * -- since running it again could transform a frame twice. */
static int complete_oldest(xsk_gpu_rx_pipe* p, struct xsk_gpu_ring* tx, struct xsk_gpu_frame_pool* pool,
                           struct xsk_gpu_stats* stats, struct xsk_gpu_rx_result* r) {
    struct pipe_slot* s = &p->s[p->head];
    const int rc = s->failed ? xsk_gpu_process(s->ctx, s->descs, s->n, s->verdict, NULL, NULL)
                             : xsk_gpu__complete(s->ctx, s->verdict, NULL, NULL);
    if (rc) {
        if (xsk_gpu__failed_untouched(s->ctx)) {
            s->failed = 1;
        } else {
            xsk_gpu__rx_drop(s->descs, s->n, pool);
            retire_oldest(p);
        }
        return rc;
    }
    xsk_gpu__rx_emit(s->descs, s->verdict, s->n, tx, pool, stats, r);
    const int n = (int)s->n;
    retire_oldest(p);
    return n;
}

int xsk_gpu_rx_pipe_step(xsk_gpu_rx_pipe* p, struct xsk_gpu_ring* rx, struct xsk_gpu_ring* fill, struct xsk_gpu_ring* tx,
                         struct xsk_gpu_frame_pool* pool, uint32_t max_batch, struct xsk_gpu_stats* stats,
                         struct xsk_gpu_rx_result* res) {
    struct xsk_gpu_rx_result r = {0, 0, 0, 0};
    if (!p || !rx || !fill || !tx || !pool || !pool->addr || max_batch == 0) return -EINVAL;
    if (max_batch > XSK_GPU_RX_MAX_STEP) max_batch = XSK_GPU_RX_MAX_STEP;
    int done = 0, rc = 0;
    if (p->count < p->depth && xr_cons_avail(rx, 1)) {
        struct pipe_slot* s = &p->s[(p->head + p->count) % p->depth];
        uint32_t idx_rx = 0;
        const uint32_t rcvd = xr_cons_peek(rx, max_batch, &idx_rx); /* :196 */
        for (uint32_t i = 0; i < rcvd; i++) s->descs[i] = *xr_desc(rx, idx_rx + i);
        rc = xsk_gpu__submit(s->ctx, s->descs, rcvd, 0, 0);
        if (rc) {
            if (xsk_gpu__failed_untouched(s->ctx)) { /* frames stay on the RX ring, as after a failed xsk_gpu_rx_step */
                rx->cached_cons -= rcvd;
            } else { /* possibly partly transformed: dropped, as xsk_gpu_rx_step does */
                xsk_gpu__rx_drop(s->descs, rcvd, pool);
                xr_cons_release(rx, rcvd);
                r.received = rcvd;
            }
            goto out;
        }
        xr_cons_release(rx, rcvd); /* :232 -- the descriptors are ours now (s->descs) */
        s->n = rcvd;
        s->failed = 0;
        p->count++;
        r.received = rcvd;
    }
    /* the oldest batch first: when every context is busy, when it is done already, and -- the RX ring was empty --
     * every batch, so an idle link is answered at once */
    while (p->count) {
        const struct pipe_slot* s = &p->s[p->head];
        if (r.received && p->count < p->depth && (s->failed || !xsk_gpu__ready(s->ctx))) break;
        const int k = complete_oldest(p, tx, pool, stats, &r);
        if (k < 0) {
            /* the batch stays the oldest, to run again; frames this call already handed on are reported first (the
             * error then comes from the next call if the rerun fails too) */
            if (!done) rc = k;
            break;
        }
        done += k;
    }
    /* :201-217 -- the fill ring restocked on every step, after the completions: a batch completed by a step that
     * received nothing (the ring ran empty) has freed its frames, and with several batches in flight they may be most
     * of the UMEM; restocked only when frames arrive, as the reference does, the fill ring could run dry and no frame
     * would arrive again */
    r.refilled = xsk_gpu__rx_refill(fill, pool);
out:
    if (res) *res = r;
    return rc ? rc : done;
}

int xsk_gpu_rx_pipe_flush(xsk_gpu_rx_pipe* p, struct xsk_gpu_ring* tx, struct xsk_gpu_frame_pool* pool,
                          struct xsk_gpu_stats* stats, struct xsk_gpu_rx_result* res) {
    struct xsk_gpu_rx_result r = {0, 0, 0, 0};
    if (!p || !tx || !pool || !pool->addr) return -EINVAL;
    int done = 0, rc = 0;
    while (p->count) {
        const int k = complete_oldest(p, tx, pool, stats, &r);
        if (k < 0) {
            if (!done) rc = k; /* (as in a step: frames handed on are reported first) */
            break;
        }
        done += k;
    }
    if (res) *res = r;
    return rc ? rc : done;
}

int xsk_gpu_rx_pipe_set_options(xsk_gpu_rx_pipe* p, uint32_t opts) {
    if (!p || (opts & ~XSK_GPU_OPT_ALL)) return -EINVAL;
    if (p->count) return -EBUSY;
    for (uint32_t i = 0; i < p->depth; i++) {
        const int rc = xsk_gpu_set_options(p->s[i].ctx, opts);
        if (rc) return rc;
    }
    return 0;
}

uint32_t xsk_gpu_rx_pipe_inflight(const xsk_gpu_rx_pipe* p) { return p ? p->count : 0u; }

uint32_t xsk_gpu_rx_pipe_depth(const xsk_gpu_rx_pipe* p) { return p ? p->depth : 0u; }

xsk_gpu_ctx* xsk_gpu__rx_pipe_ctx(xsk_gpu_rx_pipe* p, uint32_t i) { return p && i < p->depth ? p->s[i].ctx : NULL; }
