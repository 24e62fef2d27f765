/*
 * xsk_gpu_rx.c — the client's RX loop step (src/lib/xsk_receive.c:192-237) over AF_XDP rings with
 * the echo transform on the GPU and replies leaving through the XSK TX ring (the reference's
 * commented-out path :174-186) instead of one sendto() per frame (:166).  Host code (C11).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <string.h>

#include "xsk_gpu_internal.h"
#include "xsk_ring.h"

static inline void pool_push(struct xsk_gpu_frame_pool* p, uint64_t a) {
    if (p->n_free < p->capacity) p->addr[p->n_free++] = a; /* xsk_free_umem_frame (:65-70) */
}

uint32_t xsk_gpu__rx_refill(struct xsk_gpu_ring* fill, struct xsk_gpu_frame_pool* pool) {
    uint32_t stock = xr_prod_free(fill, pool->n_free);
    if (stock > pool->n_free) stock = pool->n_free;
    if (!stock) return 0;
    uint32_t idx_fq = 0;
    if (xr_prod_reserve(fill, stock, &idx_fq) != stock) return 0;
    for (uint32_t i = 0; i < stock; i++) *xr_addr(fill, idx_fq + i) = pool->addr[--pool->n_free];
    xr_prod_submit(fill, stock);
    return stock;
}

void xsk_gpu__rx_drop(const struct xsk_gpu_desc* descs, uint32_t n, struct xsk_gpu_frame_pool* pool) {
    for (uint32_t i = 0; i < n; i++) pool_push(pool, descs[i].addr);
}

void xsk_gpu__rx_emit(const struct xsk_gpu_desc* descs, const uint8_t* verdict, uint32_t n, struct xsk_gpu_ring* tx,
                      struct xsk_gpu_frame_pool* pool, struct xsk_gpu_stats* stats, struct xsk_gpu_rx_result* r) {
    uint32_t nrep = 0;
    for (uint32_t i = 0; i < n; i++) nrep += verdict[i] == XSK_GPU_TX_REPLY;
    /* :174-186 — replies onto the TX ring, as many as it has room for */
    uint32_t idx_tx = 0, room = 0, sent = 0;
    if (nrep) {
        room = xr_prod_free(tx, nrep);
        if (room > nrep) room = nrep;
        if (room) xr_prod_reserve(tx, room, &idx_tx);
    }
    uint64_t rx_bytes = 0, tx_bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        rx_bytes += descs[i].len;
        if (verdict[i] == XSK_GPU_TX_REPLY && sent < room) {
            struct xsk_gpu_desc* t = xr_desc(tx, idx_tx + sent);
            t->addr = descs[i].addr;
            t->len = descs[i].len;
            t->options = 0;
            sent++;
            tx_bytes += descs[i].len;
        } else {
            if (verdict[i] == XSK_GPU_TX_REPLY) r->tx_full++;
            pool_push(pool, descs[i].addr); /* :226-227 */
        }
    }
    if (sent) xr_prod_submit(tx, sent);
    r->replied += sent;
    if (stats) {
        stats->rx_packets += n;        /* :233 */
        stats->rx_bytes += rx_bytes;   /* :229 */
        stats->tx_packets += sent;     /* :172 */
        stats->tx_bytes += tx_bytes;   /* :171 */
    }
}

int xsk_gpu_rx_step(xsk_gpu_ctx* ctx, struct xsk_gpu_ring* rx, struct xsk_gpu_ring* fill, struct xsk_gpu_ring* tx,
                    struct xsk_gpu_frame_pool* pool, uint32_t max_batch, struct xsk_gpu_stats* stats,
                    struct xsk_gpu_rx_result* res) {
    struct xsk_gpu_desc descs[XSK_GPU_RX_MAX_STEP];
    uint8_t verdict[XSK_GPU_RX_MAX_STEP];
    struct xsk_gpu_rx_result r = {0, 0, 0, 0};
    if (!ctx || !rx || !fill || !tx || !pool || !pool->addr || max_batch == 0) return -EINVAL;
    if (max_batch > XSK_GPU_RX_MAX_STEP) max_batch = XSK_GPU_RX_MAX_STEP;
    if (!xr_cons_avail(rx, 1)) { /* nothing received: the context is not even looked at */
        if (res) *res = r;
        return 0;
    }
    /* never peek more than the context takes: xsk_gpu_process would refuse the batch after the fill
       ring had been restocked, and a caller retrying the step would spin on the same error */
    if (max_batch > xsk_gpu__ctx_max_batch(ctx)) max_batch = xsk_gpu__ctx_max_batch(ctx);

    uint32_t idx_rx = 0;
    const uint32_t rcvd = xr_cons_peek(rx, max_batch, &idx_rx); /* :196 */
    r.refilled = xsk_gpu__rx_refill(fill, pool);                /* :201-217 */
    /* :222-223 — the batch's descriptors */
    for (uint32_t i = 0; i < rcvd; i++) descs[i] = *xr_desc(rx, idx_rx + i);

    const int rc = xsk_gpu_process(ctx, descs, rcvd, verdict, NULL, NULL);
    if (rc) {
        if (xsk_gpu__failed_untouched(ctx)) { /* frames stay on the RX ring (not released): the caller may retry */
            rx->cached_cons -= rcvd;
            return rc;
        }
        /* some frames may have been transformed: a retry would transform them twice (a reply reads as
         * DROP_NOT_ECHO), so the batch is dropped -- its frames go back to the pool, none is transmitted */
        xsk_gpu__rx_drop(descs, rcvd, pool);
        xr_cons_release(rx, rcvd);
        r.received = rcvd;
        if (res) *res = r;
        return rc;
    }
    xsk_gpu__rx_emit(descs, verdict, rcvd, tx, pool, stats, &r);
    xr_cons_release(rx, rcvd); /* :232 */
    r.received = rcvd;
    if (res) *res = r;
    return (int)rcvd;
}

uint32_t xsk_gpu_tx_complete(struct xsk_gpu_ring* comp, struct xsk_gpu_frame_pool* pool, uint32_t max) {
    if (!comp || !pool || !pool->addr || max == 0) return 0;
    uint32_t idx = 0;
    const uint32_t n = xr_cons_peek(comp, max, &idx); /* :89 */
    for (uint32_t i = 0; i < n; i++) pool_push(pool, *xr_addr(comp, idx + i)); /* :94-95 */
    if (n) xr_cons_release(comp, n); /* :97 */
    return n;
}

int xsk_gpu_stats_tx_failed(struct xsk_gpu_stats* stats, const struct xsk_gpu_desc* descs, const uint8_t* verdicts,
                            const uint8_t* sent, uint32_t n) {
    if (!stats || (n && (!descs || !verdicts || !sent))) return -EINVAL;
    uint64_t p = 0, b = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (verdicts[i] == XSK_GPU_TX_REPLY && !sent[i]) { /* xsk_receive.c:166-170: no count on a failed send */
            p++;
            b += descs[i].len;
        }
    }
    if (p > stats->tx_packets || b > stats->tx_bytes) return -EINVAL; /* not frames these counters counted */
    stats->tx_packets -= p;
    stats->tx_bytes -= b;
    return (int)(p > 0x7FFFFFFFu ? 0x7FFFFFFF : p);
}
