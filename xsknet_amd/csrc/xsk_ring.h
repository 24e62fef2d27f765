/*
 * xsk_ring.h — single-producer / single-consumer AF_XDP ring operations over struct xsk_gpu_ring
 * (the field layout of libxdp's struct xsk_ring_prod / xsk_ring_cons).  Semantics follow the Linux
 * AF_XDP ring protocol the reference drives through libxdp (src/lib/xsk_receive.c:196, :206-217,
 * :222-223, :232, and the commented TX path :174-186): free-running 32-bit producer/consumer
 * indices, entry i lives at ring[i & mask], the producer index is published with release semantics
 * and read with acquire semantics (and vice versa for the consumer index).
 *
 * Host code only (C11).  Used by xsk_gpu_rx.c; unit-tested on the CPU by tests/c/test_ring.c.
 */
#ifndef XSK_RING_H
#define XSK_RING_H

#include <stdint.h>

#include "../../include/xsk_gpu.h"

/* Entries available to a consumer (refreshes the cached producer when the cache is empty). */
static inline uint32_t xr_cons_avail(struct xsk_gpu_ring* r, uint32_t want) {
    uint32_t n = r->cached_prod - r->cached_cons;
    if (n == 0) {
        r->cached_prod = __atomic_load_n(r->producer, __ATOMIC_ACQUIRE);
        n = r->cached_prod - r->cached_cons;
    }
    return n < want ? n : want;
}

/* Peek up to `want` entries: returns the count and the first index (xsk_ring_cons__peek). */
static inline uint32_t xr_cons_peek(struct xsk_gpu_ring* r, uint32_t want, uint32_t* idx) {
    const uint32_t n = xr_cons_avail(r, want);
    if (n) {
        *idx = r->cached_cons;
        r->cached_cons += n;
    }
    return n;
}

/* Give `n` peeked entries back to the producer (xsk_ring_cons__release). */
static inline void xr_cons_release(struct xsk_gpu_ring* r, uint32_t n) {
    __atomic_store_n(r->consumer, *r->consumer + n, __ATOMIC_RELEASE);
}

/* Free slots a producer may fill (refreshes the cached consumer when short; xsk_prod_nb_free). */
static inline uint32_t xr_prod_free(struct xsk_gpu_ring* r, uint32_t want) {
    uint32_t f = r->cached_cons - r->cached_prod;
    if (f < want) {
        r->cached_cons = __atomic_load_n(r->consumer, __ATOMIC_ACQUIRE) + r->size;
        f = r->cached_cons - r->cached_prod;
    }
    return f;
}

/* Reserve exactly `n` slots or none (xsk_ring_prod__reserve). */
static inline uint32_t xr_prod_reserve(struct xsk_gpu_ring* r, uint32_t n, uint32_t* idx) {
    if (xr_prod_free(r, n) < n) return 0;
    *idx = r->cached_prod;
    r->cached_prod += n;
    return n;
}

/* Publish `n` reserved slots (xsk_ring_prod__submit). */
static inline void xr_prod_submit(struct xsk_gpu_ring* r, uint32_t n) {
    __atomic_store_n(r->producer, *r->producer + n, __ATOMIC_RELEASE);
}

static inline struct xsk_gpu_desc* xr_desc(struct xsk_gpu_ring* r, uint32_t idx) {
    return &((struct xsk_gpu_desc*)r->ring)[idx & r->mask];
}
static inline uint64_t* xr_addr(struct xsk_gpu_ring* r, uint32_t idx) {
    return &((uint64_t*)r->ring)[idx & r->mask];
}

#endif
