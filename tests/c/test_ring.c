/* CPU unit test of the AF_XDP ring operations (xsknet_amd/csrc/xsk_ring.h): free-running 32-bit
 * indices across the 2^32 wrap, peek/release, reserve/submit at full and empty rings, and the
 * libxdp struct xsk_ring_prod/cons field layout.  Built and run by tests/test_ring.py. */
#include <assert.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_ring.h"

_Static_assert(offsetof(struct xsk_gpu_ring, cached_prod) == 0, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, cached_cons) == 4, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, mask) == 8, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, size) == 12, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, producer) == 16, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, consumer) == 24, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, ring) == 32, "layout");
_Static_assert(offsetof(struct xsk_gpu_ring, flags) == 40, "layout");
_Static_assert(sizeof(struct xsk_gpu_ring) == 48, "layout");

#define SZ 8u

int main(void) {
    /* one shared ring, a producer view and a consumer view, indices about to wrap */
    uint32_t prod = 0xFFFFFFFAu, cons = 0xFFFFFFFAu;
    uint64_t slots[SZ];
    memset(slots, 0, sizeof slots);
    struct xsk_gpu_ring p = {prod, cons + SZ, SZ - 1, SZ, &prod, &cons, slots, NULL};
    struct xsk_gpu_ring c = {prod, cons, SZ - 1, SZ, &prod, &cons, slots, NULL};
    uint32_t idx = 0, got = 0;
    uint64_t next_in = 100, next_out = 100;
    for (int round = 0; round < 50; round++) {
        /* producer: fill as much as possible, in two reservations */
        const uint32_t free1 = xr_prod_free(&p, 1);
        assert(free1 <= SZ);
        uint32_t want = free1 / 2 + 1;
        if (want > free1) want = free1;
        if (want && xr_prod_reserve(&p, want, &idx) == want) {
            for (uint32_t i = 0; i < want; i++) *xr_addr(&p, idx + i) = next_in++;
            xr_prod_submit(&p, want);
        }
        assert(xr_prod_reserve(&p, SZ + 1, &idx) == 0); /* never more than the ring */
        /* consumer: take up to 3 per round */
        const uint32_t n = xr_cons_peek(&c, 3, &idx);
        for (uint32_t i = 0; i < n; i++) assert(*xr_addr(&c, idx + i) == next_out++);
        if (n) xr_cons_release(&c, n);
        got += n;
        assert(prod - cons <= SZ);
    }
    assert(got > 50 && prod < 0x1000); /* indices wrapped past 2^32 */
    /* drain */
    uint32_t n;
    while ((n = xr_cons_peek(&c, SZ, &idx)) != 0) {
        for (uint32_t i = 0; i < n; i++) assert(*xr_addr(&c, idx + i) == next_out++);
        xr_cons_release(&c, n);
    }
    assert(next_out == next_in && prod == cons);
    /* an empty consumer sees nothing; a full producer gets nothing */
    assert(xr_cons_peek(&c, 4, &idx) == 0);
    assert(xr_prod_reserve(&p, SZ, &idx) == SZ);
    xr_prod_submit(&p, SZ);
    assert(xr_prod_reserve(&p, 1, &idx) == 0);
    /* descriptor rings index 16-B entries */
    struct xsk_gpu_desc d[4];
    struct xsk_gpu_ring dr = {0, 0, 3, 4, &prod, &cons, d, NULL};
    xr_desc(&dr, 6)->addr = 42;
    assert(d[2].addr == 42);
    printf("ring ok: %u entries through the wrap\n", (unsigned)got);
    return 0;
}
