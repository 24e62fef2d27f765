/* CPU unit test of STAGED mode's copy-in planner (xsk_gpu__stage_plan, xsknet_amd/csrc/xsk_stage_plan.h): the path
 * each layout takes and whether its copy-in is contained (may run beside earlier chunks' transforms).  Built and run by
 * tests/test_staged_plan.py, which also builds this file as a shared library (-DSHIM) to compare the planner with the
 * Python restatement in tests/staged_plan.py on random layouts. */
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_stage_plan.h"

/* the planner as a flat function for ctypes: out = kind, contained, aligned, lo, hi, base, stride, width, sum */
int xsk_test_stage_plan(const struct xsk_gpu_desc* d, uint32_t n, uint64_t umem_size, int wire, int have_alias,
                        int prefix_aligned, uint64_t out[9]) {
    const struct xsk_stage_plan p = xsk_gpu__stage_plan(d, n, umem_size, wire, have_alias, prefix_aligned);
    out[0] = (uint64_t)p.kind;
    out[1] = (uint64_t)p.contained;
    out[2] = p.aligned;
    out[3] = p.lo;
    out[4] = p.hi;
    out[5] = p.base;
    out[6] = p.stride;
    out[7] = p.width;
    out[8] = p.sum;
    return 0;
}

#ifndef SHIM
#define N 40000u
static struct xsk_gpu_desc d[N];

int main(void) {
    const uint64_t U = 1ull << 30;
    /* 1. aligned frames at a 2 KiB stride in a scrambled order (recycled RX addresses), ragged lengths: the gather
     *    kernel; contained (every span ends inside its frame's 16-B rounded bytes) */
    for (uint32_t i = 0; i < N; i++) {
        d[i].addr = (uint64_t)((i * 7919u) % N) * 2048u;
        d[i].len = 64u + (i * 37u) % 1437u;
    }
    struct xsk_stage_plan p = xsk_gpu__stage_plan(d, N, U, 0, 1, 1);
    assert(p.kind == XSK_STAGE_GATHER && p.contained && p.aligned);
    /* ... unless an earlier chunk of the call had an unaligned frame: an aligned frame's span end (rounded up to 16)
     * may then reach the first bytes of an unaligned neighbour that chunk is rewriting */
    p = xsk_gpu__stage_plan(d, N, U, 0, 1, 0);
    assert(p.kind == XSK_STAGE_GATHER && !p.contained && p.aligned);
    /* ... and without a mapped alias: the host pack, same containment */
    p = xsk_gpu__stage_plan(d, N, U, 0, 0, 1);
    assert(p.kind == XSK_STAGE_HOSTPACK && p.contained);
    /* 2. packed odd lengths (1537..1551 B back to back): unaligned frames, never contained */
    uint64_t a = 0;
    for (uint32_t i = 0; i < N; i++) {
        d[i].addr = a;
        d[i].len = 1537u + i % 15u;
        a += d[i].len;
    }
    p = xsk_gpu__stage_plan(d, N, U, 0, 1, 1);
    assert(!p.aligned && !p.contained && p.kind == XSK_STAGE_SPAN); /* dense: the span copy */
    /* only the aligned-start frames of that layout, as a later chunk: aligned, but after unaligned chunks */
    uint32_t k = 0;
    a = 0;
    for (uint32_t i = 0; i < N && k < 2000; i++) {
        const uint32_t ln = 1537u + i % 15u;
        if ((a & 15u) == 0) {
            d[k].addr = a;
            d[k].len = ln;
            k++;
        }
        a += ln;
    }
    p = xsk_gpu__stage_plan(d, k, U, 0, 1, 0);
    assert(p.aligned && !p.contained); /* (periodic lengths: a uniform stride, the 2-D copy) */
    p = xsk_gpu__stage_plan(d, k, U, 0, 1, 1); /* (a call whose earlier chunks were all aligned: contained) */
    assert(p.contained);
    /* 3. aligned 64-B frames at a 64-B pitch, every other frame, both modes (one 64-B window each): contained;
     *    50-B frames (own 64 B): still contained; with a 32-B unaligned neighbour in an earlier chunk: not */
    for (uint32_t i = 0; i < 3000; i++) {
        d[i].addr = (uint64_t)(2 * ((i * 1999u) % 3000u)) * 64u;
        d[i].len = 64u;
    }
    for (int wire = 0; wire < 2; wire++) {
        p = xsk_gpu__stage_plan(d, 3000, U, wire, 1, 1);
        assert(p.kind == XSK_STAGE_GATHER && p.contained && p.sum == 3000u * 64u);
    }
    for (uint32_t i = 0; i < 3000; i++) d[i].len = 50u;
    p = xsk_gpu__stage_plan(d, 3000, U, 1, 1, 1);
    assert(p.kind == XSK_STAGE_GATHER && p.contained);
    p = xsk_gpu__stage_plan(d, 3000, U, 1, 1, 0);
    assert(!p.contained);
    /* 4. a uniform 2 KiB stride of 1500-B frames: one 2-D copy, contained */
    for (uint32_t i = 0; i < 5000; i++) {
        d[i].addr = 4096u + (uint64_t)i * 2048u;
        d[i].len = 1500u;
    }
    p = xsk_gpu__stage_plan(d, 5000, U, 0, 1, 1);
    assert(p.kind == XSK_STAGE_2D && p.contained && p.width == 1504u && p.stride == 2048u);
    /* with 10 % of the frames 150 B shorter: still the 2-D copy (within budget), but its rows run past the short
     * frames' bytes into the stride gap, where another chunk's frame may lie: not contained */
    for (uint32_t i = 0; i < 5000; i += 10) d[i].len = 1350u;
    p = xsk_gpu__stage_plan(d, 5000, U, 0, 1, 1);
    assert(p.kind == XSK_STAGE_2D && !p.contained);
    /* without the alias the 2-D copy stays (a DMA copy needs none) */
    p = xsk_gpu__stage_plan(d, 5000, U, 0, 0, 1);
    assert(p.kind == XSK_STAGE_2D && !p.contained);
    /* 5. an RX-loop batch (64 frames) scattered over the C1 UMEM: gather with the alias, host pack without (never the
     *    whole span, which round 4's fallback copied) */
    for (uint32_t i = 0; i < 64; i++) {
        d[i].addr = 256u + (uint64_t)((i * 1997u) % 4096u) * 4096u;
        d[i].len = 64u;
    }
    p = xsk_gpu__stage_plan(d, 64, 16u << 20, 0, 1, 1);
    assert(p.kind == XSK_STAGE_GATHER && p.contained && p.sum == 64u * 64u);
    p = xsk_gpu__stage_plan(d, 64, 16u << 20, 0, 0, 1);
    assert(p.kind == XSK_STAGE_HOSTPACK && p.contained);
    /* 6. short frames only (len < 20: nothing read): contained, no copy */
    for (uint32_t i = 0; i < 10; i++) {
        d[i].addr = (uint64_t)i * 64u + 3u;
        d[i].len = 10u;
    }
    p = xsk_gpu__stage_plan(d, 10, U, 0, 1, 1);
    assert(p.kind == XSK_STAGE_NONE && p.contained && p.sum == 0 && !p.aligned);
    /* 7. the host pack's partition into staging halves: every frame in exactly one half, each half within its bytes,
     *    at least one frame per half, frames too large for a half carried without bytes */
    {
        uint64_t seed = 12345;
        for (int t = 0; t < 200; t++) {
            const uint32_t n = 1u + (uint32_t)(seed % 3000u);
            const uint64_t half = 4096u << (seed % 8u);
            for (uint32_t i = 0; i < n; i++) {
                seed = seed * 6364136223846793005ull + 1442695040888963407ull;
                d[i].addr = (seed >> 20) % (1u << 29);
                d[i].len = (uint32_t)((seed >> 40) % (t % 3 == 0 ? 70000u : 1600u));
            }
            uint32_t f0 = 0, halves = 0;
            while (f0 < n) {
                uint64_t bytes = 0;
                const uint32_t f1 = xsk_gpu__hostpack_split(d, f0, n, U, t & 1, half, &bytes);
                assert(f1 > f0 && f1 <= n);
                uint64_t want = 0;
                for (uint32_t f = f0; f < f1; f++) {
                    uint64_t a16 = 0;
                    const uint64_t sp = xsk_gpu__read_span(d[f].addr, d[f].len, U, t & 1, &a16);
                    want += sp + 16u > half ? 0u : sp;
                }
                assert(bytes == want && ((((uint64_t)(f1 - f0) * 4u + 15u) & ~15ull) + bytes <= half));
                f0 = f1;
                halves++;
            }
            assert(halves >= 1);
        }
    }
    printf("stage plan ok\n");
    return 0;
}
#endif
