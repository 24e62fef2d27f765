/*
 * xsk_stage_plan.h — STAGED host mode's copy-in planner (pure C11, no HIP): which path moves a chunk's bytes into the
 * device mirror, and whether that copy-in may run while earlier chunks of the same call are still being transformed.
 * xsk_gpu_host.c enqueues what it decides; tests/c/test_stage_plan.c and tests/staged_plan.py check it on the CPU.
 *
 * The reference recycles UMEM frames through a LIFO free stack (src/lib/xsk_receive.c:55-71, refilled at :201-217,
 * freed at :226-227), so an RX batch's addresses scatter over the UMEM after the first wrap; the planner must bound the
 * bytes moved whatever the layout (never more than 1.1 x the frames' read spans, xsk_gpu__read_span).
 */
#ifndef XSK_STAGE_PLAN_H
#define XSK_STAGE_PLAN_H

#include "xsk_gpu_internal.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    XSK_STAGE_NONE = 0,   /* the transform reads nothing of any frame */
    XSK_STAGE_2D = 1,     /* one strided 2-D DMA copy: a uniform stride whose rows carry <= 1.1 x the spans */
    XSK_STAGE_SPAN = 2,   /* one DMA copy of [lo, hi): the frames cover it to within 10 % */
    XSK_STAGE_GATHER = 3, /* the gather kernel reads every frame's span through the UMEM's mapped device alias */
    XSK_STAGE_HOSTPACK = 4 /* no mapped alias on this device: the host packs the spans into pinned staging, one DMA
                            * copy per staging half, and an unpack kernel puts each span at its offset in the mirror */
};

struct xsk_stage_plan {
    int kind;
    /* The copy-in writes mirror bytes of this chunk's own frames only -- [addr, align16(addr + max(len, 64))) of each
     * frame -- and every frame of the call up to this chunk starts 16-B aligned.  Then no byte it writes can belong to a
     * frame of an EARLIER chunk (whose transform may be rewriting that frame's header in the mirror right now, before
     * its pack reads it): such a frame starts at an aligned address outside this chunk's frames' owned bytes (the ABI's
     * ownership contract, include/xsk_gpu.h), so at or after align16(end) of any of them.  Only a contained copy-in may
     * run beside other chunks' transforms; any other waits for the previous chunk's header pack. */
    int contained;
    uint32_t aligned; /* every frame of this chunk starts 16-B aligned */
    uint64_t lo, hi, base, stride, width, sum;
};

/* Uniform stride S (>= 64, multiple of 16) when addr[i] = addr[0] + i*S for the whole chunk, else 0. */
static inline uint64_t xsk_gpu__uniform_stride(const struct xsk_gpu_desc* d, uint32_t n) {
    if (n < 2) return 0;
    if (d[1].addr <= d[0].addr) return 0;
    const uint64_t s = d[1].addr - d[0].addr;
    if (s < 64 || (s & 15u)) return 0;
    for (uint32_t i = 2; i < n; i++)
        if (d[i].addr != d[0].addr + (uint64_t)i * s) return 0;
    return s;
}

/* Plan chunk d[0..n) of a call.  wire: wire mode (frames parsed from 14 bytes on; the same 64-B windows); have_alias: the UMEM has a mapped device
 * alias on the context's device (the gather kernel's source); prefix_aligned: every frame of the call's EARLIER chunks
 * starts 16-B aligned.  The copy-in paths:
 *   - n <= XSK_GPU_LOWLAT_MAX (an RX-loop batch) with an alias: the gather kernel, whatever the layout (one launch beats a
 *     DMA submission there: profiles/r04/pass1/hostlat_*.jsonl);
 *   - a uniform frame stride whose rows carry at most 10 % more than the spans: one 2-D DMA copy;
 *   - frames covering [lo, hi) densely (at most 10 % of it between spans): one DMA copy of the span;
 *   - otherwise the gather kernel, or without an alias the host pack (never the whole span). */
static inline struct xsk_stage_plan xsk_gpu__stage_plan(const struct xsk_gpu_desc* d, uint32_t n, uint64_t umem_size,
                                                        int wire, int have_alias, int prefix_aligned) {
    struct xsk_stage_plan p;
    p.kind = XSK_STAGE_NONE;
    p.contained = 1;
    p.aligned = 1;
    p.lo = UINT64_MAX;
    p.hi = p.base = p.stride = p.width = p.sum = 0;
    uint64_t unaligned = 0, min_own = UINT64_MAX;
    int spans_own = 1; /* every parsed frame's span ends within align16(addr + max(len, 64)) */
    for (uint32_t i = 0; i < n; i++) {
        unaligned |= d[i].addr & 15u;
        const uint64_t ln = d[i].len;
        const uint64_t own = ((ln > 64u ? ln : 64u) + 15u) & ~15ull; /* bytes [addr, addr + own) are the frame's if
                                                                      * it is aligned (end rounded up to 16) */
        if (own < min_own) min_own = own;
        uint64_t a16 = 0;
        const uint64_t sp = xsk_gpu__read_span(d[i].addr, d[i].len, umem_size, wire, &a16);
        if (!sp) continue; /* the transform reads nothing of this frame */
        if (sp > own) spans_own = 0;
        if (a16 < p.lo) p.lo = a16;
        if (a16 + sp > p.hi) p.hi = a16 + sp;
        if (sp > p.width) p.width = sp;
        p.sum += sp;
    }
    p.aligned = unaligned == 0;
    const int prefix = prefix_aligned && p.aligned;
    if (!p.sum) return p; /* nothing copied: contained */
    const uint64_t budget = p.sum + p.sum / 10;
    p.stride = xsk_gpu__uniform_stride(d, n);
    p.base = d[0].addr & ~15ull;
    const int small = n <= XSK_GPU_LOWLAT_MAX && have_alias;
    const uint64_t s = p.stride;
    if (!small && s && p.width <= s && (uint64_t)n * p.width <= budget &&
        p.base + (uint64_t)(n - 1) * s + p.width <= umem_size) {
        p.kind = XSK_STAGE_2D;
        /* every row is `width` bytes from its frame's start: inside the frame only if width <= its own bytes */
        p.contained = prefix && p.width <= min_own;
    } else if (!small && p.hi - p.lo <= budget) {
        p.kind = XSK_STAGE_SPAN; /* covers whatever lies between the frames */
        p.contained = 0;
    } else {
        p.kind = have_alias ? XSK_STAGE_GATHER : XSK_STAGE_HOSTPACK;
        p.contained = prefix && spans_own;
    }
    return p;
}

/* XSK_STAGE_HOSTPACK's partition of a chunk into staging halves: the frames [f0, return value) whose u32 offsets table
 * (rounded up to 16 B) and read spans fit one half of `half` bytes.  A frame whose span cannot fit any half
 * (span + 16 > half) is counted with no bytes -- it takes a DMA copy of its own -- so a half always takes at least one
 * frame when f0 < n.  *bytes = the spans the half carries. */
static inline uint32_t xsk_gpu__hostpack_split(const struct xsk_gpu_desc* d, uint32_t f0, uint32_t n, uint64_t umem_size,
                                               int wire, uint64_t half, uint64_t* bytes) {
    uint32_t f1 = f0;
    uint64_t b = 0;
    for (; f1 < n; f1++) {
        uint64_t a16 = 0;
        const uint64_t sp = xsk_gpu__read_span(d[f1].addr, d[f1].len, umem_size, wire, &a16);
        const uint64_t x = sp + 16u > half ? 0u : sp;
        if ((((uint64_t)(f1 - f0 + 1) * 4u + 15u) & ~15ull) + b + x > half) break;
        b += x;
    }
    *bytes = b;
    return f1;
}

#ifdef __cplusplus
}
#endif

#endif /* XSK_STAGE_PLAN_H */
