/*
 * xsk_lowlat_proto.h — host side of the LOWLAT doorbell protocol (C11 / C++, no HIP types): the shared
 * doorbell layout, the command word, the choice of resident workgroups per batch, and the post / wait /
 * recover state machine of one call.  The HIP plumbing (launch, stream query) comes in through callbacks,
 * so the state machine -- in particular its timeout and recovery paths -- is unit-tested on the CPU
 * (tests/c/test_lowlat_proto.c) against a simulated kernel.
 *
 * The reference hands its transform RX_BATCH_SIZE = 64 descriptors per poll() (src/lib/xsk_receive.c:196,
 * :251-257; src/lib/xsk_utils.h:8); xsk_lowlat.hip keeps XSK_GPU__LL_WG workgroups of the round kernel
 * resident so that such a batch costs a doorbell store and a spin instead of a launch and a stream sync.
 */
#ifndef XSK_LOWLAT_PROTO_H
#define XSK_LOWLAT_PROTO_H

#include <errno.h>
#include <stdint.h>

#include "../../include/xsk_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* xsk_gpu__ll_slice runs on both sides (the kernel computes its own slice): a host+device function when
 * compiled by hipcc, a plain C function in the C sources and the CPU unit test. */
#ifdef __HIPCC__
#define XSK_GPU__HOSTDEV __host__ __device__
#else
#define XSK_GPU__HOSTDEV
#endif

/* Resident workgroups of a LOWLAT channel (one CU each while it serves).  Workgroup 0 is the leader: it
 * polls the doorbell AND the first 64 descriptor slots, owns `alive`, and decides the idle exit; the others
 * poll the command word only and leave when the leader does. */
#define XSK_GPU__LL_WG 4u

/* Shared doorbell (mapped, fine-grained pinned host memory): every word the host spins on or the kernel
 * polls sits on a 64-byte line of its own. */
struct xsk_gpu__bell {
    /* host -> device: ONE 64-bit word, so a poll is one PCIe read:
     *   bits 0-31 seq (bumped by one per posted batch), 32-47 n (<= XSK_GPU_LOWLAT_MAX),
     *   bit 48 write records, bits 49-55 frames per wave / 4 (0: ceil(slice / 16)),
     *   bits 56-58 workgroups serving the batch (1..XSK_GPU__LL_WG), bit 63 stop (every workgroup exits at
     *   its next poll) */
    volatile uint64_t cmd;
    /* nonzero while another context of the process unregisters host memory (the runtime then waits for every stream
     * of the device): the leader reads it with `cmd` in one 16-B load and, idle, leaves (xsk_gpu__ll_yield_all).
     * Written by whichever thread raises or drops the request, never by the channel's owner. */
    volatile uint32_t yield;
    uint32_t pad0[13];
    /* the same words again in a line of their own: the leader keeps two polls in flight, one per copy (two
     * reads of ONE line do not overlap -- the second waits for the first) */
    volatile uint64_t cmd_b;
    volatile uint32_t yield_b;
    uint32_t pad0b[13];
    /* the same word once more for each other workgroup, a line each: reads of one host line from several CUs
     * queue behind each other, so workgroups polling the leader's lines slowed its sampling of the doorbell
     * from every ~0.7 us to every ~1.0-1.6 us */
    struct {
        volatile uint64_t cmd;
        uint32_t pad[14];
    } wcmd[XSK_GPU__LL_WG - 1];
    /* device -> host, one line per workgroup: seq of the last batch it completed (its slice written back);
     * wg[0].alive = 1 while the leader runs; cancel = seq of a batch the workgroup found already cancelled (STOP
     * in the same command word) and retired WITHOUT serving it (then done == cancel too) */
    struct {
        volatile uint32_t done;
        volatile uint32_t alive;
        volatile uint32_t cancel;
        uint32_t pad[13];
    } wg[XSK_GPU__LL_WG];
};

#define XSK_GPU__BELL_N(n) ((uint64_t)(n) << 32)
#define XSK_GPU__BELL_RECS (1ull << 48)
#define XSK_GPU__BELL_TILE(q) ((uint64_t)((q) & 0x7Fu) << 49)
#define XSK_GPU__BELL_WG(w) ((uint64_t)((w) & 0x7u) << 56)
#define XSK_GPU__BELL_STOP (1ull << 63)

/* Workgroups for a doorbell batch.  A batch of <= 64 frames runs on the leader alone, whose poll already brought its
 * descriptors, and so does one of <= 128 frames and <= 16 KiB (minimum-size frames: a second workgroup's own doorbell
 * line and barrier cost more than it streams).  Any larger batch runs on all XSK_GPU__LL_WG: one CU caps the PCIe reads
 * of a batch (its waves have only so many loads in flight), and in round 5's sweep (tools/hostlat.py --groups 1-4,
 * 64 / 512 / 1500-B frames x 64-1024 per batch, profiles/r05/lowlat_groups.jsonl) four workgroups were within 1 us of
 * the best count everywhere above that line while round 4's rule (one per 256 frames or 256 KiB) lost up to 4 us there:
 * 128 x 1500 B 20.5 -> 17.5 us, 256 x 512 B 19.2 -> 15.6, 256 x 64 B 12.1 -> 10.5. */
static inline uint32_t xsk_gpu__ll_groups(const struct xsk_gpu_desc* d, uint32_t n) {
    if (n <= 64u) return 1u;
    if (n <= 128u) {
        uint64_t bytes = 0;
        for (uint32_t i = 0; i < n; i++) bytes += d[i].len < 4096u ? d[i].len : 4096u;
        if (bytes <= (16u << 10)) return 1u;
    }
    return XSK_GPU__LL_WG;
}

/* Frames of workgroup g's slice of an n-frame batch over w workgroups: contiguous, a multiple of 4 frames
 * (one 16-lane row per frame and step) except the last. */
static inline XSK_GPU__HOSTDEV void xsk_gpu__ll_slice(uint32_t n, uint32_t w, uint32_t g, uint32_t* f0, uint32_t* f1) {
    uint32_t per = (n + w - 1u) / w;
    per = (per + 3u) & ~3u;
    const uint32_t a = g * per < n ? g * per : n;
    *f0 = a;
    *f1 = a + per < n ? a + per : n;
}

/* Callbacks into the HIP side (xsk_lowlat.hip) or a simulation (tests/c/test_lowlat_proto.c). */
struct xsk_gpu__ll_ops {
    void* u;
    int (*launch)(void* u);      /* enqueue one instance of the resident grid on its stream: 0 or -errno */
    int (*stream_idle)(void* u); /* 1: no instance is running or queued on the stream */
    double (*now)(void* u);      /* seconds, monotonic */
    void (*relax)(void* u);      /* one spin-wait step */
};

struct xsk_gpu__ll_state {
    struct xsk_gpu__bell* bell;
    uint32_t seq;         /* last posted batch */
    uint64_t cmd;         /* its whole command word (a STOP keeps its n / workgroup fields) */
    uint32_t stop_unserved; /* the last ll_stop that found the grid stopped: xsk_gpu__ll_unserved of the last batch */
    int launched;         /* an instance was launched and may still run */
    int broken;           /* a timed-out batch whose instance had not stopped when the call returned */
    double timeout_s;     /* a batch not complete after this long: -ETIMEDOUT */
    double quiesce_s;     /* after a timeout, how long to wait for the instance to stop */
    double recheck_s;     /* while waiting, how often to check that an instance is still there */
    int inflight;         /* xsk_gpu__ll_begin posted seq and xsk_gpu__ll_wait has not returned for it yet */
    int last_late;        /* the last xsk_gpu__ll_wait returned 0 for a batch that had missed its timeout (STOP posted,
                           * every slice found served once the grid stopped): a late completion */
    uint32_t w_post;      /* its serving workgroups */
    double t_post;        /* when it was posted */
};

static inline void xsk_gpu__ll_post(struct xsk_gpu__bell* b, uint64_t c) {
    for (uint32_t g = 0; g + 1 < XSK_GPU__LL_WG; g++) __atomic_store_n(&b->wcmd[g].cmd, c, __ATOMIC_SEQ_CST);
    __atomic_store_n(&b->cmd_b, c, __ATOMIC_SEQ_CST);
    __atomic_store_n(&b->cmd, c, __ATOMIC_SEQ_CST);
}

/* No instance runs (its stream is idle): retire the last posted batch for every workgroup, so that a relaunched grid
 * -- whose workgroups take their baselines from `done` -- never serves a batch whose call has already returned
 * (the launch re-posts the command word without its STOP bit). */
static inline void xsk_gpu__ll_retire(struct xsk_gpu__ll_state* st) {
    for (uint32_t g = 0; g < XSK_GPU__LL_WG; g++) __atomic_store_n(&st->bell->wg[g].done, st->seq, __ATOMIC_SEQ_CST);
}

/* Slices of the last posted batch (w serving workgroups) that were NOT transformed: bit g set when workgroup g never
 * completed seq or retired it unserved (cancel == seq).  Meaningful once no instance runs. */
static inline uint32_t xsk_gpu__ll_unserved(const struct xsk_gpu__bell* b, uint32_t seq, uint32_t w) {
    uint32_t m = 0;
    for (uint32_t g = 0; g < w; g++)
        if (__atomic_load_n(&b->wg[g].done, __ATOMIC_ACQUIRE) != seq ||
            __atomic_load_n(&b->wg[g].cancel, __ATOMIC_ACQUIRE) == seq)
            m |= 1u << g;
    return m;
}

/* Stop the resident grid (xsk_gpu_fini, a large batch, new options, a timeout): post STOP in the last command
 * word (its seq, n and workgroup fields kept, so a workgroup that has not taken that batch yet retires exactly its
 * own slice unserved), and wait up to `wait_s` (< 0: for ever) for the stream to drain.  Returns 0 once no instance
 * runs -- the last batch then retired for every workgroup -- or -ETIMEDOUT if one still did at the deadline (the
 * channel is then `broken`).  A batch still in flight (posted, not waited for) ends here: stop_unserved says what was
 * done with it. */
static inline int xsk_gpu__ll_stop(struct xsk_gpu__ll_state* st, const struct xsk_gpu__ll_ops* ops, double wait_s) {
    st->inflight = 0;
    if (!st->launched && !st->broken) return 0;
    xsk_gpu__ll_post(st->bell, (st->cmd & ~0xFFFFFFFFull) | (uint64_t)st->seq | XSK_GPU__BELL_STOP);
    const double t0 = ops->now(ops->u);
    for (;;) {
        if (ops->stream_idle(ops->u)) {
            uint32_t w = (uint32_t)(st->cmd >> 56) & 7u;
            w = w < 1u ? 1u : (w > XSK_GPU__LL_WG ? XSK_GPU__LL_WG : w);
            st->stop_unserved = xsk_gpu__ll_unserved(st->bell, st->seq, w); /* what the workgroups did, then: */
            xsk_gpu__ll_retire(st);
            st->launched = 0;
            st->broken = 0;
            return 0;
        }
        if (wait_s >= 0 && ops->now(ops->u) - t0 > wait_s) {
            st->broken = 1;
            return -ETIMEDOUT;
        }
        ops->relax(ops->u);
    }
}

/* One doorbell batch, in two halves (xsk_gpu__ll_run = begin + wait; a caller with several channels keeps one batch in
 * flight on each -- the pipelined RX loop, xsk_gpu_pipe.c).
 *
 * xsk_gpu__ll_begin posts it: the caller has written the descriptors (slots 0 .. n-1, the `options` of the first 64
 * tagged with seq + 1, the seq this call posts) into the mapped buffer.  `bits` = the n / records / tile fields; w =
 * serving workgroups.  Returns 0 when the batch is posted (then xsk_gpu__ll_wait must follow before anything else is
 * posted on this channel), or:
 *   -EBUSY      an earlier batch timed out and its instance has still not stopped, or a batch is still in flight:
 *               nothing was posted;
 *   a launch error.
 *
 * xsk_gpu__ll_wait returns 0 when every serving workgroup has published completion (the caller's outputs are then
 * in the mapped buffers), or:
 *   -ETIMEDOUT  the batch did not complete within timeout_s of its post: STOP was posted and the instance waited for
 *               (quiesce_s).  Once it has stopped, every slice is either transformed exactly once or untouched
 *               (a workgroup that finds STOP with a batch it has not taken retires it unserved), *unserved says
 *               which slices are untouched (bit g: slice g of xsk_gpu__ll_slice), and no later instance serves the
 *               batch; if every slice turned out to be served the call returns 0 after all.  If the instance had not
 *               stopped by then, the channel stays `broken`, *unserved has every bit set (unknown), and later posts
 *               return -EBUSY until it has;
 *   -EINVAL     nothing in flight;
 *   a launch error. */
static inline int xsk_gpu__ll_begin(struct xsk_gpu__ll_state* st, const struct xsk_gpu__ll_ops* ops, uint64_t bits,
                                    uint32_t w) {
    struct xsk_gpu__bell* b = st->bell;
    if (st->inflight) return -EBUSY;
    if (st->broken) {
        if (!ops->stream_idle(ops->u)) return -EBUSY;
        xsk_gpu__ll_retire(st); /* the stopped instance's batch is never served by a relaunch */
        st->broken = 0;
        st->launched = 0;
    }
    int fresh = 0; /* an instance launched by this call: it takes its baselines from `done` and serves seq */
    if (!st->launched || !__atomic_load_n(&b->wg[0].alive, __ATOMIC_SEQ_CST)) {
        /* gone (idle exit) or never started: launch; stream order puts it behind an exiting instance */
        const int rc = ops->launch(ops->u);
        if (rc) return rc;
        st->launched = 1;
        fresh = 1;
    }
    const uint32_t seq = st->seq + 1u;
    st->seq = seq;
    st->cmd = (uint64_t)seq | bits | XSK_GPU__BELL_WG(w);
    xsk_gpu__ll_post(b, st->cmd);
    if (!fresh && !__atomic_load_n(&b->wg[0].alive, __ATOMIC_SEQ_CST)) {
        /* the leader was leaving (Dekker: it re-reads the doorbell after clearing alive, or this launch serves
         * the batch) */
        const int rc = ops->launch(ops->u);
        if (rc) {
            /* posted, and the leader may still have seen it before leaving: the outcome is unknown, so the channel is
             * broken -- nothing is posted until no instance runs, and then the batch is retired, never served by a
             * later relaunch behind the caller's back */
            st->broken = 1;
            return rc;
        }
    }
    st->inflight = 1;
    st->w_post = w;
    st->t_post = ops->now(ops->u);
    return 0;
}

/* The batch in flight is complete (never blocks; 0 while it is not or when nothing is in flight). */
static inline int xsk_gpu__ll_ready(const struct xsk_gpu__ll_state* st) {
    if (!st->inflight) return 0;
    for (uint32_t g = 0; g < st->w_post; g++)
        if (__atomic_load_n(&st->bell->wg[g].done, __ATOMIC_ACQUIRE) != st->seq) return 0;
    return 1;
}

static inline int xsk_gpu__ll_wait(struct xsk_gpu__ll_state* st, const struct xsk_gpu__ll_ops* ops,
                                   uint32_t* unserved) {
    struct xsk_gpu__bell* b = st->bell;
    if (unserved) *unserved = 0;
    st->last_late = 0;
    if (!st->inflight) return -EINVAL;
    st->inflight = 0; /* whatever happens below, the batch leaves the channel's hands */
    const uint32_t seq = st->seq, w = st->w_post;
    const double t_post = st->t_post;
    double t_check = t_post;
    for (uint32_t spin = 0;; ++spin) {
        uint32_t g = 0;
        while (g < w && __atomic_load_n(&b->wg[g].done, __ATOMIC_ACQUIRE) == seq) ++g;
        if (g == w) break;
        if ((spin & 255u) == 255u) {
            const double t = ops->now(ops->u);
            if (t - t_check > st->recheck_s) {
                t_check = t;
                /* every instance has exited without serving the batch: serve it now (a relaunched grid takes
                 * each workgroup's baseline from its `done`, so nothing is served twice) */
                if (ops->stream_idle(ops->u)) {
                    uint32_t h = 0;
                    while (h < w && __atomic_load_n(&b->wg[h].done, __ATOMIC_ACQUIRE) == seq) ++h;
                    if (h < w) {
                        const int rc = ops->launch(ops->u);
                        if (rc) return rc;
                    }
                }
            }
            if (t - t_post > st->timeout_s) {
                if (xsk_gpu__ll_stop(st, ops, st->quiesce_s) != 0) { /* still running: broken, outcome unknown */
                    if (unserved) *unserved = (1u << w) - 1u;
                    return -ETIMEDOUT;
                }
                /* (ll_stop recorded what the workgroups did with the batch before it retired it) */
                if (unserved) *unserved = st->stop_unserved;
                if (st->stop_unserved) return -ETIMEDOUT;
                st->last_late = 1;
                break; /* every slice was served, late: a normal completion */
            }
        }
        ops->relax(ops->u);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return 0;
}

/* Post one batch and wait for it (the returns of both halves above). */
static inline int xsk_gpu__ll_run(struct xsk_gpu__ll_state* st, const struct xsk_gpu__ll_ops* ops, uint64_t bits,
                                  uint32_t w, uint32_t* unserved) {
    if (unserved) *unserved = 0;
    const int rc = xsk_gpu__ll_begin(st, ops, bits, w);
    if (rc) return rc;
    return xsk_gpu__ll_wait(st, ops, unserved);
}

#ifdef __cplusplus
}
#endif

#endif /* XSK_LOWLAT_PROTO_H */
