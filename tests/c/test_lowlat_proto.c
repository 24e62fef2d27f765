/* CPU unit test of the LOWLAT doorbell protocol (xsknet_amd/csrc/xsk_lowlat_proto.h) against a simulated
 * resident grid that follows the kernel's order (xsk_lowlat.hip, poll_doorbell/examine): a workgroup that sees a new
 * batch with STOP in the same command word retires it unserved (cancel = done = seq) instead of serving it.
 * Cases: normal service over 1..4 workgroups, the leader's idle exit and the Dekker relaunch, an instance that exits
 * without serving, the timeout with nothing served (an instance still queued when the call gave up -- ADVICE r03),
 * with part of the batch served, with the batch finished by an instance that was inside its body (a late
 * completion: 0), the broken channel (-EBUSY until the instance has stopped, then recovery), the two halves of a call
 * (begin / wait) on two channels with a batch in flight on each, and in every case that no relaunched grid ever
 * serves a batch whose call has returned.  Built and run by tests/test_lowlat_proto.py. */
#include <assert.h>
#include <stdio.h>
#include <string.h>

#include "../../xsknet_amd/csrc/xsk_lowlat_proto.h"

/* The simulated device: `running` instances of the grid (the stream); served[g] = each workgroup's baseline (taken
 * from `done` at launch, as the kernel does).  Time advances by one tick per relax / now call. */
struct sim {
    struct xsk_gpu__bell bell;
    double t;
    int running;              /* instances running or queued */
    int launches;
    int serve_after;          /* relax steps before a running instance serves a posted batch (-1: never) */
    uint32_t serve_mask;      /* workgroups that serve before a STOP (bit g) */
    int mid_body;             /* on STOP, the serving workgroups are inside the body: they finish it (done, no cancel) */
    int stop_after;           /* relax steps a STOP takes to drain the stream (-1: never) */
    int exit_without_serving; /* the next instance exits at once, serving nothing */
    int countdown, stop_countdown;
    uint32_t served[XSK_GPU__LL_WG];
    int serves;               /* slices transformed, over the whole test */
};

static int sim_launch(void* u) {
    struct sim* s = (struct sim*)u;
    s->launches++;
    s->running++;
    s->countdown = s->serve_after;
    for (uint32_t g = 0; g < XSK_GPU__LL_WG; g++) s->served[g] = s->bell.wg[g].done; /* the kernel's baseline */
    __atomic_store_n(&s->bell.wg[0].alive, 1u, __ATOMIC_SEQ_CST);
    return 0;
}
static int sim_idle(void* u) { return ((struct sim*)u)->running == 0; }
static double sim_now(void* u) { return ((struct sim*)u)->t += 1e-6; }
static void sim_relax(void* u) {
    struct sim* s = (struct sim*)u;
    s->t += 1e-6;
    if (!s->running) return;
    if (s->exit_without_serving) {
        s->exit_without_serving = 0;
        s->running = 0;
        s->bell.wg[0].alive = 0;
        return;
    }
    const uint64_t c = s->bell.cmd;
    const uint32_t seq = (uint32_t)c;
    const int stop = (c & XSK_GPU__BELL_STOP) != 0;
    uint32_t w = (uint32_t)(c >> 56) & 7u;
    w = w ? w : 1u;
    const int due = s->serve_after >= 0 && s->countdown-- <= 0;
    for (uint32_t g = 0; g < XSK_GPU__LL_WG; g++) {
        if (s->served[g] == seq) continue;
        if (g >= w) { /* not serving this batch */
            s->served[g] = seq;
            continue;
        }
        if (stop && !s->mid_body) { /* the kernel's order: STOP before taking a batch -> retire it unserved */
            s->bell.wg[g].cancel = seq;
            s->bell.wg[g].done = seq;
            s->served[g] = seq;
            continue;
        }
        if ((stop && s->mid_body) || (due && ((s->serve_mask >> g) & 1u))) {
            s->bell.wg[g].done = seq;
            s->served[g] = seq;
            s->serves++;
        }
    }
    if (stop) {
        if (s->stop_countdown < 0) s->stop_countdown = 0;
        if (s->stop_after >= 0 && s->stop_countdown++ >= s->stop_after) {
            s->running = 0;
            s->bell.wg[0].alive = 0;
            s->stop_countdown = -1;
        }
    }
}

static struct xsk_gpu__ll_ops ops_of(struct sim* s) {
    struct xsk_gpu__ll_ops o = {s, sim_launch, sim_idle, sim_now, sim_relax};
    return o;
}

int main(void) {
    struct sim S;
    memset(&S, 0, sizeof S);
    S.stop_countdown = -1;
    S.serve_mask = 0xFu;
    struct xsk_gpu__ll_state st;
    memset(&st, 0, sizeof st);
    st.bell = &S.bell;
    st.timeout_s = 0.01; /* 10 000 ticks */
    st.quiesce_s = 0.005;
    st.recheck_s = 1e-4;
    struct xsk_gpu__ll_ops o = ops_of(&S);
    uint32_t un = 0xFFu;

    /* 1. normal service: the first call launches, later calls reuse the running grid */
    S.serve_after = 5;
    S.stop_after = 3;
    for (uint32_t w = 1; w <= XSK_GPU__LL_WG; w++) {
        assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64 * w), w, &un) == 0 && un == 0);
        for (uint32_t g = 0; g < w; g++) assert(S.bell.wg[g].done == st.seq);
    }
    assert(S.launches == 1 && st.seq == XSK_GPU__LL_WG && st.launched);
    assert(S.serves == 1 + 2 + 3 + 4);

    /* 2. the leader left (idle exit) before the post: relaunch, stream-ordered behind the old instance */
    S.bell.wg[0].alive = 0;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(10), 1, &un) == 0);
    assert(S.launches == 2);

    /* 3. an instance that exits without serving the batch: the periodic check relaunches it */
    S.running = 0;
    S.bell.wg[0].alive = 1; /* looked alive at the post */
    int before = S.launches;
    S.serve_after = 3;
    st.launched = 1;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(7), 1, &un) == 0);
    assert(S.launches == before + 1);

    /* 4. timeout with nothing served -- the instance was still queued (it never took the batch before the call gave
     *    up): it sees STOP with the batch and retires it unserved, so the call reports every slice
     *    untouched, the channel is not broken, and no relaunch serves that batch */
    S.serve_after = -1;
    S.stop_after = 10;
    S.stop_countdown = -1;
    int serves = S.serves;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64), 1, &un) == -ETIMEDOUT);
    assert(un == 1u && !st.broken && !st.launched && S.running == 0);
    assert((S.bell.cmd & XSK_GPU__BELL_STOP) && (uint32_t)S.bell.cmd == st.seq && ((S.bell.cmd >> 32) & 0xFFFFu) == 64);
    assert(S.bell.wg[0].cancel == st.seq && S.bell.wg[0].done == st.seq && S.serves == serves);
    /* the next call launches afresh (the launch re-posts the cancelled command without STOP: the new grid's baseline
     * is the retired seq, so only the new batch is served) */
    S.serve_after = 2;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64), 1, &un) == 0 && S.bell.wg[0].done == st.seq);
    assert(S.serves == serves + 1);

    /* 4b. the same on four workgroups, with workgroups 1-3 never having seen any batch (their `done` lags) */
    S.serve_after = -1;
    S.stop_after = 4;
    S.stop_countdown = -1;
    serves = S.serves;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(1024), 4, &un) == -ETIMEDOUT && un == 0xFu && !st.broken);
    for (uint32_t g = 0; g < 4; g++) assert(S.bell.wg[g].done == st.seq);
    S.serve_after = 1;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(1024), 4, &un) == 0 && un == 0 && S.serves == serves + 4);

    /* 5. timeout with part of the batch served: the leader served its slice, workgroup 1 never took its own before
     *    STOP -> -ETIMEDOUT, slice 1 untouched (the library finishes it through the launch path) */
    S.serve_after = 1;
    S.serve_mask = 0x1u;
    S.stop_after = 3;
    S.stop_countdown = -1;
    serves = S.serves;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(512), 2, &un) == -ETIMEDOUT);
    assert(un == 0x2u && !st.broken && S.serves == serves + 1);
    assert(S.bell.wg[1].cancel == st.seq && S.bell.wg[0].cancel != st.seq);
    S.serve_mask = 0xFu;

    /* 6. late completion: the serving workgroups were inside the body when STOP arrived; they finish (done, no
     *    cancel) and the call returns 0 -- every slice served exactly once */
    S.serve_after = -1;
    S.mid_body = 1;
    S.stop_after = 2;
    S.stop_countdown = -1;
    serves = S.serves;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(300), 3, &un) == 0 && un == 0 && S.serves == serves + 3);
    S.mid_body = 0;

    /* 7. timeout, the instance does NOT stop within quiesce_s: broken (outcome unknown: every bit); -EBUSY (nothing
     *    posted) until it does; then the stopped instance's batch is retired and never served by the relaunch */
    S.serve_after = -1;
    S.stop_after = -1;
    S.stop_countdown = -1;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64), 1, &un) == -ETIMEDOUT);
    assert(st.broken && S.running > 0 && un == 1u);
    const uint32_t seq_broken = st.seq;
    const uint64_t cmd_broken = S.bell.cmd;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64), 1, &un) == -EBUSY);
    assert(st.seq == seq_broken && S.bell.cmd == cmd_broken); /* nothing posted */
    S.running = 0; /* the instance finally stopped (without reaching the batch) */
    S.serve_after = 1;
    S.stop_after = 3;
    serves = S.serves;
    assert(xsk_gpu__ll_run(&st, &o, XSK_GPU__BELL_N(64), 1, &un) == 0);
    assert(!st.broken && st.seq == seq_broken + 1 && S.bell.wg[0].done == st.seq && S.serves == serves + 1);

    /* 8. stop: drains and clears */
    assert(xsk_gpu__ll_stop(&st, &o, -1.0) == 0 && !st.launched && S.running == 0);
    assert(xsk_gpu__ll_stop(&st, &o, -1.0) == 0); /* idempotent */

    /* 8b. the two halves (the pipelined RX loop): two channels, a batch in flight on each, completed out of post order;
     *     a second post while one is in flight is refused (nothing posted), ready never blocks, a wait with nothing in
     *     flight is refused, and a stop while a batch is in flight ends it (its outcome in stop_unserved) */
    {
        struct sim A, B;
        memset(&A, 0, sizeof A);
        memset(&B, 0, sizeof B);
        A.stop_countdown = B.stop_countdown = -1;
        A.serve_mask = B.serve_mask = 0xFu;
        A.serve_after = 3;
        B.serve_after = 6;
        A.stop_after = B.stop_after = 2;
        struct xsk_gpu__ll_state sa = st, sb = st;
        sa.bell = &A.bell;
        sb.bell = &B.bell;
        sa.seq = sb.seq = 0;
        sa.launched = sb.launched = sa.broken = sb.broken = sa.inflight = sb.inflight = 0;
        struct xsk_gpu__ll_ops oa = ops_of(&A), ob = ops_of(&B);
        int want_a = 0, want_b = 0;
        for (int round = 0; round < 20; round++) {
            const uint32_t wa = 1u + (uint32_t)round % XSK_GPU__LL_WG, wb = 1u + (uint32_t)(round * 3) % XSK_GPU__LL_WG;
            assert(xsk_gpu__ll_begin(&sa, &oa, XSK_GPU__BELL_N(64), wa) == 0 && sa.inflight);
            assert(xsk_gpu__ll_begin(&sb, &ob, XSK_GPU__BELL_N(200), wb) == 0 && sb.inflight);
            const uint64_t cmd = A.bell.cmd;
            assert(xsk_gpu__ll_begin(&sa, &oa, XSK_GPU__BELL_N(64), wa) == -EBUSY && A.bell.cmd == cmd);
            assert(!xsk_gpu__ll_ready(&sa) && !xsk_gpu__ll_ready(&sb)); /* nobody served anything yet */
            if (round & 1) {
                assert(xsk_gpu__ll_wait(&sb, &ob, &un) == 0 && un == 0 && !sb.inflight);
                assert(xsk_gpu__ll_wait(&sa, &oa, &un) == 0 && un == 0);
            } else {
                for (int k = 0; k < 10; k++) oa.relax(oa.u); /* A's grid serves while the host does other work */
                assert(xsk_gpu__ll_ready(&sa));
                assert(xsk_gpu__ll_wait(&sa, &oa, &un) == 0 && un == 0);
                assert(xsk_gpu__ll_wait(&sb, &ob, &un) == 0 && un == 0);
            }
            for (uint32_t g = 0; g < wa; g++) assert(A.bell.wg[g].done == sa.seq);
            for (uint32_t g = 0; g < wb; g++) assert(B.bell.wg[g].done == sb.seq);
            want_a += (int)wa;
            want_b += (int)wb;
        }
        assert(A.serves == want_a && B.serves == want_b && A.launches == 1 && B.launches == 1); /* each slice once */
        assert(xsk_gpu__ll_wait(&sa, &oa, &un) == -EINVAL);
        /* stop with a batch in flight that nobody took: retired unserved, the state has nothing in flight */
        A.serve_after = -1;
        assert(xsk_gpu__ll_begin(&sa, &oa, XSK_GPU__BELL_N(64), 1) == 0);
        assert(xsk_gpu__ll_stop(&sa, &oa, -1.0) == 0 && !sa.inflight && sa.stop_unserved == 1u);
        assert(A.bell.wg[0].cancel == sa.seq && A.bell.wg[0].done == sa.seq);
        assert(xsk_gpu__ll_wait(&sa, &oa, &un) == -EINVAL);
        A.serve_after = 1;
        assert(xsk_gpu__ll_run(&sa, &oa, XSK_GPU__BELL_N(64), 1, &un) == 0 && A.bell.wg[0].done == sa.seq);
        assert(xsk_gpu__ll_stop(&sb, &ob, -1.0) == 0 && xsk_gpu__ll_stop(&sa, &oa, -1.0) == 0);
    }

    /* 9. slices: contiguous, multiples of 4 (but the last), covering [0, n) exactly */
    for (uint32_t n = 1; n <= XSK_GPU_LOWLAT_MAX; n++)
        for (uint32_t w = 1; w <= XSK_GPU__LL_WG; w++) {
            uint32_t next = 0;
            for (uint32_t g = 0; g < w; g++) {
                uint32_t f0, f1;
                xsk_gpu__ll_slice(n, w, g, &f0, &f1);
                assert(f0 == next && f1 >= f0 && f1 <= n);
                if (f1 < n) assert((f1 - f0) % 4 == 0);
                next = f1;
            }
            assert(next == n);
        }

    /* 10. groups: <= 64 frames on the leader, and <= 128 frames of <= 16 KiB; every larger batch on every workgroup */
    struct xsk_gpu_desc d[XSK_GPU_LOWLAT_MAX];
    for (int i = 0; i < (int)XSK_GPU_LOWLAT_MAX; i++) {
        d[i].addr = 4096u * i;
        d[i].len = 1500;
        d[i].options = 0;
    }
    assert(xsk_gpu__ll_groups(d, 64) == 1);
    assert(xsk_gpu__ll_groups(d, 65) == XSK_GPU__LL_WG);  /* 95 KiB */
    assert(xsk_gpu__ll_groups(d, 100) == XSK_GPU__LL_WG); /* 146 KiB */
    assert(xsk_gpu__ll_groups(d, XSK_GPU_LOWLAT_MAX) == XSK_GPU__LL_WG);
    for (int i = 0; i < (int)XSK_GPU_LOWLAT_MAX; i++) d[i].len = 64;
    assert(xsk_gpu__ll_groups(d, 128) == 1 && xsk_gpu__ll_groups(d, 129) == XSK_GPU__LL_WG);
    assert(xsk_gpu__ll_groups(d, 300) == XSK_GPU__LL_WG && xsk_gpu__ll_groups(d, 256) == XSK_GPU__LL_WG);
    d[0].len = 1500;
    assert(xsk_gpu__ll_groups(d, 128) == 1);  /* 9.5 KiB */
    for (int i = 0; i < 16; i++) d[i].len = 1500;
    assert(xsk_gpu__ll_groups(d, 128) == XSK_GPU__LL_WG);  /* 30 KiB */
    printf("lowlat proto ok\n");
    return 0;
}
