"""Host-UMEM paths on the GPU, bit for bit against the CPU oracle: BASELINE config 1's exact workload
(4096 x 64-B frames in one 16 MiB UMEM of 4 KiB chunks, RX_BATCH_SIZE batches -- src/lib/xsk_utils.h:6-8,
src/lib/xsk_receive.c:220-233) in every host mode, the low-latency doorbell mode (resident polling kernel),
and the multi-context path (several contexts over ONE UMEM, descriptor i on context i mod G)."""
import ctypes
import time

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402

COUNTERS = ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")
MODES = [X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def run_batches(ctx, descs, batch, want_recs=True):
    tot = {k: 0 for k in COUNTERS}
    vs, rs = [], []
    for i in range(0, len(descs), batch):
        v, r, s = ctx.process(descs[i:i + batch], want_recs=want_recs)
        vs.append(v)
        rs.append(r)
        for k in tot:
            tot[k] += int(s[k])
    return np.concatenate(vs), (np.concatenate(rs) if want_recs else None), tot


def check(umem, work, descs, v, r, tot, ctx=None):
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    assert (v == v_ref).all(), np.nonzero(v != v_ref)[0][:8]
    if r is not None:
        assert (r == r_ref).all(), np.nonzero(r != r_ref)[0][:8]
    for k in COUNTERS:
        assert tot[k] == int(s_ref[k]), k
    diff = np.nonzero(work != ref)[0]
    assert len(diff) == 0, f"{len(diff)} bytes differ, first at {diff[:8]}; " + describe_diff(umem, work, ref, descs, v,
                                                                                               diff, ctx)


def describe_diff(umem, work, ref, descs, v, diff, ctx=None):
    """Which frames' bytes differ, where, and whether they are still the request's (a write that never landed)."""
    addr = descs["addr"].astype(np.int64)
    out = []
    for j in np.unique(np.searchsorted(np.sort(addr), diff, side="right") - 1)[:6]:
        a = int(np.sort(addr)[j])
        i = int(np.nonzero(addr == a)[0][0])
        d = diff[(diff >= a) & (diff < a + 4096)] - a
        gpu = ""
        if ctx is not None and ctx.mode != X.MODE_STAGED:  # the same bytes through the GPU's translation
            try:
                g = ctx.umem_view(a, 64)
                gpu = f" gpu-view {g[d[d < 64][:12]].tolist()} (matches host: {bool((g == work[a:a + 64]).all())})"
            except Exception as e:  # noqa: BLE001 -- a report, not a check
                gpu = f" gpu-view failed: {e}"
        out.append(f"frame {i} @{a} len {int(descs['len'][i])} verdict {int(v[i])}: offsets {d[:24].tolist()} "
                   f"got {work[a + d[:12]].tolist()} want {ref[a + d[:12]].tolist()} "
                   f"request {umem[a + d[:12]].tolist()}{gpu}")
    return " | ".join(out)


def test_context_teardown_beside_a_resident_lowlat_grid():
    """Round 6 (tools/fini_block.py, profiles/r06/fini_block.jsonl): the HIP runtime's hipFree, and hipHostFree /
    hipHostUnregister of host memory a kernel has used, wait for every stream of the device -- another context's
    resident LOWLAT grid included, which leaves its stream only when it stops or has been idle for 50 ms.  A context
    over a UMEM of its own unregisters it at close; the library then asks every resident grid to leave once idle (the
    yield word, xsk_gpu__ll_yield_all) and keeps released buffers for reuse (xsk_gpu__buf_free), so the close does not
    wait for the other context to go idle.  Checked here: (a) on one thread, with the other context's grid resident but
    idle, a close of every mode returns within 0.5 s and both contexts stay exact; (b) beside a LOWLAT context kept busy
    on a second thread, contexts of every mode over UMEMs of their own are created, used and closed: every batch of
    both is exact, nothing fails, and every close returns within 0.25 s while the busy context is still serving."""
    import threading
    _dev()
    umem = np.zeros(1024 * 2048, np.uint8)
    descs = oracle.synth_batch(umem, 1024, 0, 2048, 0x5EEDE100, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, _, _ = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)

    def lifecycle(mode):
        u = X.umem_copy(umem[:256 * 2048])
        d = np.ascontiguousarray(descs[:64])
        r = u.copy()
        vr, _, _ = oracle.echo_batch(r, d)
        ctx = X.EchoContext(u, 0, max_batch=64, mode=mode)
        v, _, _ = ctx.process(d, want_recs=False)
        t0 = time.perf_counter()
        ctx.close()
        t1 = time.perf_counter()
        assert (v == vr).all() and (u == r).all()
        return t1 - t0, t1

    # (a) one thread, the other context's grid resident and idle
    with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT) as a:
        assert a.mode == X.MODE_LOWLAT
        for mode in MODES:
            work[:] = umem
            v, _, _ = a.process(descs[:64], want_recs=False)  # the grid is resident again
            assert (v == v_ref[:64]).all()
            took, _ = lifecycle(mode)
            assert took < 0.5, (mode, took)
            v, _, _ = a.process(descs[64:128], want_recs=False)
            assert (v == v_ref[64:128]).all() and (work[:128 * 2048] == ref[:128 * 2048]).all()

    # (b) beside a context kept busy on a second thread
    stop, errors, calls, busy_end = threading.Event(), [], [0], [None]

    def busy():
        try:
            with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT) as c:
                assert c.mode == X.MODE_LOWLAT
                t_end = time.perf_counter() + 20.0
                while not stop.is_set() and time.perf_counter() < t_end:
                    work[:] = umem
                    vs = [c.process(descs[i:i + 64], want_recs=False)[0] for i in range(0, len(descs), 64)]
                    assert (np.concatenate(vs) == v_ref).all() and (work == ref).all()
                    calls[0] += 1
                busy_end[0] = time.perf_counter()
        except Exception as e:  # noqa: BLE001 -- reported below
            busy_end[0] = time.perf_counter()
            errors.append(repr(e))

    th = threading.Thread(target=busy)
    th.start()
    time.sleep(0.2)
    closes = []
    try:
        for mode in MODES:
            closes.append((mode, *lifecycle(mode)))
    finally:
        stop.set()
        th.join()
    report = {"errors": errors, "busy_passes": calls[0],
              "closes": [(m, round(t, 3), round(e - busy_end[0], 3)) for m, t, e in closes]}
    assert not errors and calls[0] > 0, report
    assert all(e < busy_end[0] for _, _, e in closes), report  # closed while the other context served
    assert max(t for _, t, _ in closes) < 0.25, report
    print(f"closes beside a busy LOWLAT context: {report}")


def test_queue_close_beside_a_busy_lowlat_queue_over_a_shared_umem():
    """Round 6: two RX queues over one UMEM (XDP_SHARED_UMEM).  Queue 0's LOWLAT context is kept busy on a thread;
    queue 1's contexts (every mode) are created, used and closed beside it.  The UMEM registration is shared
    (xsk_gpu__umem_ref) and the closing context's buffers are kept for reuse while a resident grid runs
    (xsk_gpu__buf_free), so no close calls a runtime free that waits for queue 0's grid: each returns within 0.25 s
    while queue 0 is still busy, every batch of both queues is exact, and once queue 0 closes nothing is kept."""
    import threading
    _dev()
    n, half = 1024, 1024 * 2048
    req = np.zeros(2 * half, np.uint8)
    d0 = oracle.synth_batch(req, n, 0, 2048, 0x5EEDE200, mode=1, len_lo=20, len_hi=1500)  # queue 0: first half
    d1 = oracle.synth_batch(req, n, half, 2048, 0x5EEDE201, mode=1, len_lo=20, len_hi=1500)  # queue 1: second half
    ref = req.copy()
    v0, _, _ = oracle.echo_batch(ref, d0)
    v1, _, _ = oracle.echo_batch(ref, d1)
    work = X.umem_copy(req)
    stop, ready, errors, calls, busy_end = threading.Event(), threading.Event(), [], [0], [None]

    def busy():
        try:
            with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT) as c:
                assert c.mode == X.MODE_LOWLAT
                ready.set()
                t_end = time.perf_counter() + 20.0
                while not stop.is_set() and time.perf_counter() < t_end:
                    work[:half] = req[:half]
                    vs = [c.process(d0[i:i + 64], want_recs=False)[0] for i in range(0, n, 64)]
                    assert (np.concatenate(vs) == v0).all() and (work[:half] == ref[:half]).all()
                    calls[0] += 1
                busy_end[0] = time.perf_counter()
        except Exception as e:  # noqa: BLE001 -- reported below
            busy_end[0] = time.perf_counter()
            errors.append(repr(e))
            ready.set()

    th = threading.Thread(target=busy)
    th.start()
    closes = []
    try:
        assert ready.wait(30)
        time.sleep(0.2)
        for rep in range(2):
            for mode in MODES:
                work[half:] = req[half:]
                ctx = X.EchoContext(work, 0, max_batch=n, mode=mode)
                v, _, _ = ctx.process(d1, want_recs=False)
                t0 = time.perf_counter()
                ctx.close()
                closes.append((mode, round(time.perf_counter() - t0, 4)))
                assert (v == v1).all() and (work[half:] == ref[half:]).all()
        kept_while_busy = X.lib().xsk_gpu__buf_kept(0)
        alive = th.is_alive()
    finally:
        stop.set()
        th.join()
    report = {"errors": errors, "busy_passes": calls[0], "closes": closes, "kept": kept_while_busy}
    assert not errors and alive and calls[0] > 0, report
    assert max(t for _, t in closes) < 0.25, report
    assert kept_while_busy > 0, report
    assert X.lib().xsk_gpu__buf_kept(0) == 0 and X.lib().xsk_gpu__umem_refs(work.ctypes.data) == 0, report
    print(f"queue closes beside a busy LOWLAT queue: {report}")


def test_context_churn_on_threads():
    """Round 6: the shared registrations (xsk_gpu__umem_ref) and the kept buffers (xsk_gpu__buf_alloc) under concurrent
    use.  For 3 s, on four threads: (0) a LOWLAT context serves quarter 0 of one UMEM; (1) contexts of every mode are
    created over quarter 1 of the same UMEM, serve one batch and close; (2) the same over quarter 2 with multi objects
    and pipes; (3) contexts over fresh page-aligned UMEMs of their own.  Every batch is exact, nothing fails, and at
    the end no registration reference and no kept buffer is left."""
    import threading
    _dev()
    n, q = 256, 256 * 2048
    req = np.zeros(4 * q, np.uint8)
    ds = [oracle.synth_batch(req, n, k * q, 2048, 0x5EEDC400 + k, mode=1, len_lo=20, len_hi=1500) for k in range(4)]
    ref = req.copy()
    vs = [oracle.echo_batch(ref, d)[0] for d in ds]
    work = X.umem_copy(req)
    stop, errors, counts = threading.Event(), [], [0, 0, 0, 0]

    def part(k):
        return slice(k * q, (k + 1) * q)

    def served(k, v):
        assert (v == vs[k]).all() and (work[part(k)] == ref[part(k)]).all(), k

    def t0():
        with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT) as c:
            while not stop.is_set():
                work[part(0)] = req[part(0)]
                served(0, np.concatenate([c.process(ds[0][i:i + 64], want_recs=False)[0] for i in range(0, n, 64)]))
                counts[0] += 1

    def t1():
        while not stop.is_set():
            for mode in MODES:
                work[part(1)] = req[part(1)]
                with X.EchoContext(work, 0, max_batch=n, mode=mode) as c:
                    served(1, c.process(ds[1], want_recs=False)[0])
                counts[1] += 1

    def t2():
        while not stop.is_set():
            for mode in MODES:
                work[part(2)] = req[part(2)]
                m = X.MultiContext(work, [0, 0], max_batch=n, mode=mode)
                try:
                    served(2, m.process(ds[2], want_recs=False)[0])
                finally:
                    m.close()
                X.RxPipe(work, 0, depth=2, mode=mode).close()
                counts[2] += 1

    def t3():
        own = req[part(3)]
        d = ds[3].copy()
        d["addr"] -= 3 * q
        while not stop.is_set():
            for mode in MODES:
                u = X.umem_copy(own)
                with X.EchoContext(u, 0, max_batch=n, mode=mode) as c:
                    v = c.process(d, want_recs=False)[0]
                assert (v == vs[3]).all() and (u == ref[part(3)]).all()
                counts[3] += 1

    def run(fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(f"{fn.__name__}: {e!r}")
            stop.set()

    ths = [threading.Thread(target=run, args=(f,)) for f in (t0, t1, t2, t3)]
    for th in ths:
        th.start()
    time.sleep(3.0)
    stop.set()
    for th in ths:
        th.join()
    assert not errors, errors
    assert min(counts) > 0, counts
    assert X.lib().xsk_gpu__umem_refs(work.ctypes.data) == 0 and X.lib().xsk_gpu__buf_kept(0) == 0
    print(f"churn: passes per thread {counts}")


@pytest.mark.parametrize("mode", MODES)
def test_contexts_sharing_one_umem(mode):
    """Round 6 (tools/doublereg_probe.py, profiles/r06/doublereg_attributes.jsonl): the HIP runtime keeps ONE registration
    per base address and counts nothing -- a second hipHostRegister of the base succeeds, the first hipHostUnregister
    removes it for both -- so when one of two contexts over one UMEM (AF_XDP sockets sharing a UMEM, one context per RX
    queue) closed, the other went on over a UMEM the runtime no longer held registered, and a UMEM the caller had
    registered itself lost its registration at the library's close.  The library now counts its users of each
    registration (xsk_gpu__umem_ref).  Checked: two contexts, a context over a part of the UMEM, a multi object and a
    pipe over one UMEM serve their shares exactly; after any of them closes the others still serve exactly; a UMEM
    that overlaps a registration without lying inside it gets -EBUSY; the last close releases the registration; a
    UMEM the caller registered itself stays registered."""
    _dev()
    n = 2048
    req = np.zeros(n * 4096, np.uint8)
    descs = oracle.synth_batch(req, n, 0, 4096, 0x5EED5A4E + mode, mode=1, len_lo=20, len_hi=1500)
    ref = req.copy()
    v_ref, _, _ = oracle.echo_batch(ref, descs)
    big = X.umem_zeros(2 * req.nbytes)
    u = big[:req.nbytes]  # the same base as `big`, half its bytes
    refs = lambda: X.lib().xsk_gpu__umem_refs(u.ctypes.data)  # noqa: E731

    def serve(ctx, idx):
        v, _, _ = ctx.process(np.ascontiguousarray(descs[idx]), want_recs=False)
        assert (v == v_ref[idx]).all()

    a = X.EchoContext(u, 0, max_batch=n, mode=mode)
    b = X.EchoContext(u, 0, max_batch=n, mode=mode)
    try:
        assert refs() == 2
        u[:] = req
        serve(a, slice(0, n, 2))  # queue 0: even frames
        serve(b, slice(1, n, 2))  # queue 1: odd frames
        assert (u == ref).all()
        with pytest.raises(X.XskGpuError, match="EBUSY"):  # overlaps the registration without lying inside it
            X.EchoContext(big, 0, max_batch=64, mode=mode)
        assert refs() == 2
        b.close()
        assert refs() == 1
        u[:] = req
        serve(a, slice(0, n))  # round 5's library: -EIO here
        assert (u == ref).all()
        half = n // 2  # a context over the second half of the UMEM: a reference of the same registration
        dp = descs[half:].copy()
        dp["addr"] -= half * 4096
        with X.EchoContext(u[half * 4096:], 0, max_batch=n, mode=mode) as c:
            assert refs() == 2
            u[:] = req
            v, _, _ = c.process(dp, want_recs=False)
            assert (v == v_ref[half:]).all() and (u[half * 4096:] == ref[half * 4096:]).all()
        assert refs() == 1
        m = X.MultiContext(u, [0], max_batch=n, mode=mode)
        p = X.RxPipe(u, 0, depth=2, mode=mode)
        assert refs() == 3
        u[:] = req
        v, _, _ = m.process(descs, want_recs=False)
        assert (v == v_ref).all() and (u == ref).all()
        m.close()
        p.close()
        assert refs() == 1
        u[:] = req
        serve(a, slice(0, n))
        assert (u == ref).all()
    finally:
        b.close()
        a.close()
    assert refs() == 0
    # the registration is gone: the runtime no longer knows the base
    hip = ctypes.CDLL("libamdhip64.so")
    flags = ctypes.c_uint()
    assert hip.hipHostGetFlags(ctypes.byref(flags), ctypes.c_void_p(u.ctypes.data)) != 0
    hip.hipGetLastError()
    # a UMEM the caller registered: used, and left registered at close
    assert hip.hipHostRegister(ctypes.c_void_p(u.ctypes.data), ctypes.c_size_t(u.nbytes), 3) == 0
    try:
        with X.EchoContext(u, 0, max_batch=n, mode=mode) as c:
            u[:] = req
            serve(c, slice(0, n))
            assert (u == ref).all()
        assert refs() == 0
    finally:
        assert hip.hipHostUnregister(ctypes.c_void_p(u.ctypes.data)) == 0  # still the caller's


@pytest.mark.parametrize("mode", MODES)
def test_host_umem_starts_on_a_page_of_its_own(mode):
    """two UMEMs carved from one allocation so that they share a page -- the layout round 5's numpy
    fixtures had when glibc served consecutive arrays from its heap -- are refused (-EINVAL) by every host entry point,
    as AF_XDP refuses an area that is not page-aligned; round 5's library accepted them.  Two page-aligned neighbours
    of the same allocation then run the verdict's sequence (init A, init B, fini A, B's batches; re-init A, fini B, A's
    batches) exact against the oracle."""
    import errno
    _dev()
    S = 1 << 20
    whole = X.umem_zeros(2 * S + 2 * 4096)
    L = X.lib()
    import ctypes as C
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    for base in (whole.ctypes.data + 16, whole.ctypes.data + 16 + S):
        assert L.xsk_gpu_init(C.byref(h), 0, base, S, 64, mode) == -errno.EINVAL
        assert L.xsk_gpu_multi_init(C.byref(h), devs, 2, base, S, 64, mode) == -errno.EINVAL
        assert L.xsk_gpu_rx_pipe_init(C.byref(h), 0, base, S, 2, mode) == -errno.EINVAL
    a, b = whole[:S], whole[S:2 * S]  # page-aligned neighbours: adjacent, sharing no page
    sets = []
    for k, u in enumerate((a, b)):
        descs = oracle.synth_batch(u, 512, 0, 2048, 0x5EEDE000 + 16 * mode + k, mode=1, len_lo=20, len_hi=1500)
        req = u.copy()
        ref = req.copy()
        v_ref, r_ref, _ = oracle.echo_batch(ref, descs)
        sets.append((u, descs, req, ref, v_ref, r_ref))

    def run(ctx, k, reps=3):
        u, descs, req, ref, v_ref, r_ref = sets[k]
        for _ in range(reps):
            u[:] = req
            v, r, _ = run_batches(ctx, descs, 64)
            assert (v == v_ref).all() and (r == r_ref).all()
            diff = np.nonzero(u != ref)[0]
            assert len(diff) == 0, describe_diff(req, u, ref, descs, v, diff, ctx)

    ca = X.EchoContext(a, 0, max_batch=64, mode=mode)
    cb = X.EchoContext(b, 0, max_batch=64, mode=mode)
    run(ca, 0, 1)
    run(cb, 1, 1)
    ca.close()
    run(cb, 1)
    ca = X.EchoContext(a, 0, max_batch=64, mode=mode)
    cb.close()
    run(ca, 0)
    ca.close()


@pytest.mark.parametrize("mode", MODES)
def test_c1_exact_workload(mode):
    """BASELINE config 1: 4096 x 64-B ICMP echo requests, one per 4 KiB chunk at the 256-B AF_XDP headroom,
    in RX_BATCH_SIZE (64) batches -- every frame replied, every byte as process_packet() leaves it."""
    _dev()
    n = 4096
    umem = np.zeros(4096 * 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 4096, seed=0x5EED0001, mode=0, len_lo=64, len_hi=64)
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=64, mode=mode) as ctx:
        v, r, tot = run_batches(ctx, descs, 64)
    check(umem, work, descs, v, r, tot)
    assert (v == X.TX_REPLY).all() and tot["tx_packets"] == n and tot["tx_bytes"] == 64 * n


@pytest.mark.parametrize("batch", [1, 64, 1000, 1024])
def test_lowlat_mixed_batches(batch):
    """The doorbell path over mixed traffic (every negative / edge case) at odd batch sizes up to the
    doorbell's 1024 frames, records on and off."""
    _dev()
    n = 5000
    umem = np.zeros(n * 2048 + 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 2048, seed=0x5EED1C1C + batch, mode=1, len_lo=20, len_hi=1900)
    for want in (True, False):
        work = X.umem_copy(umem)
        with X.EchoContext(work, 0, max_batch=max(batch, 1), mode=X.MODE_LOWLAT) as ctx:
            v, r, tot = run_batches(ctx, descs, batch, want_recs=want)
        check(umem, work, descs, v, r, tot)


def test_lowlat_completion_never_overtakes_outputs():
    """The completion hand-off under the fastest reader: 20 000 one- and three-frame doorbell calls whose
    consecutive frames alternate between replies and drops (so a verdict or record left over from the
    previous call can never pass for the new one), every verdict, record and byte checked.  A `done` word
    that overtook the L2 write-back of the verdicts failed ~1 call in 10^4 here (xsk_lowlat.hip release)."""
    _dev()
    n = 15000
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 2048, seed=0x5EED1F1F, mode=0, len_lo=42, len_hi=1500)
    descs[1::2]["len"] = np.minimum(descs[1::2]["len"], 19)  # every other frame a DROP_SHORT
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    assert (v_ref[0::2] == X.TX_REPLY).all() and (v_ref[1::2] != X.TX_REPLY).all()
    for batch in (1, 3):  # odd: consecutive calls' verdict patterns differ
        work = X.umem_copy(umem)
        with X.EchoContext(work, 0, max_batch=batch, mode=X.MODE_LOWLAT) as ctx:
            v, r, tot = run_batches(ctx, descs, batch)
        check(umem, work, descs, v, r, tot)


def test_lowlat_idle_exit_large_batches_and_options():
    """The resident kernel leaves after 50 ms without a batch and the next call brings it back; a batch
    above the doorbell's size stops it and takes the launch path; switching to wire-format options
    restarts it in wire mode -- results exact throughout, frames recycled between calls."""
    _dev()
    n = 3 * 1024 + 2048 + 512
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED1D1D, mode=1, len_lo=20, len_hi=1500)
    work = X.umem_copy(umem)
    parts = [(0, 64), (64, 1024), (1088, 2048), (3136, 1000), (4136, 512), (4648, n - 4648)]
    tot = {k: 0 for k in COUNTERS}
    vs = []
    with X.EchoContext(work, 0, max_batch=2048, mode=X.MODE_LOWLAT) as ctx:
        for i, (a, m) in enumerate(parts):
            if i == 3:
                time.sleep(0.12)  # > 50 ms idle: the kernel exits on its own
            v, _, s = ctx.process(descs[a:a + m], want_recs=False)
            vs.append(v)
            for k in tot:
                tot[k] += int(s[k])
    check(umem, work, descs, np.concatenate(vs), None, tot)
    # wire mode through the doorbell (the spec oracle: oracle_echo_batch_opts)
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=1024, mode=X.MODE_LOWLAT) as ctx:
        v0, _, _ = ctx.process(descs[:64], want_recs=False)
        ctx.set_options(X.OPT_ALL)
        v1, r1, _ = ctx.process(descs[64:1088])
    ref = umem.copy()
    v_ref0, _, _ = oracle.echo_batch_opts(ref, descs[:64], 0)
    v_ref1, r_ref1, _ = oracle.echo_batch_opts(ref, descs[64:1088], X.OPT_ALL)
    assert (v0 == v_ref0).all() and (v1 == v_ref1).all() and (r1 == r_ref1).all()
    assert (work == ref).all()


def test_lowlat_many_small_calls():
    """20 000 back-to-back 64-frame doorbell calls over a recycled 4096-frame UMEM (the RX loop's steady
    state): the polling kernel must see every new frame, never a stale cached one."""
    _dev()
    n, batch, passes = 4096, 64, 5
    umem = np.zeros(n * 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 4096, seed=0x5EED1E1E, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)
    t = 0.0
    with X.EchoContext(work, 0, max_batch=batch, mode=X.MODE_LOWLAT) as ctx:
        for p in range(passes):
            work[:] = umem  # the frames are recycled: new requests at the same UMEM addresses
            t0 = time.perf_counter()
            v, r, tot = run_batches(ctx, descs, batch)
            t += time.perf_counter() - t0
            assert (v == v_ref).all() and (r == r_ref).all(), p
            for k in COUNTERS:
                assert tot[k] == int(s_ref[k])
            assert (work == ref).all(), p
    print(f"lowlat: {t / (passes * n // batch) * 1e6:.1f} us per 64-frame call (Python driver)")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_context_one_gpu(mode, devices):
    """G contexts on device 0 over ONE registered UMEM (the rehearsal of G GPUs): descriptor i on context
    i mod G, each on its own host thread and stream; verdicts, records and every byte exact, counters summed."""
    _dev()
    n = 20000
    umem = np.zeros(n * 2048 + 256, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 2048, seed=0x5EED2020 + len(devices), mode=1, len_lo=20, len_hi=1500)
    for batch in (64, 3001, n):
        work = X.umem_copy(umem)
        with X.MultiContext(work, devices, max_batch=batch, mode=mode) as m:
            v, r, tot = run_batches(m, descs, batch)
        check(umem, work, descs, v, r, tot)


def test_multi_context_wire_options():
    _dev()
    n = 4000
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED2121, mode=1, len_lo=20, len_hi=1500)
    work = X.umem_copy(umem)
    with X.MultiContext(work, [0, 0], max_batch=n, mode=X.MODE_STAGED, opts=X.OPT_ALL) as m:
        v, r, _ = m.process(descs)
    ref = umem.copy()
    v_ref, r_ref, _ = oracle.echo_batch_opts(ref, descs, X.OPT_ALL)
    assert (v == v_ref).all() and (r == r_ref).all() and (work == ref).all()


def test_multi_context_argument_checks():
    import ctypes as C
    import errno
    L = X.lib()
    buf = X.umem_zeros(4096)
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    # a host UMEM starts on a page of its own (include/xsk_gpu.h; AF_XDP's rule)
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 2, buf.ctypes.data + 16, buf.nbytes - 16, 64, 0) == -errno.EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 0, buf.ctypes.data, buf.nbytes, 64, 0) == -errno.EINVAL
    assert L.xsk_gpu_multi_init(C.byref(h), devs, 2, buf.ctypes.data, buf.nbytes, 64, 9) == -errno.EINVAL
    bad = (C.c_int * 2)(0, 999)
    assert L.xsk_gpu_multi_init(C.byref(h), bad, 2, buf.ctypes.data, buf.nbytes, 64, 0) == -errno.ENODEV
    assert L.xsk_gpu_multi_process(None, None, 0, None, None, None) == -errno.EINVAL
    L.xsk_gpu_multi_fini(None)


@pytest.mark.parametrize("batch", [64, 512])
def test_lowlat_posts_near_idle_exit(batch):
    """Batches posted right around the resident kernel's 50-ms idle exit (the exit / relaunch race): every
    batch is served exactly once and exactly right -- 64-frame batches (the leader alone) and 512-frame
    batches served by two resident workgroups (the leader's exit takes the other workgroup with it)."""
    _dev()
    n = batch * 40
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED2323, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)
    rng = np.random.default_rng(11)
    tot = {k: 0 for k in COUNTERS}
    with X.EchoContext(work, 0, max_batch=batch, mode=X.MODE_LOWLAT) as ctx:
        for i in range(0, n, batch):
            time.sleep(float(rng.uniform(0.046, 0.054)))
            v, r, s = ctx.process(descs[i:i + batch])
            assert (v == v_ref[i:i + batch]).all() and (r == r_ref[i:i + batch]).all(), i
            for k in tot:
                tot[k] += int(s[k])
    for k in COUNTERS:
        assert tot[k] == int(s_ref[k]), k
    assert (work == ref).all()


@pytest.mark.parametrize("groups", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("flen", [64, 1500])
def test_lowlat_workgroup_slices(groups, flen):
    """Doorbell batches of 65-1024 frames served by 1-4 resident workgroups (0: chosen from the batch's size),
    each a contiguous slice of the descriptors: every verdict, record, counter and byte exact, consecutive
    batches of different sizes so a workgroup's slice moves between calls, plus one-frame and 64-frame calls
    (the leader alone) in between."""
    _dev()
    sizes = [65, 1024, 256, 1, 300, 777, 64, 1023, 4, 1024]
    n = sum(sizes)
    umem = np.zeros(n * 2048 + 4096, np.uint8)
    mode = 0 if flen == 1500 else 1
    descs = oracle.synth_batch(umem, n, 256, 2048, seed=0x5EED2424 + groups + flen, mode=mode, len_lo=20 if mode else flen,
                               len_hi=flen)
    work = X.umem_copy(umem)
    tot = {k: 0 for k in COUNTERS}
    vs, rs = [], []
    with X.EchoContext(work, 0, max_batch=1024, mode=X.MODE_LOWLAT) as ctx:
        ctx.lowlat_tune(groups=groups)
        a = 0
        for m in sizes:
            v, r, st = ctx.process(descs[a:a + m])
            vs.append(v)
            rs.append(r)
            for k in tot:
                tot[k] += int(st[k])
            a += m
    check(umem, work, descs, np.concatenate(vs), np.concatenate(rs), tot)


def test_lowlat_timeout_quiesces_and_recovers():
    """A doorbell batch that misses its completion timeout (set to 1 us here, so a 1024 x 1500-B batch cannot
    make it): the call returns -ETIMEDOUT only after STOP has been posted and the resident grid has stopped, so
    the caller owns its frames again -- each frame of that batch is either untouched or exactly transformed and
    nothing changes it afterwards; the next call (default timeout) relaunches the grid and is exact."""
    import errno
    _dev()
    n = 2048
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED2525, mode=0, len_lo=1500, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, _ = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)
    timed_out = 0
    with X.EchoContext(work, 0, max_batch=1024, mode=X.MODE_LOWLAT) as ctx:
        ctx.process(descs[1024:1025])  # the grid is up
        work[1024 * 2048:1025 * 2048] = umem[1024 * 2048:1025 * 2048]
        ctx.lowlat_tune(timeout_us=1)
        try:
            ctx.process(descs[:1024])
        except X.XskGpuError as e:
            assert e.rc == -errno.ETIMEDOUT, e
            timed_out = 1
        snap = work[:1024 * 2048].copy()
        time.sleep(0.2)  # a kernel still running would change frames now
        assert (work[:1024 * 2048] == snap).all(), "frames changed after the timed-out call returned"
        for j in range(1024):
            f = work[j * 2048:(j + 1) * 2048]
            assert (f == umem[j * 2048:(j + 1) * 2048]).all() or (f == ref[j * 2048:(j + 1) * 2048]).all(), j
        ctx.lowlat_tune(timeout_us=0)
        v, r, _ = ctx.process(descs[1024:])
    assert (v == v_ref[1024:]).all() and (r == r_ref[1024:]).all()
    assert (work[1024 * 2048:] == ref[1024 * 2048:]).all()
    print(f"timed out: {timed_out}")


def test_multi_context_partial_failure():
    """One context of three fails (injected): the call returns its error and adds NOTHING to the counters; the
    other contexts' shares are transformed with their verdicts / records written, the failed share's frames and
    output positions are untouched; xsk_gpu_multi_status says which share failed; the next call is whole."""
    import ctypes as C
    import errno
    _dev()
    n = 6000
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED2626, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    for mode in (X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT):
        for batch in (300, n):  # doorbell-sized shares (LOWLAT) and launched ones
            work = X.umem_copy(umem)
            with X.MultiContext(work, [0, 0, 0], max_batch=batch, mode=mode) as m:
                m.inject_failure(1, -errno.EIO)
                d = np.ascontiguousarray(descs[:batch])
                verd = np.full(batch, 0xEE, np.uint8)
                recs = np.zeros(batch, X.REC_DTYPE)
                stats = np.zeros(1, X.STATS_DTYPE)
                stats["rx_packets"] = 7
                rc = X.lib().xsk_gpu_multi_process(m._ctx, d.ctypes.data, batch, verd.ctypes.data, recs.ctypes.data,
                                                   stats.ctypes.data)
                assert rc == -errno.EIO
                assert m.status() == [0, -errno.EIO, 0]
                assert int(stats["rx_packets"][0]) == 7 and int(stats["tx_bytes"][0]) == 0  # nothing added
                ok = np.arange(batch) % 3 != 1
                assert (verd[ok] == v_ref[:batch][ok]).all() and (recs[ok] == r_ref[:batch][ok]).all()
                assert (verd[~ok] == 0xEE).all() and (recs[~ok] == np.zeros(1, X.REC_DTYPE)).all()
                for j in range(batch):
                    exp = ref if ok[j] else umem
                    assert (work[j * 2048:(j + 1) * 2048] == exp[j * 2048:(j + 1) * 2048]).all(), (mode, batch, j)
                # the next call: every context, counters applied
                work[:] = umem
                v, r, st = m.process(descs[:batch])
                assert m.status() == [0, 0, 0]
                assert (v == v_ref[:batch]).all() and (r == r_ref[:batch]).all()
                assert int(st["tx_packets"]) == int((v_ref[:batch] == 0).sum())
    del C


def test_multi_lowlat_path_chosen_per_batch():
    """LOWLAT contexts sharing one GPU: a batch whose shares straddle the doorbell limit (2049 frames over two
    contexts: 1025 + 1024) takes the launch path in every context; doorbell-sized batches before and after
    it go through the resident kernels -- every byte exact."""
    _dev()
    n = 2049 + 128 + 2049
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED2727, mode=1, len_lo=20, len_hi=1500)
    work = X.umem_copy(umem)
    tot = {k: 0 for k in COUNTERS}
    vs = []
    with X.MultiContext(work, [0, 0], max_batch=2049, mode=X.MODE_LOWLAT) as m:
        for a, b in ((0, 2049), (2049, 2177), (2177, n)):
            v, _, st = m.process(descs[a:b], want_recs=False)
            vs.append(v)
            for k in tot:
                tot[k] += int(st[k])
    check(umem, work, descs, np.concatenate(vs), None, tot)


def test_lowlat_contexts_per_device_limit():
    """At most XSK_GPU_LOWLAT_PER_DEVICE resident LOWLAT kernels per device in one process (more would queue behind
    each other on the runtime's few high-priority hardware queues and time out, tools/rxqueues): further LOWLAT
    requests run as ZEROCOPY (xsk_gpu_ctx_mode), every context bit-exact on 64-frame RX batches, and fini gives the
    slots back."""
    import gc
    _dev()
    gc.collect()  # contexts of earlier tests are closed (their slots released)
    n = 256
    umems, descss, ctxs = [], [], []
    try:
        for q in range(X.LOWLAT_PER_DEVICE + 2):
            umem = np.zeros(n * 4096, np.uint8)
            descs = oracle.synth_batch(umem, n, 256, 4096, 0x5EED4040 + q, mode=1, len_lo=20, len_hi=1500)
            umems.append(umem)
            descss.append(descs)
            ctxs.append(X.EchoContext(X.umem_copy(umem), 0, max_batch=64, mode=X.MODE_LOWLAT))
        modes = [c.mode for c in ctxs]
        # LOWLAT while a slot is free, ZEROCOPY from then on (a context another test still holds takes a slot too)
        k = modes.count(X.MODE_LOWLAT)
        assert 1 <= k <= X.LOWLAT_PER_DEVICE and modes == [X.MODE_LOWLAT] * k + [X.MODE_ZEROCOPY] * (len(modes) - k), modes
        for umem, descs, ctx in zip(umems, descss, ctxs):
            v, r, tot = run_batches(ctx, descs, 64)
            check(umem, ctx.umem, descs, v, r, tot, ctx)
            ref = umem.copy()
            oracle.echo_batch(ref, descs)
            assert (ctx.umem == ref).all()
    finally:
        for c in ctxs:
            c.close()
    again = [X.EchoContext(X.umem_zeros(1 << 16), 0, max_batch=64, mode=X.MODE_LOWLAT) for _ in range(k)]
    try:
        assert [c.mode for c in again] == [X.MODE_LOWLAT] * k  # fini gave the slots back
    finally:
        for c in again:
            c.close()


@pytest.mark.parametrize("mode", [X.MODE_ZEROCOPY, X.MODE_STAGED])
def test_long_batch_split_launches_host_counters(mode):
    """A host batch of 2.5 M packed 64-B frames of mixed traffic in ONE call: on 256 CUs the zerocopy share is five
    rounds, so the call runs as three launches of about two rounds, each folding its per-workgroup counter rows
    into the mapped host slot after the previous fold (xsk_echo.hip: echo_launch); STAGED cuts it into chunks first.
    Every byte, verdict, record and counter exact."""
    _dev()
    n = 2_500_000
    umem = np.zeros(n * 64, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 64, 0x5EED5252, mode=1, len_lo=20, len_hi=64,
                               threads=min(16, oracle.cpu_threads()))
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=n, mode=mode) as ctx:
        v, r, st = ctx.process(descs)
    check(umem, work, descs, v, r, {k: int(st[k]) for k in COUNTERS})


def _small_frames_case(seed, n, wire):
    """Small frames (<= 112 B) for the doorbell path: valid requests and every negative, unaligned starts,
    frames at the UMEM's very end (window cut), descriptors past it (DROP_BAD_DESC), scrambled order."""
    rng = np.random.default_rng(seed)
    stride = 160
    size = n * stride + 48
    umem = rng.integers(0, 256, size, dtype=np.uint8)
    tmp = np.zeros(n * 4096, np.uint8)
    d = oracle.synth_batch(tmp, n, 0, 4096, seed=seed, mode=1, len_lo=20, len_hi=112, threads=4)
    descs = np.zeros(n, X.DESC_DTYPE)
    for j in range(n):
        L = int(d["len"][j])
        a = j * stride + int(rng.integers(0, 16))
        if j == n - 1:
            a = size - max(L, 38)  # the frame's end is the UMEM's end: its 64-B window is cut
        umem[a:a + L] = tmp[j * 4096:j * 4096 + L]
        descs[j] = (a, L, 0)
    bad = rng.random(n) < 0.03
    descs["addr"][bad] = size - 8
    descs["len"][bad] = 100
    if wire:
        from tests.wire_frames import random_frame
        for j in range(0, n, 3):
            f, L = random_frame(rng, 40)
            if L > 112 or len(f) > 112:
                continue
            a = int(descs["addr"][j])
            if a + 112 > size or bad[j]:
                continue
            umem[a:a + len(f)] = np.frombuffer(f, np.uint8)
            descs["len"][j] = L
    return umem, np.ascontiguousarray(descs[rng.permutation(n)])


@pytest.mark.parametrize("opts", [0, X.OPT_ALL])
def test_lowlat_small_frames(opts):
    """Doorbell batches of small frames (<= 112 B) at batch sizes 1-64: every byte, verdict, record and counter exactly
    the oracle's, with unaligned frames, a frame whose 64-B window the UMEM's end cuts, and descriptors the transform
    refuses."""
    _dev()
    umem, descs = _small_frames_case(0x5EEDD000 + opts, 900, opts != 0)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    for batch in (1, 5, 64):
        work = X.umem_copy(umem)
        with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT, opts=opts) as ctx:
            assert ctx.mode == X.MODE_LOWLAT
            v, r, tot = run_batches(ctx, descs, batch)
        assert (v == v_ref).all() and (r == r_ref).all(), batch
        for k in COUNTERS:
            assert tot[k] == int(s_ref[k]), (batch, k)
        diff = np.nonzero(work != ref)[0]
        assert len(diff) == 0, (batch, describe_diff(umem, work, ref, descs, v, diff))


def test_lowlat_small_frames_partial_timeout():
    """64-frame batches of small frames posted for two workgroups to a grid launched one workgroup wide: slice 0 is
    served by the resident grid, slice 1 times out untouched and takes the launch path -- every call returns 0 and
    every byte is the oracle's."""
    _dev()
    umem, descs = _small_frames_case(0x5EEDD100, 256, False)
    ref = umem.copy()
    v_ref, r_ref, _ = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=64, mode=X.MODE_LOWLAT) as ctx:
        ctx.lowlat_tune(groups=2, timeout_us=5000)
        ctx.lowlat_test_width(1)
        v, r, _ = run_batches(ctx, descs, 64)
        out = ctx.lowlat_outcomes()
    assert out["partial"] == 4 and out["untouched"] == 0, out
    assert (v == v_ref).all() and (r == r_ref).all()
    diff = np.nonzero(work != ref)[0]
    assert len(diff) == 0, describe_diff(umem, work, ref, descs, v, diff)


@pytest.mark.parametrize("mode", MODES)
def test_c1_on_a_huge_page_umem(mode):
    """BASELINE config 1 on a UMEM from xsk_gpu_umem_alloc (2 MiB aligned, transparent huge pages where the kernel
    gives them): every mode exact, 64-frame batches, scrambled recycled order."""
    _dev()
    n = 4096
    base = np.zeros(4096 * 4096, np.uint8)
    descs = oracle.synth_batch(base, n, 256, 4096, seed=0x5EED0E0E, mode=1, len_lo=20, len_hi=1500)
    descs = np.ascontiguousarray(descs[np.random.default_rng(3).permutation(n)])
    with X.HugeUmem(base.size) as u:
        u.array[:] = base
        with X.EchoContext(u.array, 0, max_batch=64, mode=mode) as ctx:
            v, r, tot = run_batches(ctx, descs, 64)
        check(base, u.array, descs, v, r, tot)
        print(f"huge-page bytes: {u.huge_bytes}")
