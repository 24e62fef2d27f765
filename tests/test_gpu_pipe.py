"""The pipelined RX loop (xsk_gpu_rx_pipe_*) end to end on the GPU, against the same simulated AF_XDP kernel side as
tests/test_gpu_rxloop.py (whose driver, `_drive`, plays it): up to `depth` batches in flight, one per context over one
registration of the UMEM, completed in RX order, every frame, verdict and counter exactly the oracle's.

Round 5 ran these last (the file was test_gpu_zpipe.py) after tests that ran later in the same process had seen
replies land a few pages away from their host frames on some boxes; round 6 put them back in collection order once the
host UMEMs of every test were page-aligned (xsk_gpu_init now requires it, as AF_XDP does) -- DESIGN.md §4 has the
investigation and what it did and did not establish.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402
from tests.test_gpu_rxloop import _dev, _drive  # noqa: E402


@pytest.mark.parametrize("mode,depth,step_batch", [(X.MODE_LOWLAT, 2, 64), (X.MODE_LOWLAT, 4, 64),
                                                   (X.MODE_LOWLAT, 3, 1024), (X.MODE_ZEROCOPY, 3, 64),
                                                   (X.MODE_STAGED, 2, 256), (X.MODE_LOWLAT, 1, 64)])
def test_rx_pipe_end_to_end(mode, depth, step_batch):
    """The pipelined loop (xsk_gpu_rx_pipe_*): up to `depth` batches in flight, one per context, completed in RX order;
    every frame, verdict and counter exactly xsk_gpu_rx_step's (the oracle's), nothing left in flight after the flush."""
    _dev()
    holder = {}

    def step(umem, rx, fq, tx, pool, n, totals):
        if "p" not in holder:
            holder["p"] = X.RxPipe(umem, 0, depth=depth, mode=mode)
        got, res = holder["p"].step(rx, fq, tx, pool, n, totals)
        assert holder["p"].inflight <= depth
        return got, res

    def flush(tx, pool, totals):
        got, res = holder["p"].flush(tx, pool, totals)
        assert holder["p"].inflight == 0
        return got, res

    try:
        _drive(step, flush, step_batch, depth * step_batch)
    finally:
        if "p" in holder:
            holder["p"].close()


def test_rx_pipe_partial_timeouts():
    """Every batch of a pipelined LOWLAT loop times out half served -- each context's resident grid is launched one
    workgroup wide while its batches are posted for two (xsk_gpu__lowlat_test_width) -- and completes through the
    launch path: still every frame exact, in order, and the contexts' outcome counters show the partial services."""
    _dev()
    holder = {}

    def step(umem, rx, fq, tx, pool, n, totals):
        if "p" not in holder:
            p = holder["p"] = X.RxPipe(umem, 0, depth=2, mode=X.MODE_LOWLAT)
            for i in range(2):
                c = p.context(i)
                if c.mode == X.MODE_LOWLAT:
                    c.lowlat_tune(groups=2, timeout_us=3000)
                    c.lowlat_test_width(1)
        return holder["p"].step(rx, fq, tx, pool, n, totals)

    try:
        _drive(step, lambda tx, pool, totals: holder["p"].flush(tx, pool, totals), 64, 2 * 64, n_pkts=3000)
        lowlat = [holder["p"].context(i) for i in range(2) if holder["p"].context(i).mode == X.MODE_LOWLAT]
        assert lowlat, "no LOWLAT slot on this device"
        for c in lowlat:
            oc = c.lowlat_outcomes()
            assert oc["partial"] > 0 and oc["untouched"] == 0, oc
    finally:
        if "p" in holder:
            holder["p"].close()


@pytest.mark.parametrize("seed", range(12))
def test_rx_pipe_randomised(seed):
    """Random pipes: mode, depth, step size, wire options and traffic drawn per seed (fixed seeds), every frame exact."""
    _dev()
    rng = np.random.default_rng(0x5EEDB000 + seed)
    mode = int(rng.choice([X.MODE_LOWLAT, X.MODE_LOWLAT, X.MODE_ZEROCOPY, X.MODE_STAGED]))
    depth = int(rng.integers(1, X.RX_PIPE_MAX + 1))
    step_batch = int(rng.choice([1, 7, 64, 200, 1024]))
    wire = bool(rng.random() < 0.5)
    opts = int(rng.choice([0, X.OPT_VLAN, X.OPT_STRICT_IPV4, X.OPT_VERIFY_CSUM, X.OPT_ALL])) if wire else 0
    holder = {}

    def step(umem, rx, fq, tx, pool, n, totals):
        if "p" not in holder:
            holder["p"] = X.RxPipe(umem, 0, depth=depth, mode=mode, opts=opts)
        return holder["p"].step(rx, fq, tx, pool, n, totals)

    try:
        _drive(step, lambda tx, pool, totals: holder["p"].flush(tx, pool, totals), step_batch, depth * step_batch,
               n_pkts=4000, seed=0x5EEDB100 + seed, opts=opts, wire=wire)
    finally:
        if "p" in holder:
            holder["p"].close()


@pytest.mark.parametrize("reserved", [2, 4])
def test_rx_pipe_keeps_doorbell_contexts_only(reserved):
    """A LOWLAT pipe deeper than the device's free resident-kernel slots keeps the LOWLAT contexts it got and lets the
    first downgraded one go (completion is in RX order: one launched context among doorbell ones holds every batch
    behind it -- 4 LOWLAT + 4 ZEROCOPY ran 5.2 Mframes/s against 29 for the 4 alone, profiles/r05/lowlat_hwq8.jsonl).
    With `reserved` of the hardware queues set aside for the application (xsk_gpu_lowlat_reserve): 2 -> a depth-8
    request holds cap LOWLAT contexts; 4 -> no slot at all, so all 8 run ZEROCOPY.  Every frame exact, in order."""
    _dev()
    import gc
    gc.collect()
    cap = X.lowlat_reserve(0, reserved)
    holder = {}
    try:
        def step(umem, rx, fq, tx, pool, n, totals):
            if "p" not in holder:
                p = holder["p"] = X.RxPipe(umem, 0, depth=8, mode=X.MODE_LOWLAT)
                modes = [p.context(i).mode for i in range(p.depth)]
                if cap:
                    assert 1 <= p.depth <= cap and modes == [X.MODE_LOWLAT] * p.depth, (cap, modes)
                else:
                    assert p.depth == 8 and modes == [X.MODE_ZEROCOPY] * 8, modes
            return holder["p"].step(rx, fq, tx, pool, n, totals)

        _drive(step, lambda tx, pool, totals: holder["p"].flush(tx, pool, totals), 64, 8 * 64, n_pkts=8000)
    finally:
        if "p" in holder:
            holder["p"].close()
        X.lowlat_reserve(0, 0)


@pytest.mark.parametrize("mode", [X.MODE_LOWLAT, X.MODE_ZEROCOPY])
def test_rx_pipe_on_a_huge_page_umem(mode):
    """The pipelined loop over a UMEM from xsk_gpu_umem_alloc (2 MiB aligned, transparent huge pages where the kernel
    gives them; the registration then covers whole huge pages): depth 4, 64-frame steps, every frame exact."""
    _dev()
    holder = {}

    def step(umem, rx, fq, tx, pool, n, totals):
        if "p" not in holder:
            holder["p"] = X.RxPipe(umem, 0, depth=4, mode=mode)
        return holder["p"].step(rx, fq, tx, pool, n, totals)

    def flush(tx, pool, totals):
        got, res = holder["p"].flush(tx, pool, totals)
        assert holder["p"].inflight == 0
        return got, res

    from tests.test_gpu_rxloop import FRAME_SIZE, NUM_FRAMES
    with X.HugeUmem(NUM_FRAMES * FRAME_SIZE) as u:
        try:
            _drive(step, flush, 64, 4 * 64, umem=u.array)
        finally:
            if "p" in holder:
                holder["p"].close()
        print(f"huge-page bytes: {u.huge_bytes}")


def test_eight_doorbell_channels_under_gpu_max_hw_queues_8():
    """XSK_GPU_LOWLAT_PER_DEVICE is 8, the cap min(8, GPU_MAX_HW_QUEUES): a process started with GPU_MAX_HW_QUEUES=8
    runs a depth-8 LOWLAT pipe on eight resident kernels.  tools/rxring in a child process (the variable is read by the
    runtime at its start): 64-frame steps for a second, every context LOWLAT, every reply checked, no failure, no
    timeout."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "rxring")
    if not os.path.exists(exe):
        pytest.skip("tools/rxring not built (make)")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([exe, "64", "lowlat", "1", "pipe=8", "len=64", "ring=16384", "frames=16384", "nic=burst"],
                       capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-500:], r.stderr[-500:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    q = d["per_queue"][0]
    print(f"depth-8 pipe under GPU_MAX_HW_QUEUES=8: {q['mframes_s']} Mframes/s")
    assert q["mode"] == X.MODE_LOWLAT  # (the pipe's last context: all eight kept their slot)
    assert d["failures"] == 0 and d["checked"] == d["frames"] > 0 and q["rc"] == 0
    assert q["lowlat_timeouts_all_partial_failed_late"] == [0, 0, 0, 0] and d["tx_full"] == 0
