"""The AF_XDP RX loop step (xsk_gpu_rx_step / xsk_gpu_tx_complete) end to end on the GPU.

The test plays the kernel side of an AF_XDP socket over the reference client's UMEM shape (4096
frames of 4096 B, src/lib/xsk_utils.h:6-7, fill queue prefilled with 2048 frames as
src/lib/xsk_utils.c:110-120 does, libxdp's default 2048-entry rings): it takes frames from the fill
ring, writes packets at a 256-B headroom into them, posts RX descriptors, collects TX descriptors,
checks every transmitted reply byte for byte against the CPU oracle, and completes them.  The loop
must transform every packet exactly as process_packet() would and account the same counters.
"""
import collections
import ctypes as C

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402
from tests.wire_frames import random_frame  # noqa: E402

NUM_FRAMES, FRAME_SIZE, RING, HEADROOM = 4096, 4096, 2048, 256


class KRing:
    """One ring's shared state: producer/consumer indices + slots, and the app-side view."""

    def __init__(self, dtype, app_is_producer):
        self.ctr = np.zeros(2, np.uint32)  # [producer, consumer]
        self.slots = np.zeros(RING, dtype)
        base = self.ctr.ctypes.data
        self.view = X.Ring(0, RING if app_is_producer else 0, RING - 1, RING, base, base + 4,
                           self.slots.ctypes.data, None)

    # kernel side
    def k_avail(self):
        return int((int(self.ctr[0]) - int(self.ctr[1])) & 0xFFFFFFFF)

    def k_pop(self, n):
        c = int(self.ctr[1])
        out = [self.slots[(c + i) & (RING - 1)].copy() for i in range(n)]
        self.ctr[1] = (c + n) & 0xFFFFFFFF
        return out

    def k_push(self, items):
        p = int(self.ctr[0])
        for i, it in enumerate(items):
            self.slots[(p + i) & (RING - 1)] = it
        self.ctr[0] = (p + len(items)) & 0xFFFFFFFF


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _drive(step, flush, step_batch, cap, n_pkts=20000, seed=0x5EED0A0A, opts=0, wire=False, umem=None):
    """Play the kernel side around `step(rx, fq, tx, pool, step_batch, totals) -> (frames completed, RxResult)` (and,
    for a pipelined loop, `flush(tx, pool, totals)` once the last packet is in): every transmitted reply and every
    frame handed back is checked byte for byte against the oracle (with wire options `opts`), in RX order, and the
    counters at the end.  wire: the packets are the wire generator's (VLAN stacks, IHL 3-15, fragments, padding, bad
    checksums, tests/wire_frames.py) instead of the reference-mode generator's mixed traffic.  umem: a caller-owned
    zeroed uint8 array of NUM_FRAMES * FRAME_SIZE bytes (e.g. X.HugeUmem's) instead of a fresh page-aligned one."""
    if umem is None:
        umem = X.umem_zeros(NUM_FRAMES * FRAME_SIZE)
    assert umem.dtype == np.uint8 and umem.size == NUM_FRAMES * FRAME_SIZE
    rx, fq = KRing(X.DESC_DTYPE, False), KRing(np.uint64, True)
    tx, cq = KRing(X.DESC_DTYPE, True), KRing(np.uint64, False)
    # app: prefill the fill ring with 2048 frames, keep the rest on the free stack
    stack = np.zeros(NUM_FRAMES, np.uint64)
    fq.slots[:] = np.arange(RING, dtype=np.uint64) * FRAME_SIZE
    fq.ctr[0] = RING
    fq.view.cached_prod = RING
    stack[:NUM_FRAMES - RING] = np.arange(RING, NUM_FRAMES, dtype=np.uint64) * FRAME_SIZE
    pool = X.FramePool(stack.ctypes.data, NUM_FRAMES - RING, NUM_FRAMES)

    expect = {}  # addr -> (packet index, len, expected output bytes, verdict)
    totals = np.zeros(1, X.STATS_DTYPE)
    ref_tot = {"rx_packets": 0, "rx_bytes": 0, "tx_packets": 0, "tx_bytes": 0}
    rng = np.random.default_rng(5)
    rng_w = np.random.default_rng(seed ^ 0x77)
    sent = 0
    replies_seen = 0
    delivered = collections.deque()  # RX order

    def kernel_tx(got):
        nonlocal replies_seen
        # kernel: transmit -> check bytes -> complete
        txd = tx.k_pop(tx.k_avail())
        for t in txd:
            a, L = int(t["addr"]), int(t["len"])
            i, L0, exp, verdict = expect.pop(a)
            assert L == L0 and verdict == X.TX_REPLY
            assert bytes(umem[a:a + len(exp)]) == bytes(exp), i
            replies_seen += 1
        cq.k_push(np.array([int(t["addr"]) for t in txd], np.uint64))
        X.lib().xsk_gpu_tx_complete(C.byref(cq.view), C.byref(pool), RING)
        # frames the step completed but did not send went back to the pool untouched by anyone else yet: their bytes
        # must match the oracle too
        for _ in range(got):
            a = delivered.popleft()
            if a in expect:
                i, L0, exp, verdict = expect.pop(a)
                assert verdict != X.TX_REPLY
                assert bytes(umem[a:a + len(exp)]) == bytes(exp), i

    guard = 0
    while sent < n_pkts or rx.k_avail():
        guard += 1
        assert guard < 100000
        # kernel: deliver a burst into frames taken from the fill ring
        burst = min(int(rng.integers(1, 200)), fq.k_avail(), RING - rx.k_avail(), n_pkts - sent)
        descs = []
        for addr in fq.k_pop(burst):
            # aligned-chunk mode: the kernel masks a fill address to its chunk (the free stack
            # holds descriptor addresses, headroom included, as xsk_free_umem_frame stores them)
            a = (int(addr) & ~(FRAME_SIZE - 1)) + HEADROOM
            if wire:
                f, L = random_frame(rng_w, int(rng_w.choice([40, 200, 1400])))
                buf = np.zeros(FRAME_SIZE - HEADROOM, np.uint8)
                m = min(len(f), FRAME_SIZE - HEADROOM)
                buf[:m] = np.frombuffer(f, np.uint8)[:m]
                L = min(L, FRAME_SIZE - HEADROOM)
            else:
                L, buf = oracle.synth_frame(seed, sent, 1, 20, 1500, cap=FRAME_SIZE - HEADROOM)
            umem[a:a + FRAME_SIZE - HEADROOM] = buf[:FRAME_SIZE - HEADROOM]
            ref = buf[:FRAME_SIZE - HEADROOM].copy()
            d1 = np.zeros(1, oracle.DESC_DTYPE)
            d1[0] = (0, L, 0)
            v, _, st = oracle.echo_batch_opts(ref, d1, opts)
            for k in ref_tot:
                ref_tot[k] += int(st[k])
            expect[a] = (sent, L, ref[:max(L, 64)].copy(), int(v[0]))
            descs.append((a, L, 0))
            delivered.append(a)
            sent += 1
        if descs:
            rx.k_push(np.array(descs, X.DESC_DTYPE))
        got, res = step(umem, rx.view, fq.view, tx.view, pool, step_batch, totals)
        assert got <= cap and res.received <= step_batch
        assert res.tx_full == 0
        kernel_tx(got)
    if flush is not None:
        got, res = flush(tx.view, pool, totals)
        kernel_tx(got)
    assert sent == n_pkts and not delivered and not expect
    assert replies_seen == ref_tot["tx_packets"]
    for k in ref_tot:
        assert int(totals[0][k]) == ref_tot[k], k
    # every frame is accounted for: free stack + fill ring + nothing in flight
    assert pool.n_free + fq.k_avail() == NUM_FRAMES
    return umem


@pytest.mark.parametrize("mode,ctx_batch,step_batch", [(X.MODE_ZEROCOPY, 1024, 64), (X.MODE_STAGED, 1024, 64),
                                                      (X.MODE_LOWLAT, 1024, 64), (X.MODE_LOWLAT, 64, 1024),
                                                      (X.MODE_ZEROCOPY, 64, 1024), (X.MODE_STAGED, 1024, 1024)])
def test_rx_loop_end_to_end(mode, ctx_batch, step_batch):
    """ctx_batch < step_batch: the step peeks no more than the context takes (never an -EINVAL after the
    fill ring was restocked).  The free stack recycles frames LIFO (xsk_receive.c:55-71), so after the first wrap
    every step's addresses are scattered over the UMEM: STAGED steps of up to 1024 frames take the gather copy-in."""
    _dev()
    holder = {}

    def step(umem, rx, fq, tx, pool, n, totals):
        if "ctx" not in holder:
            holder["ctx"] = X.EchoContext(umem, 0, max_batch=ctx_batch, mode=mode)
        return holder["ctx"].rx_step(rx, fq, tx, pool, n, totals)

    try:
        _drive(step, None, step_batch, min(ctx_batch, step_batch))
    finally:
        if "ctx" in holder:
            holder["ctx"].close()
