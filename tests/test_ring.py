"""AF_XDP ring loop pieces that need no GPU: the ring operations (compiled C unit test), the ctypes
mirrors of the ring structs, and xsk_gpu_tx_complete / the empty-ring path of xsk_gpu_rx_step."""
import ctypes as C
import os
import subprocess
import tempfile

import numpy as np

from tests.conftest import ROOT


def test_ring_ops_c_unit():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-o", exe,
                        os.path.join(ROOT, "tests", "c", "test_ring.c")], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    assert "ring ok" in out


def _ring(size, entry_dtype):
    ctr = np.zeros(2, np.uint32)  # producer, consumer
    slots = np.zeros(size, entry_dtype)
    import xsknet_amd as X
    r = X.Ring(0, 0, size - 1, size, ctr.ctypes.data, ctr.ctypes.data + 4, slots.ctypes.data, None)
    return r, ctr, slots


def test_tx_complete_returns_frames_to_pool():
    import xsknet_amd as X
    L = X.lib()
    comp, ctr, slots = _ring(8, np.uint64)
    # the kernel completed 5 frames (producer side)
    slots[:5] = [4096 * i for i in (3, 1, 4, 1, 5)]
    ctr[0] = 5
    stack = np.zeros(16, np.uint64)
    pool = X.FramePool(stack.ctypes.data, 2, 16)
    stack[:2] = [777, 888]
    assert L.xsk_gpu_tx_complete(C.byref(comp), C.byref(pool), 3) == 3
    assert pool.n_free == 5 and list(stack[:5]) == [777, 888, 3 * 4096, 4096, 4 * 4096]
    assert ctr[1] == 3  # consumer released
    assert L.xsk_gpu_tx_complete(C.byref(comp), C.byref(pool), 64) == 2
    assert ctr[1] == 5 and pool.n_free == 7
    assert L.xsk_gpu_tx_complete(C.byref(comp), C.byref(pool), 64) == 0


def test_rx_step_empty_ring_and_bad_args():
    import errno
    import xsknet_amd as X
    L = X.lib()
    rx, _, _ = _ring(8, X.DESC_DTYPE)
    fq, fctr, _ = _ring(8, np.uint64)
    tx, tctr, _ = _ring(8, X.DESC_DTYPE)
    fctr[1] = 0
    stack = np.zeros(4, np.uint64)
    pool = X.FramePool(stack.ctypes.data, 4, 4)
    res = X.RxResult()
    fake_ctx = C.c_void_p(0x1000)  # never dereferenced: the RX ring is empty
    assert L.xsk_gpu_rx_step(fake_ctx, C.byref(rx), C.byref(fq), C.byref(tx), C.byref(pool), 64, None,
                             C.byref(res)) == 0
    assert res.received == 0 and fctr[0] == 0 and tctr[0] == 0 and pool.n_free == 4
    assert L.xsk_gpu_rx_step(None, C.byref(rx), C.byref(fq), C.byref(tx), C.byref(pool), 64, None,
                             None) == -errno.EINVAL


def test_stats_tx_failed_applies_sendto_outcomes():
    """xsk_gpu_stats_tx_failed: the reference counts tx_* only after a successful sendto (xsk_receive.c:166-172);
    replies whose send failed are taken back out of the counters, nothing else changes."""
    import errno
    import oracle
    import xsknet_amd as X
    L = X.lib()
    n = 500
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=77, mode=1, len_lo=20, len_hi=1500)
    v, _, s = oracle.echo_batch(umem, descs)
    stats = np.zeros(1, X.STATS_DTYPE)
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        stats[k] = s[k]
    sent = (np.arange(n) % 5 != 0).astype(np.uint8)  # every fifth send fails
    got = L.xsk_gpu_stats_tx_failed(stats.ctypes.data, descs.ctypes.data, v.ctypes.data, sent.ctypes.data, n)
    fail = (v == X.TX_REPLY) & (sent == 0)
    assert got == int(fail.sum())
    ok = (v == X.TX_REPLY) & (sent == 1)
    assert int(stats["tx_packets"][0]) == int(ok.sum())
    assert int(stats["tx_bytes"][0]) == int(descs["len"][ok].sum())
    assert int(stats["rx_packets"][0]) == int(s["rx_packets"]) and int(stats["rx_bytes"][0]) == int(s["rx_bytes"])
    # argument checks; frames the counters never counted are refused, the counters untouched
    assert L.xsk_gpu_stats_tx_failed(None, descs.ctypes.data, v.ctypes.data, sent.ctypes.data, n) == -errno.EINVAL
    assert L.xsk_gpu_stats_tx_failed(stats.ctypes.data, None, v.ctypes.data, sent.ctypes.data, n) == -errno.EINVAL
    before = stats.copy()
    none_sent = np.zeros(n, np.uint8)
    assert L.xsk_gpu_stats_tx_failed(stats.ctypes.data, descs.ctypes.data, v.ctypes.data, none_sent.ctypes.data,
                                     n) == -errno.EINVAL
    assert (stats == before).all()
    assert L.xsk_gpu_stats_tx_failed(stats.ctypes.data, None, None, None, 0) == 0
