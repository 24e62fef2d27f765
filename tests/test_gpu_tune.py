"""The tuning laboratory (libxsknet_amd_tune.so, xsknet_amd/csrc/tune/): kernel variants that tools/kbench.py,
tools/abbench.py and `bench.py --variant` time against the shipped kernel.  None of them is on the product path
(tests/test_gpu_parity.py covers that); their parity is checked here so an A/B never times a wrong kernel.

By default only a few variants run (the lab's copies of the shipped parameter sets); XSK_TUNE_TESTS=1 runs the
whole sweep (every variant at three grid shapes and three length mixes, the uniform / short-tile sets, the
dynamic schedules at full size)."""
import os

import numpy as np
import pytest

import oracle
from tests.test_gpu_parity import _dev, _threads, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402

FULL = os.environ.get("XSK_TUNE_TESTS") == "1"
ALL_VARIANTS = [0, 1, 2, 3, 4, 5, 6, 50, 51, 52, 53, 54, 60, 61, 62, 63, 64, 65, 66, 67, 68, 69, 70, 71, 72, 73, 74,
                75, 76, 77, 78, 80, 81, 82, 83, 84, 86, 87, 88, 92, 93, 95, 96, 99, 101, 103, 104, 107, 108, 110, 111,
                112, 113, 116, 117, 118, 119, 121, 122, 123, 125, 126, 130, 131, 132, 133, 134, 135, 136, 137, 138,
                144, 146, 151, 152, 153, 154, 155, 156, 157, 158, 159, 163, 164, 165, 166, 170, 172, 173, 174, 175]
DEFAULT_VARIANTS = [158, 131, 170, 172, 173, 174, 175]  # the lab copy of the shipped kernel; the same with plain write-phase stores;
# the shipped switches in two 8-wave workgroups per CU, and with U = 2 / 3 / 6
full_only = pytest.mark.skipif(not FULL, reason="the full tuning sweep runs with XSK_TUNE_TESTS=1")


@pytest.mark.parametrize("variant", ALL_VARIANTS if FULL else DEFAULT_VARIANTS)
@pytest.mark.parametrize("grid", [0, 1, 7])
@pytest.mark.parametrize("len_hi", [2048, 112, 48])
def test_kernel_variants_parity(variant, grid, len_hi):
    """Every ring depth / grid shape the tuning sweep may select is bit-exact (multi-tile waves too);
    len_hi 112 makes tiles of ping-size frames (every frame within 128 B of its 16-B aligned start), 48
    tiles whose frames all fit their 64-B windows."""
    L = X.tune_lib()
    dev = _dev()
    n, stride = 3000, 2048 + 16
    umem = np.zeros(n * stride + 64, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed=0x5EED0707, mode=1, len_lo=20, len_hi=len_hi)
    descs["addr"] += (np.arange(n) % 7).astype(np.uint64)  # shift frames: odd / unaligned starts
    for j in range(n - 1, -1, -1):  # move the bytes accordingly (back to front)
        a = j * stride
        umem[a + j % 7:a + j % 7 + 2048 + 8] = umem[a:a + 2048 + 8].copy()
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)  # 93-95: queue counters at +768 KiB
    rc = L.xsk_gpu__echo_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                 d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert (d_verd.cpu().numpy() == v_ref).all()
    assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem.cpu().numpy() == ref).all()
    if variant in (93, 95, 99, 101):  # dynamic schedules leave their queue counters zeroed for the next launch
        assert int(ws[768 << 10:(768 << 10) + 36].sum().item()) == 0


@full_only
@pytest.mark.parametrize("variant", [92, 119, 121, 123, 125, 126, 133, 135, 136, 137, 138, 146, 151])
@pytest.mark.parametrize("flen", [20, 33, 42, 63, 64, 100, 256, 300, 769, 1024, 1500, 4000, 9000])
def test_uniform_tile_streams(variant, flen):
    """Tiles whose frames all share one length and one 16-B offset (the uniform long-tile stream, ULONG: byte
    masks computed once per tile) at several start offsets, plus a last partial tile and one odd frame out in
    the middle tile (it falls back to the general streams) -- bit-exact against the oracle."""
    L = X.tune_lib()
    dev = _dev()
    n = 64 * 5 + 17
    stride = ((flen + 16 + 255) // 256) * 256 + 256
    for off in (0, 1, 6, 15):
        umem = np.zeros(n * stride + 256, np.uint8)
        descs = oracle.synth_batch(umem, n, 256 + off, stride, seed=0x5EED1919 + flen + off, mode=0, len_lo=flen,
                                   len_hi=flen)
        descs["len"][64 * 2 + 5] = max(20, flen - 1)  # one frame of tile 2 ends elsewhere: general streams
        ref = umem.copy()
        v_ref, r_ref, _ = oracle.echo_batch(ref, descs)
        d_umem, d_descs = to_dev(umem), to_dev(descs)
        d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        for grid in (0, 1):
            rc = L.xsk_gpu__echo_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                         d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            assert (d_verd.cpu().numpy() == v_ref).all(), (off, grid)
            assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all(), (off, grid)
            assert (d_umem.cpu().numpy() == ref).all(), (off, grid)
            d_umem.copy_(to_dev(umem))


@full_only
@pytest.mark.parametrize("variant", [131, 146, 151, 153])
@pytest.mark.parametrize("case", ["packed64", "mixed_short", "one_long", "ragged"])
@pytest.mark.parametrize("grid", [1, 2, 3])
def test_short_tile_rounds(variant, case, grid):
    """Shares of several rounds of short tiles (every frame within its 64-B window) on 1-3 workgroups, so that
    the paired short-tile path (PAIR) runs for real in every round of a share: 9000 frames = 141 tiles, a
    partial last tile; "one_long" puts one 200-B frame in a second-round tile (that round falls back to the
    row streams), "mixed_short" adds every negative case at odd offsets."""
    L = X.tune_lib()
    dev = _dev()
    n = 9000
    if case == "packed64":
        stride, off, mode, lo, hi = 64, 0, 0, 64, 64
    elif case == "ragged":  # ranked streams in every round (the adaptive descriptor prefetch, 151)
        stride, off, mode, lo, hi = 2048, 0, 1, 20, 1500
    else:
        stride, off, mode, lo, hi = 256, 3, 1 if case == "mixed_short" else 0, 20, 48
    umem = np.zeros(n * stride + 1024, np.uint8)
    descs = oracle.synth_batch(umem, n, off, stride, seed=0x5EED2222 + stride, mode=mode, len_lo=lo, len_hi=hi)
    if case == "one_long":
        descs["len"][64 * 40 + 9] = 200  # tile 40: the second round of workgroup 0 at grid 1
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    rc = L.xsk_gpu__echo_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                 d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert (d_verd.cpu().numpy() == v_ref).all()
    assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem.cpu().numpy() == ref).all()
    part = ws[:grid * 32].cpu().numpy().view(np.uint64).reshape(grid, 4).sum(axis=0)
    assert [int(v) for v in part] == [int(s_ref[k]) for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")]


@full_only
def test_dynamic_schedule_full_size_and_reuse():
    """The dynamic schedules (tuning variants 93 / 95: per-XCD rounds; 99: a tail pool) over 1 M mixed frames, three launches on one
    workspace: every frame exact each time (the counters reset themselves between launches)."""
    L = X.tune_lib()
    dev = _dev()
    n, stride = 1 << 20, 2048
    for variant in (93, 95, 99):
        d_umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(d_umem, d_descs, n, 0, stride, 0x5EED9393, 0, 1, 0, 64, 1500)
        before = d_umem.clone()
        host = np.zeros(n * stride, np.uint8)
        descs = oracle.synth_batch(host, n, 0, stride, 0x5EED9393, 0, 1, 0, 64, 1500, threads=_threads())
        v_ref, r_ref, _ = oracle.echo_batch(host, descs, threads=_threads())
        d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        for rep in range(3):
            if rep:
                d_umem.copy_(before)
            rc = L.xsk_gpu__echo_variant(variant, 0, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                         d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            assert (d_verd.cpu().numpy() == v_ref).all()
            assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
            assert (d_umem.cpu().numpy() == host).all(), (variant, rep)
        del d_umem, before


@full_only
@pytest.mark.parametrize("variant", [160, 161, 162])
@pytest.mark.parametrize("grid", [1, 3])
def test_wire_tuning_variants(variant, grid):
    """The wire-mode round kernel from the tuning library (160: as shipped, 161: write-through write phases)
    on mixed wire traffic, shares of many rounds (1-3 workgroups), every option on, against the oracle."""
    from tests.wire_frames import random_frame
    dev = _dev()
    L = X.tune_lib()
    rng = np.random.default_rng(4242)
    pool = []
    while len(pool) < 512:
        f, ln = random_frame(rng)
        pool.append((np.frombuffer(f, np.uint8), ln))
    n, stride = 20_000, 2048
    umem = rng.integers(0, 256, n * stride + 256, dtype=np.uint8)
    descs = np.zeros(n, oracle.DESC_DTYPE)
    for i in range(n):
        fr, ln = pool[(i * 7919) % len(pool)]
        a = i * stride + (i % 16)
        umem[a:a + fr.size] = fr
        descs[i] = (a, ln, 0)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, X.OPT_ALL)
    d_umem, d_descs = to_dev(umem), to_dev(np.ascontiguousarray(descs, X.DESC_DTYPE))
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    rc = L.xsk_gpu__echo_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                 d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert (d_verd.cpu().numpy() == v_ref).all()
    assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem.cpu().numpy() == ref).all()
    part = ws[:grid * 32].cpu().numpy().view(np.uint64).reshape(grid, 4).sum(axis=0)
    assert [int(v) for v in part] == [int(s_ref[k]) for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")]


@pytest.mark.parametrize("variant", [0, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("grid", [0, 1, 3])
def test_product_switch_variants(variant, grid):
    """The product kernel's source at alternative switch values (tune/xsk_tune_product.hip, the A/B candidates of
    tools/abbench.py's 1000 + v) on ragged mixed traffic at odd starts, shares of many rounds: every byte, verdict,
    record and counter partial exact against the oracle (0: reference mode as shipped, 2: wire mode with every
    option, 3 / 4: reference mode with 4 / 8 row-loads per batch in the ranked streams instead of 6, 5 / 6: the uniform
    stream without SPLIT (batches of 4 and a remainder), reference / wire mode, 7 / 8: without PRIO, reference / wire)."""
    dev = _dev()
    L = X.tune_lib()
    from tests.test_gpu_parity import _shifted_mixed_batch
    umem, descs = _shifted_mixed_batch(9000, 2048 + 16, 1500, 0x5EED3232 + variant)
    ref = umem.copy()
    opts = X.OPT_ALL if variant in (2, 6, 8) else 0
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    n = len(descs)
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    rc = L.xsk_gpu__product_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                    d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert (d_verd.cpu().numpy() == v_ref).all()
    assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem.cpu().numpy() == ref).all()
    part = ws[:1 << 15].cpu().numpy().view(np.uint64).reshape(-1, 4).sum(axis=0)  # every partial row (<= 1024)
    assert [int(x) for x in part] == [int(s_ref[k]) for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")]


@pytest.mark.parametrize("variant", [0, 5, 6, 7, 8])
@pytest.mark.parametrize("flen", [20, 42, 64, 100, 300, 769, 1024, 1500, 2300, 4000])
def test_product_switch_uniform_tiles(variant, flen):
    """The product kernel's switches on tiles whose frames share one length and one 16-B offset (the uniform
    stream: as shipped, i.e. SPLIT -- its row-loads in equal batches --, and without SPLIT in reference and wire mode) at four start
    offsets, with one odd frame in one tile (the general streams) and a partial last tile: bit-exact vs the oracle."""
    L = X.tune_lib()
    dev = _dev()
    n = 64 * 20 + 17  # past XSK_GPU_LOWLAT_MAX: the round kernel's geometry
    stride = ((flen + 16 + 255) // 256) * 256 + 256
    opts = X.OPT_ALL if variant in (6, 8) else 0
    for off in (0, 1, 6, 15):
        umem = np.zeros(n * stride + 256, np.uint8)
        descs = oracle.synth_batch(umem, n, 256 + off, stride, seed=0x5EED2121 + flen + off, mode=0, len_lo=flen,
                                   len_hi=flen)
        descs["len"][64 * 7 + 5] = max(20, flen - 1)
        ref = umem.copy()
        v_ref, r_ref, _ = oracle.echo_batch_opts(ref, descs, opts)
        d_umem, d_descs = to_dev(umem), to_dev(descs)
        d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
        for grid in (0, 1, 3):
            rc = L.xsk_gpu__product_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                            d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            assert (d_verd.cpu().numpy() == v_ref).all(), (off, grid)
            assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all(), (off, grid)
            assert (d_umem.cpu().numpy() == ref).all(), (off, grid)
            d_umem.copy_(to_dev(umem))


@full_only
@pytest.mark.parametrize("variant", [0, 1, 2, 4])
@pytest.mark.parametrize("grid", [0, 1, 3])
def test_slack_candidate_variants(variant, grid):
    """The round-4 candidate SLACK (tune/xsk_tune_slack.hip: the product kernel built from a patched copy of its header;
    heavy waves write once all but SLACK waves have read) on ragged mixed traffic at odd starts: every byte, verdict,
    record and counter partial exact against the oracle (the write-phase wait is a schedule, never a dependency)."""
    dev = _dev()
    L = X.tune_lib()
    from tests.test_gpu_parity import _shifted_mixed_batch
    umem, descs = _shifted_mixed_batch(9000, 2048 + 16, 1500, 0x5EED3535 + variant)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, 0)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    n = len(descs)
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    rc = L.xsk_gpu__slack_variant(variant, grid, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                  d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    assert (d_verd.cpu().numpy() == v_ref).all()
    assert (d_recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem.cpu().numpy() == ref).all()
    part = ws[:1 << 15].cpu().numpy().view(np.uint64).reshape(-1, 4).sum(axis=0)
    assert [int(x) for x in part] == [int(s_ref[k]) for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")]
