"""GPU parity of the wire-format widening (xsk_gpu_echo_dev_opts) against the CPU
oracle (oracle_echo_batch_opts) and the independent Python spec's golden vectors, bit for bit."""
import json
import os

import numpy as np
import pytest

import oracle
from tests.conftest import ROOT

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402
from tests.wire_frames import mixed_batch  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def to_dev(a):
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(_dev())


def gpu_wire(umem, descs, opts):
    dev = _dev()
    n = len(descs)
    d_umem = to_dev(umem)
    d_descs = to_dev(np.ascontiguousarray(descs, X.DESC_DTYPE))
    d_verd = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.full((max(n, 1) * 16,), 0xEE, dtype=torch.uint8, device=dev)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(max(X.workspace_size(0, n), 16), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws, opts=opts)
    torch.cuda.synchronize()
    return (d_umem.cpu().numpy(), d_verd.cpu().numpy()[:n], d_recs.cpu().numpy()[:n * 16].view(X.REC_DTYPE),
            d_stats.cpu().numpy().view(X.STATS_DTYPE)[0])


def check(umem, descs, opts):
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    out, v, r, s = gpu_wire(umem, descs, opts)
    bad = np.nonzero(v != v_ref)[0]
    assert len(bad) == 0, (bad[:5], v[bad[:5]], v_ref[bad[:5]])
    bad = np.nonzero(r != r_ref)[0]
    assert len(bad) == 0, (bad[:3], r[bad[:3]], r_ref[bad[:3]])
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k]), k
    diff = np.nonzero(out != ref)[0]
    assert len(diff) == 0, f"{len(diff)} bytes differ, first at {diff[:8]}"
    return v_ref


@pytest.mark.parametrize("opts", [1, 2, 3, 4, 5, 6, 7])
def test_wire_golden_gpu(opts):
    """Every golden frame at all 16 start offsets, against the Python spec's expected outputs."""
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "wire.json")))
    stride = 2048
    n = len(cases) * 16
    umem = np.zeros(n * stride, np.uint8)
    descs = np.zeros(n, oracle.DESC_DTYPE)
    for i in range(n):
        c = cases[i // 16]
        fr = np.frombuffer(bytes.fromhex(c["frame"]), np.uint8)
        a = i * stride + (i % 16)
        umem[a:a + len(fr)] = fr
        descs[i] = (a, c["len"], 0)
    out, v, r, s = gpu_wire(umem, descs, opts)
    for i in range(n):
        c = cases[i // 16]
        exp = c["results"][str(opts)]
        assert v[i] == exp["verdict"], (c["name"], c["len"], i % 16)
        assert {k: int(r[i][k]) for k in r.dtype.names} == exp["rec"], (c["name"], c["len"], i % 16)
        a, L = int(descs[i]["addr"]), int(descs[i]["len"])
        assert out[a:a + max(L, 1)].tobytes().hex() == exp["out"], (c["name"], L, i % 16)
    check(umem, descs, opts)


@pytest.mark.parametrize("opts", [1, 2, 4, 7])
@pytest.mark.parametrize("n", [1, 64, 65, 3000])
def test_wire_mixed_parity(opts, n):
    umem, descs = mixed_batch(n, 2048, seed=1000 + n + opts, offsets=True)
    v = check(umem, descs, opts)
    if n >= 3000:  # the mix really exercises the gates
        assert len(np.unique(v)) >= (6 if opts == 7 else 4)


def test_wire_aligned_sector_path_and_window_edge():
    """16-B aligned replies (64-B sector write-back) at a 1536-B stride, plus frames whose 128-B window
    runs past the UMEM end and descriptors past it (DROP_BAD_DESC)."""
    umem, descs = mixed_batch(2000, 1536, seed=77, offsets=False, max_payload=1300)
    check(umem, descs, 7)
    # last frame flush with the UMEM end: window clipped
    L = 70
    umem2 = umem[: int(descs[-1]["addr"]) + L + (16 - L % 16) % 16].copy()
    d2 = descs.copy()
    d2[-1]["len"] = min(int(d2[-1]["len"]), L)
    d2[-2]["addr"] = umem2.size - 8  # frame leaving the UMEM
    d2[-3]["addr"] = umem2.size + 64
    v = check(umem2, d2, 7)
    assert v[-2] == X.DROP_BAD_DESC and v[-3] == X.DROP_BAD_DESC


@pytest.mark.parametrize("mode", [X.MODE_ZEROCOPY, X.MODE_STAGED])
def test_wire_host_umem_modes(mode):
    _dev()
    umem, descs = mixed_batch(3000, 2048, seed=5, offsets=True)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, 7)
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=1024, mode=mode, opts=7) as ctx:
        vs, rs, tx = [], [], 0
        for i in range(0, len(descs), 1024):
            v, r, s = ctx.process(descs[i:i + 1024])
            vs.append(v)
            rs.append(r)
            tx += int(s["tx_packets"])
    assert (np.concatenate(vs) == v_ref).all()
    assert (np.concatenate(rs) == r_ref).all()
    assert tx == int(s_ref["tx_packets"])
    assert (work == ref).all(), np.nonzero(work != ref)[0][:8]


def test_wire_bad_options_rejected():
    dev = _dev()
    d = torch.zeros(4096, dtype=torch.uint8, device=dev)
    with pytest.raises(X.XskGpuError):
        X.echo_dev(d, d, 1, opts=8)


def wire_full_batch_parity(n, lo, hi, stride, seed, opts, mode=0, chunk=1 << 19):
    """n frames generated on the GPU, transformed in wire mode by ONE xsk_gpu_echo_dev_opts call; every byte of
    the slab, every verdict, record and counter against oracle_echo_batch_opts on a host image regenerated by
    oracle.synth_batch chunk by chunk (bounded host memory)."""
    from tests.test_gpu_parity import _threads
    dev = _dev()
    d_umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(d_umem, d_descs, n, 0, stride, seed, 0, 1, mode, lo, hi)
    d_verd = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws, opts=opts)
    torch.cuda.synchronize()
    verdicts = d_verd.cpu().numpy()
    recs = d_recs.cpu().numpy().view(X.REC_DTYPE)
    descs_all = d_descs.cpu().numpy().view(X.DESC_DTYPE)
    tot = {k: 0 for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")}
    th = _threads()
    for j0 in range(0, n, chunk):
        m = min(chunk, n - j0)
        host = np.zeros(m * stride, np.uint8)
        descs = oracle.synth_batch(host, m, 0, stride, seed, j0, 1, mode, lo, hi, threads=th)
        assert (descs["len"] == descs_all["len"][j0:j0 + m]).all()
        v_ref, r_ref, s_ref = oracle.echo_batch_opts(host, descs, opts, threads=th)
        got = d_umem[j0 * stride:(j0 + m) * stride].cpu().numpy()
        diff = np.nonzero(got != host)[0]
        assert len(diff) == 0, f"frames from {j0}: {len(diff)} bytes differ, first at {diff[:8]}"
        bad = np.nonzero(verdicts[j0:j0 + m] != v_ref)[0]
        assert len(bad) == 0, (j0 + bad[:5])
        bad = np.nonzero(recs[j0:j0 + m] != r_ref)[0]
        assert len(bad) == 0, (j0 + bad[:5])
        for k in tot:
            tot[k] += int(s_ref[k])
        del host, got
    st = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for k in tot:
        assert int(st[k]) == tot[k], k
    return verdicts, recs


@pytest.mark.parametrize("cfg", ["c2_64", "c3_1500", "c4_mixed"])
def test_wire_full_size_configs(cfg):
    """BASELINE configs 2-4 at full size (1 M frames, one call) in wire mode with every option on: every frame
    byte-exact vs the oracle (the widening replaces the fixed offsets of xsk_receive.c:120-121)."""
    lo, hi, stride = {"c2_64": (64, 64, 64), "c3_1500": (1500, 1500, 4096), "c4_mixed": (64, 1500, 2048)}[cfg]
    seed = 0x5EED0000 + {"c2_64": 2, "c3_1500": 3, "c4_mixed": 4}[cfg]
    v, r = wire_full_batch_parity(1 << 20, lo, hi, stride, seed, X.OPT_ALL)
    assert (v == 0).all() and ((r["flags"] & 3) == 3).all()


@pytest.mark.parametrize("opts", [1, 2, 7])
def test_wire_full_size_mixed_traffic(opts):
    """1 M frames of every negative / edge case (synth mode 1) at a 2 KiB stride in wire mode, every frame vs
    the oracle."""
    v, _ = wire_full_batch_parity(1 << 20, 20, 1500, 2048, 0x5EED0044 + opts, opts, mode=1)
    assert len(np.unique(v)) >= 5


def test_wire_multi_round_mixed():
    """More tiles than one round of the persistent grid (270 K frames: several rounds per workgroup) of
    random mixed traffic at odd and even offsets, every option on; also hits the STRICT re-read of a
    message that ends before its frame and past the 128-B window."""
    from tests.wire_frames import G, random_frame
    _dev()
    rng = np.random.default_rng(42)
    pool = []
    while len(pool) < 2048:
        f, L = random_frame(rng)
        pool.append((np.frombuffer(f, np.uint8), L))
    # a few frames whose tot_len ends the message past the window but before the frame end
    for _ in range(64):
        f = G.build(payload=bytes(rng.integers(0, 256, 900, dtype=np.uint8)), tot_len=400, pad=0)
        pool.append((np.frombuffer(f, np.uint8), len(f)))
    n, stride = 270_000, 2048
    umem = rng.integers(0, 256, n * stride + 256, dtype=np.uint8)
    descs = np.zeros(n, oracle.DESC_DTYPE)
    for i in range(n):
        fr, L = pool[(i * 7919) % len(pool)]
        a = i * stride + (i % 16)
        umem[a:a + fr.size] = fr
        descs[i] = (a, L, 0)
    v = check(umem, descs, X.OPT_ALL)
    assert (v == X.DROP_BAD_IP).any() and (v == 0).any()
