"""GPU parity: the gfx950 kernels (through the C ABI) vs the CPU oracle, bit for bit.

Everything here runs on a real MI355X (``-m gpu``).  Every case compares every byte of the UMEM, every
verdict, record and counter with ``oracle/`` -- the full-size BASELINE configs too (c2/c3/c4 at 1 M
frames, C5's 8 M-frame per-GPU shard), plus the re-arm round trip.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle
from tests.conftest import ROOT, golden_frames

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def to_dev(a: np.ndarray):
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(_dev())


def gpu_echo(umem: np.ndarray, descs: np.ndarray, with_recs=True, with_stats=True):
    """Run xsk_gpu_echo_dev on copies of host arrays; return (umem, verdicts, recs, stats)."""
    dev = _dev()
    n = len(descs)
    d_umem = to_dev(umem)
    d_descs = to_dev(np.ascontiguousarray(descs, X.DESC_DTYPE))
    d_verd = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=dev) if with_recs else None
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev) if with_stats else None
    ws = torch.zeros(max(X.workspace_size(0, n), 16), dtype=torch.uint8, device=dev) if with_stats else None
    X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws)
    torch.cuda.synchronize()
    out = d_umem.cpu().numpy()
    verd = d_verd.cpu().numpy()[:n]
    recs = d_recs.cpu().numpy()[: n * 16].view(X.REC_DTYPE) if with_recs else None
    stats = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0] if with_stats else None
    return out, verd, recs, stats


def check_against_oracle(umem, descs, **kw):
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, np.ascontiguousarray(descs, oracle.DESC_DTYPE))
    out, v, r, s = gpu_echo(umem, descs, **kw)
    assert (v == v_ref).all(), np.nonzero(v != v_ref)[0][:10]
    if r is not None:
        bad = np.nonzero(r != r_ref)[0]
        assert len(bad) == 0, (bad[:5], r[bad[:3]], r_ref[bad[:3]])
    if s is not None:
        for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
            assert int(s[k]) == int(s_ref[k]), k
    diff = np.nonzero(out != ref)[0]
    assert len(diff) == 0, f"{len(diff)} bytes differ, first at {diff[:8]}"
    return v_ref


# ----------------------------------------------------------------------------------------------
def test_synth_gpu_matches_oracle():
    dev = _dev()
    for mode, lo, hi, stride in [(0, 1500, 1500, 2048), (0, 64, 64, 64), (1, 64, 1500, 2048), (0, 64, 4096, 4096)]:
        n = 777
        size = n * stride + 4096
        ref = np.zeros(size, np.uint8)
        d_ref = oracle.synth_batch(ref, n, 256 if stride > 64 else 0, stride, seed=0x5EED0003, first=5, step=3,
                                   mode=mode, len_lo=lo, len_hi=hi)
        d_umem = torch.zeros(size, dtype=torch.uint8, device=dev)
        d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(d_umem, d_descs, n, 256 if stride > 64 else 0, stride, 0x5EED0003, 5, 3, mode, lo, hi)
        torch.cuda.synchronize()
        assert (d_descs.cpu().numpy().view(X.DESC_DTYPE) == d_ref.view(X.DESC_DTYPE)).all()
        got = d_umem.cpu().numpy()
        diff = np.nonzero(got != ref)[0]
        assert len(diff) == 0, (mode, stride, diff[:8])


@pytest.mark.parametrize("offset", [256, 0, 1, 2, 3, 4, 6, 8, 13, 15])
def test_golden_frames_gpu(offset):
    vecs = golden_frames()
    stride = 2048
    umem = np.zeros(len(vecs) * stride, np.uint8)
    descs = np.zeros(len(vecs), X.DESC_DTYPE)
    for i, v in enumerate(vecs):
        fr = np.frombuffer(bytes.fromhex(v["input"]), np.uint8)
        a = i * stride + offset
        umem[a:a + len(fr)] = fr
        descs[i] = (a, v["len"], 0)
    out, verd, recs, stats = gpu_echo(umem, descs)
    for i, v in enumerate(vecs):
        a = i * stride + offset
        exp = bytes.fromhex(v["output"])
        assert bytes(out[a:a + len(exp)]) == exp, v["name"]
        assert verd[i] == v["rec"]["verdict"], v["name"]
        for k, val in v["rec"].items():
            assert int(recs[i][k]) == val, (v["name"], k)
    assert (out[: offset] == 0).all()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 20000])
def test_mixed_parity(n):
    stride = 2048
    umem = np.zeros(n * stride + 64, np.uint8)
    descs = oracle.synth_batch(umem, n, 64, stride, seed=0x5EED0101 + n, mode=1, len_lo=20, len_hi=1500)
    check_against_oracle(umem, descs)


@pytest.mark.parametrize("stride,lo,hi", [(64, 64, 64), (1536, 1500, 1500), (4096, 1500, 1500), (4096, 64, 4032),
                                           (2048, 98, 98), (2048, 42, 128), (128, 98, 128)])
def test_valid_parity_layouts(stride, lo, hi):
    n = 5000
    umem = np.zeros(n * stride, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed=0x5EED0002, mode=0, len_lo=lo, len_hi=hi)
    v = check_against_oracle(umem, descs)
    assert (v == 0).all()


@pytest.mark.parametrize("off,ln", [(2, 60), (6, 98), (13, 98), (9, 64), (0, 112)])
def test_uniform_tiles_at_offsets(off, ln):
    """Tiles of identical frames at one 16-B offset (c2 / ping shapes): the per-tile byte-mask path."""
    n, stride = 4096, 2048
    umem = np.zeros(n * stride + 64, np.uint8)
    descs = oracle.synth_batch(umem, n, off, stride, seed=0x5EED0C0C + off, mode=0, len_lo=ln, len_hi=ln)
    v = check_against_oracle(umem, descs)
    assert (v == 0).all()


def test_unaligned_non_uniform_addresses():
    """Frames at random byte offsets (odd ones too) inside 4 KiB chunks, in shuffled order."""
    rng = np.random.default_rng(1)
    n = 3000
    tmp = np.zeros(n * 2048, np.uint8)
    src = oracle.synth_batch(tmp, n, 0, 2048, seed=0x5EED0404, mode=1, len_lo=20, len_hi=1900)
    umem = np.zeros(n * 4096, np.uint8)
    descs = np.zeros(n, X.DESC_DTYPE)
    order = rng.permutation(n)
    for i in range(n):
        j = order[i]
        off = int(rng.integers(0, 4096 - 2048))
        a = j * 4096 + off
        L = int(src[i]["len"])
        umem[a:a + 2048] = tmp[i * 2048:(i + 1) * 2048]
        descs[i] = (a, L, 0)
    check_against_oracle(umem, descs)


def test_jumbo_and_edge_lengths():
    """Lengths around every chunk boundary, plus jumbo frames streamed in many 1 KiB chunks."""
    lens = [20, 33, 34, 35, 36, 37, 38, 39, 41, 42, 43, 47, 48, 49, 63, 64, 65, 79, 80, 81, 1023, 1024, 1087,
            1088, 1089, 2111, 2112, 2113, 9000, 9001, 65535]
    stride = 65536 + 64
    n = len(lens) * 4
    umem = np.zeros(n * stride, np.uint8)
    descs = np.zeros(n, X.DESC_DTYPE)
    rng = np.random.default_rng(7)
    for i in range(n):
        L = lens[i % len(lens)]
        off = [0, 1, 2, 7][i // len(lens)]
        a = i * stride + off
        body = np.frombuffer(bytes.fromhex(golden_frames()[1]["input"]), np.uint8)  # valid 1500-B echo
        umem[a:a + 1500] = body
        if L > 1500:
            umem[a + 1500:a + L] = rng.integers(0, 256, L - 1500, dtype=np.uint8)
        descs[i] = (a, L, 0)
    check_against_oracle(umem, descs)


def test_bad_descriptors_gpu():
    umem = np.zeros(8192, np.uint8)
    descs = np.zeros(6, X.DESC_DTYPE)
    descs[0] = (8192, 0, 0)
    descs[1] = (8186, 20, 0)
    descs[2] = (9000, 64, 0)
    descs[3] = (8192 - 38, 20, 0)
    descs[4] = (1 << 40, 1500, 0)
    descs[5] = (0, (1 << 30) + 1, 0)
    check_against_oracle(umem, descs)


def test_outputs_optional():
    n = 500
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=99, mode=1, len_lo=20, len_hi=1500)
    check_against_oracle(umem, descs, with_recs=False, with_stats=False)


def test_n_zero_is_noop():
    dev = _dev()
    u = torch.zeros(64, dtype=torch.uint8, device=dev)
    d = torch.zeros(16, dtype=torch.uint8, device=dev)
    X.echo_dev(u, d, 0)
    torch.cuda.synchronize()


def test_stats_accumulate_across_calls():
    dev = _dev()
    n = 4096
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=123, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    _, _, s_ref = oracle.echo_batch(ref, descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, 64), dtype=torch.uint8, device=dev)
    for i in range(0, n, 64):  # RX_BATCH_SIZE batches, one call each
        X.echo_dev(d_umem, d_descs[i * 16:(i + 64) * 16], 64, None, None, d_stats, ws)
    torch.cuda.synchronize()
    s = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k])
    assert int(s["timestamp"]) == 0
    assert (d_umem.cpu().numpy() == ref).all()


def test_counters_device_atomics():
    """Every workgroup adds its counters to the caller's stats with device-scope atomics, on top of what
    they already hold, leaving `timestamp` alone (many workgroups plus a ragged tail)."""
    dev = _dev()
    n = 300_000
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=77, mode=1, len_lo=0, len_hi=1500)
    ref = umem.copy()
    _, _, s_ref = oracle.echo_batch(ref, descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    base = np.zeros(1, X.STATS_DTYPE)
    base["timestamp"], base["rx_packets"], base["rx_bytes"] = 0x1234, 5, 1 << 40
    base["tx_packets"], base["tx_bytes"] = 7, 11
    d_stats = to_dev(base)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, None, None, d_stats, ws)
    torch.cuda.synchronize()
    s = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k]) + int(base[k][0]), k
    assert int(s["timestamp"]) == 0x1234
    assert (d_umem.cpu().numpy() == ref).all()


def test_small_batches_share_stats_across_streams():
    """One-workgroup calls (RX_BATCH_SIZE frames) on four streams at once, all adding into ONE device
    stats_record: the counts are exact (device atomics, never a plain read-modify-write)."""
    dev = _dev()
    n, calls = 64, 400
    umem = np.zeros(n * calls * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n * calls, 0, 2048, seed=0x5EED5151, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    _, _, s_ref = oracle.echo_batch(ref, descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    torch.cuda.synchronize()
    for c in range(calls):
        X.echo_dev(d_umem, d_descs[c * n * 16:(c + 1) * n * 16], n, None, None, d_stats, ws, stream=streams[c % 4])
    torch.cuda.synchronize()
    s = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k]), k
    assert (d_umem.cpu().numpy() == ref).all()


@pytest.mark.parametrize("mode", [X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT])
def test_host_umem_modes(mode):
    """C1 shape: 4096 frames in a 16 MiB UMEM of 4 KiB chunks, RX batches of 64 (and one big batch)."""
    n = 4096
    umem = np.zeros(4096 * 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 4096, seed=0x5EED0001, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    for batch in (64, 4096):
        work = X.umem_copy(umem)
        with X.EchoContext(work, 0, max_batch=batch, mode=mode) as ctx:
            tot = {k: 0 for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")}
            vs, rs = [], []
            for i in range(0, n, batch):
                v, r, s = ctx.process(descs[i:i + batch])
                vs.append(v)
                rs.append(r)
                for k in tot:
                    tot[k] += int(s[k])
        assert (np.concatenate(vs) == v_ref).all()
        assert (np.concatenate(rs) == r_ref).all()
        for k in tot:
            assert tot[k] == int(s_ref[k])
        assert (work == ref).all(), np.nonzero(work != ref)[0][:8]


def test_echo_replay_tool():
    """The C host driver (tools/echo_replay) end to end against the oracle."""
    exe = os.path.join(ROOT, "tools", "echo_replay")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", ROOT, "tools/echo_replay"], check=True)
    n = 4096
    umem = np.zeros(4096 * 4096, np.uint8)
    descs = oracle.synth_batch(umem, n, 256, 4096, seed=0x5EED0001, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, _, s_ref = oracle.echo_batch(ref, descs)
    with tempfile.TemporaryDirectory() as td:
        p = lambda s: os.path.join(td, s)  # noqa: E731
        umem.tofile(p("u"))
        descs.tofile(p("d"))
        for mode, extra in (("zerocopy", []), ("staged", []), ("lowlat", []), ("lowlat", ["reps=3"]),
                            ("zerocopy", ["gpus=0,0"]), ("staged", ["gpus=0,0,0", "reps=2"])):
            r = subprocess.run([exe, p("u"), p("d"), p("o"), p("v"), "64", mode] + extra, capture_output=True,
                               text=True, timeout=300)
            assert r.returncode == 0, r.stderr
            kv = dict(x.split("=") for x in r.stdout.split())
            assert int(kv["rx_packets"]) == int(s_ref["rx_packets"])
            assert int(kv["tx_bytes"]) == int(s_ref["tx_bytes"])
            assert (np.fromfile(p("o"), np.uint8) == ref).all()
            assert (np.fromfile(p("v"), np.uint8) == v_ref).all()


def test_rearm_gpu_roundtrip():
    dev = _dev()
    n = 10000
    d_umem = torch.zeros(n * 2048, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    # valid requests only: mixed-mode frames whose input checksum is 0xFFFF (e.g. len < 34) are not
    # invertible (RFC 1624 maps both 0x0000 and 0xFFFF to 0x0800), so re-arm is exact only on these
    X.synth_dev(d_umem, d_descs, n, 0, 2048, 77, 0, 1, 0, 64, 1500)
    before = d_umem.clone()
    d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, d_verd)
    X.rearm_dev(d_umem, d_descs, d_verd, n)
    torch.cuda.synchronize()
    assert torch.equal(before, d_umem)


def _threads():
    return min(16, oracle.cpu_threads())


def full_batch_parity(n, lo, hi, stride, seed, first=0, step=1, mode=0, chunk=1 << 20):
    """Generate n frames on the GPU, transform them with ONE xsk_gpu_echo_dev call, and compare every
    byte of the slab, every verdict, record and counter with the oracle run on a host image regenerated
    by oracle.synth_batch (chunk by chunk, so host memory stays bounded); then the rearm round trip."""
    dev = _dev()
    d_umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(d_umem, d_descs, n, 0, stride, seed, first, step, mode, lo, hi)
    d_verd = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws)
    torch.cuda.synchronize()
    tot = {k: 0 for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")}
    verdicts = d_verd.cpu().numpy()
    recs = d_recs.cpu().numpy().view(X.REC_DTYPE)
    descs_all = d_descs.cpu().numpy().view(X.DESC_DTYPE)
    th = _threads()
    for j0 in range(0, n, chunk):
        m = min(chunk, n - j0)
        host = np.zeros(m * stride, np.uint8)
        descs = oracle.synth_batch(host, m, 0, stride, seed, first + j0 * step, step, mode, lo, hi, threads=th)
        assert (descs["len"] == descs_all["len"][j0:j0 + m]).all()
        v_ref, r_ref, s_ref = oracle.echo_batch(host, descs, threads=th)
        got = d_umem[j0 * stride:(j0 + m) * stride].cpu().numpy()
        diff = np.nonzero(got != host)[0]
        assert len(diff) == 0, f"frames from {j0}: {len(diff)} bytes differ, first at {diff[:8]}"
        assert (verdicts[j0:j0 + m] == v_ref).all()
        bad = np.nonzero(recs[j0:j0 + m] != r_ref)[0]
        assert len(bad) == 0, (j0 + bad[:5])
        for k in tot:
            tot[k] += int(s_ref[k])
        del host, got
    st = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for k in tot:
        assert int(st[k]) == tot[k], k
    # round trip: re-arm restores the exact generated input (valid requests only, mode 0)
    if mode == 0:
        before = torch.zeros_like(d_umem)
        X.synth_dev(before, d_descs, n, 0, stride, seed, first, step, mode, lo, hi)
        X.rearm_dev(d_umem, d_descs, d_verd, n)
        torch.cuda.synchronize()
        assert torch.equal(before, d_umem)
    return verdicts


@pytest.mark.parametrize("cfg", ["c2_64", "c3_1500", "c4_mixed"])
def test_full_size_configs(cfg):
    """BASELINE configs 2-4 at full size (1 M frames, one call): every frame byte-exact vs the oracle."""
    lo, hi, stride = {"c2_64": (64, 64, 64), "c3_1500": (1500, 1500, 4096), "c4_mixed": (64, 1500, 2048)}[cfg]
    seed = 0x5EED0000 + {"c2_64": 2, "c3_1500": 3, "c4_mixed": 4}[cfg]
    v = full_batch_parity(1 << 20, lo, hi, stride, seed)
    assert (v == 0).all()


def test_full_size_mixed_traffic():
    """1 M frames of every negative / edge case (mode 1) at a 2 KiB stride, every frame vs the oracle."""
    full_batch_parity(1 << 20, 20, 1500, 2048, 0x5EED0044, mode=1)


@pytest.mark.parametrize("rank", [0, 7])
def test_c5_shard(rank):
    """BASELINE config 5 at 8 GPUs: this rank's shard of the 64 M x 1500 B step -- 8 M frames, global
    frame first + j * 8 (round-robin, bench.py / shard.py), 2 KiB stride (16 GiB of UMEM) -- in ONE
    call, every byte of every frame vs the oracle."""
    from xsknet_amd import shard
    world = 8
    n = (1 << 26) // world
    first, step = shard.shard_range(0, n, rank, world)
    v = full_batch_parity(n, 1500, 1500, 2048, 0x5EED0005, first=first, step=step, chunk=1 << 21)
    assert (v == 0).all()


def test_timing_hook():
    dev = _dev()
    n = 65536
    d_umem = torch.zeros(n * 2048, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(d_umem, d_descs, n, 0, 2048, 5, 0, 1, 0, 1500, 1500)
    X.timing_enable(True)
    for _ in range(3):
        X.echo_dev(d_umem, d_descs, n)
    ms, cnt = X.timing_read()
    X.timing_enable(False)
    assert cnt == 3 and ms > 0


def _shifted_mixed_batch(n, stride, len_hi, seed):
    """n mixed frames (every negative / edge case) at a stride of 2048 + 16, frame j shifted by j % 7 bytes
    (odd and unaligned starts)."""
    umem = np.zeros(n * stride + 64, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed=seed, mode=1, len_lo=20, len_hi=len_hi)
    descs["addr"] += (np.arange(n) % 7).astype(np.uint64)
    for j in range(n - 1, -1, -1):  # move the bytes accordingly (back to front)
        a = j * stride
        umem[a + j % 7:a + j % 7 + 2048 + 8] = umem[a:a + 2048 + 8].copy()
    return umem, descs


def _run_grid(umem, descs, grid, opts=0):
    """The product kernel on copies of host arrays with `grid` workgroups (0 = one per CU)."""
    dev = _dev()
    n = len(descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_verd = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(max(16, X.workspace_size(0, n)), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws, opts=opts, grid=grid)
    torch.cuda.synchronize()
    return (d_umem.cpu().numpy(), d_verd.cpu().numpy(), d_recs.cpu().numpy().view(X.REC_DTYPE),
            d_stats.cpu().numpy().view(X.STATS_DTYPE)[0])


def _check_grid(umem, descs, grid, opts=0):
    ref = umem.copy()
    if opts:
        v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    else:
        v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    out, v, r, s = _run_grid(umem, descs, grid, opts)
    assert (v == v_ref).all(), np.nonzero(v != v_ref)[0][:10]
    bad = np.nonzero(r != r_ref)[0]
    assert len(bad) == 0, (bad[:5], r[bad[:3]], r_ref[bad[:3]])
    diff = np.nonzero(out != ref)[0]
    assert len(diff) == 0, f"{len(diff)} bytes differ, first at {diff[:8]}"
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k]), k


@pytest.mark.parametrize("opts", [0, 7])
@pytest.mark.parametrize("grid", [0, 1, 7])
@pytest.mark.parametrize("len_hi", [2048, 112, 48])
def test_product_kernel_geometries(grid, len_hi, opts):
    """The shipped kernel at several grid shapes (1 and 7 workgroups: shares of many rounds; 0: one per CU)
    over 3000 mixed frames at odd / unaligned starts: len_hi 112 makes tiles of ping-size frames (every frame
    within 128 B of its 16-B aligned start), 48 tiles whose frames all fit their 64-B windows; reference mode
    and wire mode with every option."""
    umem, descs = _shifted_mixed_batch(3000, 2048 + 16, len_hi, 0x5EED0707)
    _check_grid(umem, descs, grid, opts)


@pytest.mark.parametrize("opts", [0, 7])
@pytest.mark.parametrize("grid", [1, 2, 5, 16])
@pytest.mark.parametrize("n", [1, 64, 301, 1024])
def test_small_batch_workgroups(n, grid, opts):
    """Small batches (n <= XSK_GPU_LOWLAT_MAX: sub-tiles) spread over 1-16 workgroups (the tools/smallbatch.py
    geometries): every byte, verdict, record and counter exact in reference and wire mode."""
    umem, descs = _shifted_mixed_batch(n, 2048 + 16, 1500, 0x5EED3030 + n)
    _check_grid(umem, descs, grid, opts)


@pytest.mark.parametrize("flen", [20, 33, 42, 63, 64, 100, 256, 300, 769, 1024, 1500, 4000, 9000])
def test_uniform_tile_streams(flen):
    """Tiles whose frames all share one length and one 16-B offset (the uniform long-tile stream: byte masks
    computed once per tile) at several start offsets, plus a last partial tile and one odd frame out in the
    middle tile (it falls back to the ranked streams) -- 1105 frames (> XSK_GPU_LOWLAT_MAX: the round kernel),
    on 1 and 2 workgroups and one per CU."""
    n = 64 * 17 + 17
    stride = ((flen + 16 + 255) // 256) * 256 + 256
    for off in (0, 1, 6, 15):
        umem = np.zeros(n * stride + 256, np.uint8)
        descs = oracle.synth_batch(umem, n, 256 + off, stride, seed=0x5EED1919 + flen + off, mode=0, len_lo=flen,
                                   len_hi=flen)
        descs["len"][64 * 2 + 5] = max(20, flen - 1)  # one frame of tile 2 ends elsewhere: ranked streams
        for grid in (0, 1, 2):
            _check_grid(umem, descs, grid)


@pytest.mark.parametrize("case", ["packed64", "mixed_short", "one_long", "ragged"])
@pytest.mark.parametrize("grid", [1, 2, 3])
def test_short_tile_rounds(case, grid):
    """Shares of several rounds of short tiles (every frame within its 64-B window) on 1-3 workgroups, so that
    the paired short-tile path runs for real in every round of a share: 9000 frames = 141 tiles, a partial last
    tile; "one_long" puts one 200-B frame in a second-round tile (that round falls back to the row streams),
    "mixed_short" adds every negative case at odd offsets, "ragged" runs the ranked streams in every round."""
    n = 9000
    if case == "packed64":
        stride, off, mode, lo, hi = 64, 0, 0, 64, 64
    elif case == "ragged":
        stride, off, mode, lo, hi = 2048, 0, 1, 20, 1500
    else:
        stride, off, mode, lo, hi = 256, 3, 1 if case == "mixed_short" else 0, 20, 48
    umem = np.zeros(n * stride + 1024, np.uint8)
    descs = oracle.synth_batch(umem, n, off, stride, seed=0x5EED2222 + stride, mode=mode, len_lo=lo, len_hi=hi)
    if case == "one_long":
        descs["len"][64 * 40 + 9] = 200  # tile 40: the second round of workgroup 0 at grid 1
    _check_grid(umem, descs, grid)


def test_staged_pipeline_multi_chunk():
    """A host batch of several staged chunks (two-stream pipeline), mixed frames at a 2 KiB stride."""
    n = 3 * 32768 + 777
    umem = np.zeros(n * 2048, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 2048, seed=0x5EED0909, mode=1, len_lo=20, len_hi=1500)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch(ref, descs)
    work = X.umem_copy(umem)
    with X.EchoContext(work, 0, max_batch=n, mode=X.MODE_STAGED) as ctx:
        v, r, s = ctx.process(descs)
    assert (v == v_ref).all()
    assert (r == r_ref).all()
    for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(s[k]) == int(s_ref[k])
    assert (work == ref).all(), np.nonzero(work != ref)[0][:8]


# ---- XDP ingress filter (inner_xdp.c:26-61) on the device ------------------------------------------
def gpu_classify(umem, descs, bound):
    dev = _dev()
    n = len(descs)
    d_umem = to_dev(umem)
    d_descs = to_dev(np.ascontiguousarray(descs, X.DESC_DTYPE))
    act = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=dev)
    out = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=dev)
    nout = torch.full((1,), 0xFFFFFFFF, dtype=torch.int64, device=dev)
    X.classify_dev(d_umem, d_descs, n, bound, act, out, nout)
    torch.cuda.synchronize()
    k = int(nout.cpu().numpy().view(np.uint32)[0])
    return act.cpu().numpy()[:n], out.cpu().numpy().view(X.DESC_DTYPE)[:k]


@pytest.mark.parametrize("bound", [True, False])
@pytest.mark.parametrize("n,lo,hi,stride", [(1, 0, 200, 256), (255, 0, 200, 256), (257, 0, 200, 256),
                                            (1025, 0, 200, 256), (100000, 0, 1500, 1536), (70000, 64, 64, 64),
                                            (3_000_000, 20, 64, 64)])
def test_classify_parity(n, lo, hi, stride, bound):
    """Actions and the in-order REDIRECT list against the oracle, from one frame to 3 M (11 719 workgroups of the
    classify and scatter launches)."""
    umem = np.zeros(n * stride, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed=0x5EED0C0C + n, mode=1, len_lo=lo, len_hi=hi)
    a_ref, r_ref = oracle.xdp_classify_batch(umem, descs, bound)
    a, r = gpu_classify(umem, descs, bound)
    assert (a == a_ref).all(), np.nonzero(a != a_ref)[0][:8]
    assert len(r) == len(r_ref) and (r == r_ref).all()


def test_classify_golden_and_bad_descriptors():
    import json
    cls = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "classify.json")))}
    vecs = golden_frames()
    stride = 2048
    umem = np.zeros(len(vecs) * stride, np.uint8)
    descs = np.zeros(len(vecs) + 3, X.DESC_DTYPE)
    for i, v in enumerate(vecs):
        fr = np.frombuffer(bytes.fromhex(v["input"]), np.uint8)
        umem[i * stride + 3:i * stride + 3 + len(fr)] = fr  # odd start
        descs[i] = (i * stride + 3, v["len"], 0)
    descs[len(vecs)] = (umem.nbytes - 20, 34, 0)      # IPv4 header would cross the UMEM end
    descs[len(vecs) + 1] = (umem.nbytes + 5, 64, 0)   # outside
    descs[len(vecs) + 2] = (umem.nbytes - 13, 13, 0)  # short, inside: DROP by the length test
    a, r = gpu_classify(umem, descs, True)
    for i, v in enumerate(vecs):
        assert a[i] == cls[v["name"]]["bound"], v["name"]
    assert list(a[len(vecs):]) == [1, 1, 1]
    a_ref, r_ref = oracle.xdp_classify_batch(umem, descs, True)
    assert (a == a_ref).all() and (r == r_ref).all()


def test_classify_then_echo_pipeline():
    """Filter a mixed 1 M batch on the device, transform only the redirected frames, compare with the
    CPU filter + oracle transform on sampled frames and on the counters."""
    dev = _dev()
    n, stride = 1 << 20, 2048
    d_umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(d_umem, d_descs, n, 0, stride, 0x5EED0D0D, 0, 1, 1, 20, 1500)
    host = d_umem.cpu().numpy()
    descs = d_descs.cpu().numpy().view(X.DESC_DTYPE)
    act = torch.empty(n, dtype=torch.uint8, device=dev)
    red = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    nred = torch.zeros(1, dtype=torch.int64, device=dev)
    X.classify_dev(d_umem, d_descs, n, True, act, red, nred)
    torch.cuda.synchronize()
    k = int(nred.cpu().numpy().view(np.uint32)[0])
    a_ref, r_ref = oracle.xdp_classify_batch(host, descs, True)
    assert (act.cpu().numpy() == a_ref).all() and k == len(r_ref)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, k), dtype=torch.uint8, device=dev)
    verd = torch.empty(k, dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, red, k, verd, None, stats, ws)
    torch.cuda.synchronize()
    ref = host.copy()
    v_ref, _, s_ref = oracle.echo_batch(ref, r_ref, threads=8)
    assert (verd.cpu().numpy() == v_ref).all()
    st = stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    for key in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes"):
        assert int(st[key]) == int(s_ref[key])
    assert (d_umem.cpu().numpy() == ref).all()


def test_more_tiles_than_grid():
    """4.5 M packed 64-B frames: more tiles than the 16 384-workgroup grid cap, so waves loop."""
    dev = _dev()
    n, stride = 4_500_000, 64
    d_umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    d_descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(d_umem, d_descs, n, 0, stride, 0x5EED1111, 0, 1, 0, 64, 64)
    before = d_umem.clone()
    verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, verd, recs, stats, ws)
    torch.cuda.synchronize()
    st = stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    assert int(st["rx_packets"]) == n and int(st["tx_packets"]) == n and int(st["tx_bytes"]) == 64 * n
    assert bool((verd == 0).all()) and bool((recs.view(-1, 16)[:, 1] == 3).all())
    idx = np.sort(np.random.default_rng(3).choice(n, 256, replace=False))
    idx[-1] = n - 1
    got = d_umem.view(-1, stride)[torch.from_numpy(idx).to(dev)].cpu().numpy()
    for k, j in enumerate(idx):
        L, buf = oracle.synth_frame(0x5EED1111, int(j), 0, 64, 64, cap=64)
        frame = buf[:64].copy()
        d1 = np.zeros(1, oracle.DESC_DTYPE)
        d1[0] = (0, L, 0)
        oracle.echo_batch(frame, d1)
        assert (got[k] == frame).all(), j
    X.rearm_dev(d_umem, d_descs, verd, n)
    torch.cuda.synchronize()
    assert torch.equal(before, d_umem)


@pytest.mark.parametrize("mode,lo,hi,opts", [(1, 20, 1500, 0), (0, 1500, 1500, 0), (1, 20, 1500, 7), (0, 1500, 1500, 7)])
def test_tile_spanning_more_than_2gib(mode, lo, hi, opts):
    """Frames of one tile more than 2 GiB apart (the kernel's 64-bit-address path): ragged tiles take the
    sorted streams, uniform 1500-B tiles the per-step streams; reference and wire mode."""
    dev = _dev()
    size = (2 << 30) + (512 << 20)  # 2.5 GiB UMEM
    far = (2 << 30) + (64 << 20)
    n = 200
    tmp = np.zeros(n * 2048, np.uint8)
    src = oracle.synth_batch(tmp, n, 0, 2048, seed=0x5EED1212, mode=mode, len_lo=lo, len_hi=hi)
    d_umem = torch.zeros(size, dtype=torch.uint8, device=dev)
    descs = np.zeros(n, X.DESC_DTYPE)
    for i in range(n):
        a = (far if i % 2 else 0) + i * 2048 + (i % 5)
        d_umem[a:a + 2048] = torch.from_numpy(tmp[i * 2048:(i + 1) * 2048]).to(dev)
        descs[i] = (a, src[i]["len"], 0)
    d_descs = to_dev(descs)
    lo_before = d_umem[:n * 2048 + 64].cpu().numpy().copy()
    hi_before = d_umem[far:far + n * 2048 + 64].cpu().numpy().copy()
    verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, d_descs, n, verd, recs, opts=opts)
    torch.cuda.synchronize()
    # oracle on a compact host image: both regions, same relative layout
    img = np.zeros(2 * (n * 2048 + 64), np.uint8)
    img[:n * 2048 + 64] = lo_before
    img[n * 2048 + 64:] = hi_before
    hd = descs.copy()
    hd["addr"] = np.where(np.arange(n) % 2 == 1, descs["addr"] - far + n * 2048 + 64, descs["addr"])
    v_ref, r_ref, _ = oracle.echo_batch_opts(img, hd, opts)
    assert (verd.cpu().numpy() == v_ref).all()
    assert (recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    assert (d_umem[:n * 2048 + 64].cpu().numpy() == img[:n * 2048 + 64]).all()
    assert (d_umem[far:far + n * 2048 + 64].cpu().numpy() == img[n * 2048 + 64:]).all()


def test_write_through_across_4gib_regions():
    """The write phase's write-through stores address a tile's windows from the 4 GiB-aligned UMEM region they
    share: tiles whose windows lie in two regions, tiles wholly above 4 GiB, and a window that straddles the
    4 GiB line itself (plain stores for those tiles) -- every byte against the oracle (large-batch kernel)."""
    dev = _dev()
    G4 = 1 << 32
    size = G4 + (256 << 20)
    n, stride = 2048, 2048
    tmp = np.zeros(n * stride, np.uint8)
    src = oracle.synth_batch(tmp, n, 0, stride, seed=0x5EED4444, mode=0, len_lo=64, len_hi=1500)
    d_umem = torch.zeros(size, dtype=torch.uint8, device=dev)
    addr = np.zeros(n, np.uint64)
    for i in range(n):
        t = i // 64
        if t == 0:    # tile 0: windows in both regions
            a = (G4 + (64 << 20) if i % 2 else 0) + i * stride
        elif t == 1:  # tile 1: every window above 4 GiB
            a = G4 + (128 << 20) + i * stride
        elif i == 64 * 2 + 5:  # tile 2: one window across the 4 GiB line (16-B aligned, 32 B below it)
            a = G4 - 32
        else:
            a = (16 << 20) + i * stride + (i % 3) * 16
        addr[i] = a
        L = min(stride, size - a)
        d_umem[a:a + L] = torch.from_numpy(tmp[i * stride:i * stride + L]).to(dev)
    descs = np.zeros(n, X.DESC_DTYPE)
    descs["addr"], descs["len"] = addr, src["len"]
    span = 1600  # >= a frame (<= 1500 B) and its window; the frames' spans do not overlap
    spans = [(int(a), int(a) + span) for a in addr]
    before = [d_umem[s:e].cpu().numpy().copy() for s, e in spans]
    verd = torch.zeros(n, dtype=torch.uint8, device=dev)
    recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.echo_dev(d_umem, to_dev(descs), n, verd, recs)
    torch.cuda.synchronize()
    # oracle on a compact host image: each frame's span at i * span (16-B alignment kept)
    img = np.concatenate(before + [np.zeros(64, np.uint8)])
    hd = descs.copy()
    hd["addr"] = np.arange(n, dtype=np.uint64) * span
    v_ref, r_ref, _ = oracle.echo_batch(img, hd)
    assert (v_ref == 0).all()
    assert (verd.cpu().numpy() == v_ref).all()
    assert (recs.cpu().numpy().view(X.REC_DTYPE) == r_ref).all()
    for i, (s, e) in enumerate(spans):
        got = d_umem[s:e].cpu().numpy()
        assert (got == img[i * span:(i + 1) * span]).all(), i


@pytest.mark.parametrize("nbytes", [16, 16 * 1023, 16 * 4097 * 3, (1 << 26) + 16 * 77])
def test_stream_read_ceiling_reads_every_byte(nbytes):
    """xsk_gpu_stream_read_dev (the bench's read-ceiling kernel: per-workgroup contiguous shares) loads every 16-B
    vector exactly once: its sum of dwords equals the host's, for sizes that leave ragged shares and tails."""
    dev = _dev()
    rng = np.random.default_rng(nbytes)
    host = rng.integers(0, 2**32, nbytes // 4, dtype=np.uint32)
    src = torch.from_numpy(host.view(np.uint8).copy()).to(dev)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    X.stream_read_dev(src, nbytes, out)
    torch.cuda.synchronize()
    assert int(out.item()) & (2**64 - 1) == int(host.astype(np.uint64).sum()) & (2**64 - 1)
