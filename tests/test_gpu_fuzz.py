"""Randomised parity over every entry point (round 5): random frame layouts, lengths, offsets, traffic, wire options and
batch splits, each against the oracle byte for byte.

A case draws n frames and places them as the ABI's ownership contract allows (`include/xsk_gpu.h`: a frame owns
[addr, addr + max(len, 64)), frames of a call never overlap): packed back to back, at a stride, or with random gaps,
at any byte offset, in a shuffled descriptor order (the RX ring after AF_XDP's free stack has recycled frames,
`src/lib/xsk_receive.c:55-71`), plus a few descriptors that do not fit the UMEM.  The frames are the generator's
reference-mode traffic (valid requests and every negative of SURVEY §8c) or the wire generator's (VLAN stacks, IHL
3-15, fragments, padding, bad checksums).  Each case then runs through one entry point -- the device-resident call, a
ZEROCOPY / STAGED (with or without the UMEM's device alias) / LOWLAT context or a 2- or 3-context multi object on the one
GPU in random batch splits -- with random wire
options, and every byte of the UMEM, every verdict, record and counter must equal the oracle's.  Seeds are fixed: a
failure names its case."""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402
from tests.test_gpu_host import COUNTERS  # noqa: E402
from tests.wire_frames import random_frame  # noqa: E402

ENTRIES = ["device", "zerocopy", "staged", "staged_noalias", "lowlat", "multi"]
OPTS = [0, 0, X.OPT_STRICT_IPV4, X.OPT_VLAN, X.OPT_VERIFY_CSUM, X.OPT_ALL]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def make_case(seed):
    """(umem, descs, opts, entry, splits) of one fuzz case."""
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 3, 17, 64, 200, 1000, 1025, 5000, 40000]))
    wire_traffic = rng.random() < 0.4
    frames = []
    if wire_traffic:
        for _ in range(n):
            f, L = random_frame(rng, int(rng.choice([40, 200, 1400])))
            frames.append((np.frombuffer(f, np.uint8), L))
    else:
        lo, hi = [(0, 64), (20, 200), (42, 1500), (64, 4000)][int(rng.integers(0, 4))]
        tmp = np.zeros(n * 4096, np.uint8)
        d = oracle.synth_batch(tmp, n, 0, 4096, seed=seed, mode=1, len_lo=max(lo, 20), len_hi=hi,
                               threads=min(8, oracle.cpu_threads()))
        for j in range(n):
            L = int(d["len"][j])
            frames.append((tmp[j * 4096:j * 4096 + max(L, 1)], L))
    layout = ["packed", "stride", "gaps"][int(rng.integers(0, 3))]
    max_own = max(max(L, 64) for _, L in frames)
    stride = max(int(rng.choice([2048, 4096])), (max_own + 16 + 2047) // 2048 * 2048) if layout == "stride" else 0
    addrs, a = [], int(rng.integers(0, 64))
    for j, (_, L) in enumerate(frames):
        own = max(L, 64)
        if layout == "stride":
            a = j * stride + (int(rng.integers(0, 16)) if rng.random() < 0.3 else 0)
            assert own <= stride - 16
        addrs.append(a)
        if layout == "packed":
            a += own
        elif layout == "gaps":
            a += own + int(rng.choice([0, int(rng.integers(1, 16)), int(rng.integers(16, 600))]))
    size = (max(x + max(L, 64) for x, (_, L) in zip(addrs, frames)) + 4096 + 15) & ~15
    umem = rng.integers(0, 256, size, dtype=np.uint8)  # garbage between the frames
    descs = np.zeros(n, X.DESC_DTYPE)
    for j, ((f, L), x) in enumerate(zip(frames, addrs)):
        umem[x:x + min(L, len(f))] = f[:L]
        descs[j] = (x, L, 0)
    bad = rng.random(n) < 0.01  # descriptors that do not fit the UMEM (DROP_BAD_DESC, nothing read or written)
    descs["addr"][bad] = size - 8
    descs["len"][bad] = 100
    descs = np.ascontiguousarray(descs[rng.permutation(n)] if rng.random() < 0.7 else descs)
    opts = int(rng.choice(OPTS)) if wire_traffic or rng.random() < 0.5 else 0
    entry = ENTRIES[int(rng.integers(0, len(ENTRIES)))]
    if entry == "lowlat":
        splits = int(rng.choice([1, 7, 64, 128, 1024]))
    elif entry == "device":
        splits = n
    else:
        splits = int(rng.choice([64, 1000, n]))
    return umem, descs, opts, entry, splits


@pytest.mark.parametrize("seed", range(120))
def test_fuzz_parity(seed):
    dev = _dev()
    umem, descs, opts, entry, splits = make_case(0x5EED7000 + seed)
    n = len(descs)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    case = f"seed {seed}: n={n} opts={opts} entry={entry} splits={splits}"
    if entry == "device":
        d_umem = torch.from_numpy(umem.copy()).to(dev)
        d_descs = torch.from_numpy(descs.view(np.uint8).copy()).to(dev)
        d_verd = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        d_stats = torch.zeros(40, dtype=torch.uint8, device=dev)
        ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
        X.echo_dev(d_umem, d_descs, n, d_verd, d_recs, d_stats, ws, opts=opts)
        torch.cuda.synchronize()
        work, v = d_umem.cpu().numpy(), d_verd.cpu().numpy()
        r = d_recs.cpu().numpy().view(X.REC_DTYPE)
        st = d_stats.cpu().numpy().view(X.STATS_DTYPE)[0]
        tot = {k: int(st[k]) for k in COUNTERS}
    else:
        rng = np.random.default_rng(seed)
        mode = {"zerocopy": X.MODE_ZEROCOPY, "staged": X.MODE_STAGED, "staged_noalias": X.MODE_STAGED,
                "lowlat": X.MODE_LOWLAT, "multi": int(rng.choice([X.MODE_ZEROCOPY, X.MODE_STAGED, X.MODE_LOWLAT]))}[entry]
        work = X.umem_copy(umem)
        vs, rs, tot = [], [], {k: 0 for k in COUNTERS}
        mk = (lambda: X.MultiContext(work, [0] * int(rng.integers(2, 4)), max_batch=splits, mode=mode, opts=opts)) \
            if entry == "multi" else (lambda: X.EchoContext(work, 0, max_batch=splits, mode=mode, opts=opts))
        with mk() as ctx:
            modes = [X.ContextView(ctx.context(g)).mode for g in range(len(ctx.status()))] if entry == "multi" \
                else [ctx.mode]
            case += f" modes={modes}"
            if entry == "staged_noalias":
                ctx.drop_alias(int(rng.choice([0, 8192, 65536])))
            for i in range(0, n, splits):
                v, r, st = ctx.process(descs[i:i + splits])
                vs.append(v)
                rs.append(r)
                for k in COUNTERS:
                    tot[k] += int(st[k])
        v, r = np.concatenate(vs), np.concatenate(rs)
    bad = np.nonzero(v != v_ref)[0]
    if len(bad):
        nb = np.nonzero(work != ref)[0]
        raise AssertionError(f"{case}: {len(bad)} verdicts differ, first {bad[:8]}: got {v[bad[:8]]} want "
                             f"{v_ref[bad[:8]]}, descs {descs[bad[:8]]}; {len(nb)} UMEM bytes differ, first {nb[:8]}")
    assert (r == r_ref).all(), (case, np.nonzero(r != r_ref)[0][:8])
    for k in COUNTERS:
        assert tot[k] == int(s_ref[k]), (case, k)
    diff = np.nonzero(work != ref)[0]
    assert len(diff) == 0, (case, f"{len(diff)} bytes differ, first at {diff[:8]}")
