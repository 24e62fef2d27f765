"""The product kernel at alternative switch values (libxsknet_amd_tune.so, xsknet_amd/csrc/tune/xsk_tune_product.hip):
the A/B candidates tools/abbench.py and `bench.py --variant` time against the shipped kernel.  None of them is on the
product path (tests/test_gpu_parity.py covers that); their parity is checked here so an A/B never times a wrong
kernel.  (Round 4 removed the round-1/2 laboratory and its ~220-test sweep: every variant there was shipped or lost.)"""
import numpy as np
import pytest

import oracle
from tests.test_gpu_parity import _dev, to_dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import xsknet_amd as X  # noqa: E402

# 0 as shipped (reference), 2 wire mode as shipped, 5 / 6 no SPLIT (reference / wire), 7 / 8 no PRIO (reference / wire),
# 9 / 13 SLACK 0 / 4, 22 / 23 wire as shipped with VLAN only / SLACK 0, 42 / 43 without HB (the header phases' windows
# read with eleven ds_read_b32 instead of three ds_read_b128; reference / wire).  (Round 5 removed 14-18, 21 and 24 with
# their switches from the product header: RS 2, LASTW, the 128-B wire windows and unpaired wire tiles, each lost in a
# committed A/B log.)
VARIANTS = [0, 2, 5, 6, 7, 8, 9, 13, 22, 23, 42, 43]
WIRE_OPTS = {2: X.OPT_ALL, 6: X.OPT_ALL, 8: X.OPT_ALL, 22: X.OPT_VLAN, 23: X.OPT_ALL, 43: X.OPT_ALL}


@pytest.mark.parametrize("variant,grid", [(v, 0) for v in VARIANTS] + [(2, 3)])
def test_product_switch_variants(variant, grid):
    """The product kernel's source at alternative switch values (tune/xsk_tune_product.hip, the A/B candidates of
    tools/abbench.py's 1000 + v) on ragged mixed traffic at odd starts, shares of many rounds: every byte, verdict,
    record and counter partial exact against the oracle (VARIANTS above)."""
    dev = _dev()
    L = X.tune_lib()
    from tests.test_gpu_parity import _shifted_mixed_batch
    umem, descs = _shifted_mixed_batch(9000, 2048 + 16, 1500, 0x5EED3232 + variant)
    ref = umem.copy()
    opts = WIRE_OPTS.get(variant, 0)
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


@pytest.mark.parametrize("variant", [5, 6])
@pytest.mark.parametrize("flen", [42, 769, 1500, 4000])
def test_product_switch_uniform_tiles(variant, flen):
    """The product kernel's switches on tiles whose frames share one length and one 16-B offset (the uniform
    stream: as shipped, i.e. SPLIT -- its row-loads in equal batches --, and without SPLIT in reference and wire mode) at four start
    offsets, with one odd frame in one tile (the general streams) and a partial last tile: bit-exact vs the oracle."""
    L = X.tune_lib()
    dev = _dev()
    n = 64 * 20 + 17  # past XSK_GPU_LOWLAT_MAX: the round kernel's geometry
    stride = ((flen + 16 + 255) // 256) * 256 + 256
    opts = WIRE_OPTS.get(variant, 0)
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


@pytest.mark.parametrize("variant", [2, 22, 23, 43])
def test_product_wire_variants_on_wire_traffic(variant):
    """The wire-mode variants on the wire generator's traffic (tests/wire_frames.py: VLAN stacks, IHL 3-15 with
    options -- headers reaching past a 64-B window --, fragments, tot_len errors, padding, bad checksums,
    truncations) at all 16 start offsets, and on the golden frames: bit-exact vs the oracle with the variant's
    options."""
    import json
    import os
    from tests.conftest import ROOT
    from tests.wire_frames import mixed_batch
    L = X.tune_lib()
    dev = _dev()
    opts = WIRE_OPTS[variant]
    umem, descs = mixed_batch(3000, 2048, seed=0x5EED4141 + variant, offsets=True)
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "wire.json")))
    g = len(cases) * 16
    gu = np.zeros(g * 2048, np.uint8)
    gd = np.zeros(g, descs.dtype)
    for i in range(g):
        fr = np.frombuffer(bytes.fromhex(cases[i // 16]["frame"]), np.uint8)
        a = i * 2048 + (i % 16)
        gu[a:a + len(fr)] = fr
        gd[i] = (a, cases[i // 16]["len"], 0)
    gd["addr"] += umem.size
    umem = np.concatenate([umem, gu])
    descs = np.ascontiguousarray(np.concatenate([descs, gd]), X.DESC_DTYPE)
    ref = umem.copy()
    v_ref, r_ref, s_ref = oracle.echo_batch_opts(ref, descs, opts)
    n = len(descs)
    d_umem, d_descs = to_dev(umem), to_dev(descs)
    d_verd = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_recs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    rc = L.xsk_gpu__product_variant(variant, 0, d_umem.data_ptr(), d_umem.numel(), d_descs.data_ptr(), n,
                                    d_verd.data_ptr(), d_recs.data_ptr(), ws.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    v = d_verd.cpu().numpy()
    bad = np.nonzero(v != v_ref)[0]
    assert len(bad) == 0, (bad[:5], v[bad[:5]], v_ref[bad[:5]])
    r = d_recs.cpu().numpy().view(X.REC_DTYPE)
    bad = np.nonzero(r != r_ref)[0]
    assert len(bad) == 0, (bad[:3], r[bad[:3]], r_ref[bad[:3]])
    out = d_umem.cpu().numpy()
    diff = np.nonzero(out != ref)[0]
    assert len(diff) == 0, f"{len(diff)} bytes differ, first at {diff[:8]}"
    part = ws[:1 << 15].cpu().numpy().view(np.uint64).reshape(-1, 4).sum(axis=0)
    assert [int(x) for x in part] == [int(s_ref[k]) for k in ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")]
