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

# 0 as shipped (reference), 2 wire mode as shipped, 3 / 4 ranked streams with 4 / 8 row-loads per batch, 5 / 6 no SPLIT
# (reference / wire), 7 / 8 no PRIO (reference / wire), 9 / 13 SLACK 0 / 4, 14 / 15 / 16 lean ranked streams (RS 2) with
# 6 / 8 / 4 row-loads per batch, 17 / 18 no write-phase wait in the last round (reference / wire)
VARIANTS = [0, 2, 3, 4, 5, 6, 7, 8, 9, 13, 14, 15, 16, 17, 18]
WIRE_VARIANTS = (2, 6, 8, 18)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("grid", [0, 3])
def test_product_switch_variants(variant, grid):
    """The product kernel's source at alternative switch values (tune/xsk_tune_product.hip, the A/B candidates of
    tools/abbench.py's 1000 + v) on ragged mixed traffic at odd starts, shares of many rounds: every byte, verdict,
    record and counter partial exact against the oracle (VARIANTS above)."""
    dev = _dev()
    L = X.tune_lib()
    from tests.test_gpu_parity import _shifted_mixed_batch
    umem, descs = _shifted_mixed_batch(9000, 2048 + 16, 1500, 0x5EED3232 + variant)
    ref = umem.copy()
    opts = X.OPT_ALL if variant in WIRE_VARIANTS else 0
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
