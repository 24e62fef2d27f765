"""CPU oracle vs published KATs, SURVEY-recorded reference facts and golden frames (no GPU)."""
import numpy as np
import pytest

import oracle
from tests.conftest import golden_frames, golden_kat

VERD = oracle  # noqa


def bswap16(x):
    return ((x & 0xFF) << 8) | (x >> 8)


def test_rfc1071_example():
    k = golden_kat()["rfc1071_example"]
    b = np.frombuffer(bytes.fromhex(k["bytes"]), np.uint8).copy()
    assert oracle.fold_sum(b, 0, len(b)) == k["folded_sum"]
    assert (~oracle.fold_sum(b, 0, len(b))) & 0xFFFF == k["checksum"]


def test_rfc1624_eqn3_example():
    k = golden_kat()["rfc1624_eqn3"]
    # byte-order independence: the same numbers work on host-order and swapped operands
    assert oracle.csum_replace2(k["HC"], k["m"], k["m_new"]) == k["HC_new"]
    assert oracle.csum_replace2(bswap16(k["HC"]), bswap16(k["m"]), bswap16(k["m_new"])) == bswap16(k["HC_new"])
    assert k["HC_new"] != k["HC_new_eqn2"]


def test_ipv4_header_example():
    k = golden_kat()["ipv4_header_b861"]
    b = np.frombuffer(bytes.fromhex(k["bytes"]), np.uint8).copy()
    assert (~oracle.fold_sum(b, 0, 20)) & 0xFFFF == k["checksum"]
    b[10], b[11] = k["checksum"] >> 8, k["checksum"] & 0xFF
    assert oracle.fold_sum(b, 0, 20) == 0xFFFF


def closed_form(old_be):
    s = ((~old_be) & 0xFFFF) + 0xF7FF
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def test_csum_replace2_exhaustive_closed_form():
    """0/65536 mismatches vs the network-order closed form; 0 only from 0xF7FF."""
    samples = golden_kat()["csum_replace2_8_0"]["samples"]
    zero_from = []
    for old_be in range(65536):
        out_le = oracle.csum_replace2(bswap16(old_be), 8, 0)  # the reference loads the field LE
        out_be = bswap16(out_le)
        assert out_be == closed_form(old_be), hex(old_be)
        assert out_be != 0xFFFF
        if out_be == 0:
            zero_from.append(old_be)
    assert zero_from == [0xF7FF]
    for k, v in samples.items():
        assert bswap16(oracle.csum_replace2(bswap16(int(k, 16)), 8, 0)) == v


@pytest.mark.parametrize("vec", golden_frames(), ids=lambda v: v["name"])
def test_golden_frame(vec):
    frame = bytes.fromhex(vec["input"])
    umem = np.zeros(4096, np.uint8)
    addr = 256  # XDP_PACKET_HEADROOM-like offset inside a 4 KiB chunk
    umem[addr:addr + len(frame)] = np.frombuffer(frame, np.uint8)
    descs = np.zeros(1, oracle.DESC_DTYPE)
    descs[0] = (addr, vec["len"], 0)
    verdicts, recs, stats = oracle.echo_batch(umem, descs)
    assert bytes(umem[addr:addr + len(frame)]) == bytes.fromhex(vec["output"])
    for k, v in vec["rec"].items():
        assert int(recs[0][k]) == v, k
    assert verdicts[0] == vec["rec"]["verdict"]
    assert stats["rx_packets"] == 1 and stats["rx_bytes"] == vec["len"]
    assert stats["tx_packets"] == (1 if vec["rec"]["verdict"] == 0 else 0)
    # nothing outside [addr, addr+38) may change
    assert not umem[:addr].any() and not umem[addr + len(frame):].any()


def test_process_packet_matches_batch_on_golden():
    for vec in golden_frames():
        f = np.frombuffer(bytes.fromhex(vec["input"]), np.uint8).copy()
        v = oracle.process_packet(f, vec["len"])
        assert v == vec["rec"]["verdict"]
        assert bytes(f) == bytes.fromhex(vec["output"])


def test_bad_descriptors():
    umem = np.zeros(4096, np.uint8)
    descs = np.zeros(4, oracle.DESC_DTYPE)
    descs[0] = (4096, 0, 0)        # addr == size, len 0: in bounds (empty)
    descs[1] = (4090, 20, 0)       # needs 38 bytes -> out of bounds
    descs[2] = (5000, 64, 0)       # out of bounds
    descs[3] = (4096 - 38, 20, 0)  # exactly fits the 38-byte header read
    v, recs, st = oracle.echo_batch(umem, descs)
    assert list(v) == [1, 5, 5, 2]
    assert st["rx_packets"] == 4 and st["rx_bytes"] == 0 + 20 + 64 + 20 and st["tx_packets"] == 0


def test_synth_valid_frames_verify():
    umem = np.zeros(64 * 2048, np.uint8)
    descs = oracle.synth_batch(umem, 64, 0, 2048, seed=7, mode=0, len_lo=64, len_hi=1500)
    assert (descs["len"] >= 64).all() and (descs["len"] <= 1500).all()
    v, recs, st = oracle.echo_batch(umem, descs)
    assert (v == 0).all()
    assert (recs["flags"] == 3).all()  # IP and ICMP checksums of the generated requests verify
    assert st["tx_bytes"] == descs["len"].sum()


def test_synth_mixed_covers_all_verdicts():
    n = 4000
    umem = np.zeros(n * 128, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 128, seed=3, mode=1, len_lo=64, len_hi=128)
    v, recs, st = oracle.echo_batch(umem, descs)
    counts = np.bincount(v, minlength=6)
    assert counts[0] > 0 and counts[1] > 0 and counts[2] > 0 and counts[3] > 0 and counts[4] > 0
    # bad-checksum and all-zero cases are accepted by the reference gates
    assert ((recs["flags"] & 2) == 0)[v == 0].any()
    assert (recs["icmp_csum_in"] == 0xF7FF).any() and ((recs["icmp_csum_out"] == 0) & (v == 0)).any()


def test_synth_deterministic_and_sharded():
    """Frame j of a (first, step) shard is global frame first + j*step (round-robin sharding)."""
    a = np.zeros(16 * 2048, np.uint8)
    d_all = oracle.synth_batch(a, 16, 0, 2048, seed=11, mode=1, len_lo=64, len_hi=1500)
    for rank in range(4):
        b = np.zeros(4 * 2048, np.uint8)
        d = oracle.synth_batch(b, 4, 0, 2048, seed=11, first=rank, step=4, mode=1, len_lo=64, len_hi=1500)
        for j in range(4):
            g = rank + 4 * j
            L = d[j]["len"]
            assert L == d_all[g]["len"]
            assert bytes(b[j * 2048:j * 2048 + max(L, 64)]) == bytes(a[g * 2048:g * 2048 + max(L, 64)])


def test_rearm_restores_requests():
    umem = np.zeros(256 * 2048, np.uint8)
    descs = oracle.synth_batch(umem, 256, 0, 2048, seed=5, mode=0, len_lo=64, len_hi=1500)
    before = umem.copy()
    v, _, _ = oracle.echo_batch(umem, descs)
    assert (umem != before).any()
    oracle.rearm(umem, descs, v)
    assert (umem == before).all()


def test_mt_matches_single_thread():
    n = 3000
    u1 = np.zeros(n * 256, np.uint8)
    descs = oracle.synth_batch(u1, n, 0, 256, seed=9, mode=1, len_lo=20, len_hi=200)
    u2 = u1.copy()
    v1, r1, s1 = oracle.echo_batch(u1, descs)
    v2, r2, s2 = oracle.echo_batch(u2, descs, threads=4)
    assert (v1 == v2).all() and (r1 == r2).all() and s1 == s2 and (u1 == u2).all()
    # more threads than frames, and the synth side
    u3 = np.zeros(n * 256, np.uint8)
    d3 = oracle.synth_batch(u3, n, 0, 256, seed=9, mode=1, len_lo=20, len_hi=200, threads=7)
    assert (d3 == descs).all()
    v4, r4, s4 = oracle.echo_batch(u3[:5 * 256].copy(), d3[:5], threads=16)
    v5, r5, s5 = oracle.echo_batch(u3[:5 * 256].copy(), d3[:5])
    assert (v4 == v5).all() and (r4 == r5).all() and s4 == s5


@pytest.mark.parametrize("opts", [1, 2, 7])
def test_wire_mt_matches_single_thread(opts):
    from tests.wire_frames import mixed_batch
    u1, descs = mixed_batch(3000, 2048, seed=31 + opts, offsets=True)
    u2 = u1.copy()
    v1, r1, s1 = oracle.echo_batch_opts(u1, descs, opts)
    v2, r2, s2 = oracle.echo_batch_opts(u2, descs, opts, threads=5)
    assert (v1 == v2).all() and (r1 == r2).all() and s1 == s2 and (u1 == u2).all()


def test_xdp_classify_golden():
    """oracle_xdp_classify (inner_xdp.c:26-61) against the independent restatement's actions."""
    import json
    import os
    from tests.conftest import ROOT
    cls = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "classify.json")))}
    for vec in golden_frames():
        f = np.frombuffer(bytes.fromhex(vec["input"]), np.uint8).copy()
        c = cls[vec["name"]]
        assert oracle.xdp_classify(f, vec["len"], True) == c["bound"], vec["name"]
        assert oracle.xdp_classify(f, vec["len"], False) == c["unbound"], vec["name"]


def test_xdp_classify_batch_compacts_in_order():
    n = 3000
    umem = np.zeros(n * 256, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, 256, seed=21, mode=1, len_lo=0, len_hi=200)
    act, red = oracle.xdp_classify_batch(umem, descs, True)
    assert set(np.unique(act)) <= {1, 2, 4} and (act == 4).any() and (act == 2).any() and (act == 1).any()
    assert (red == descs[act == 4]).all()
    act0, red0 = oracle.xdp_classify_batch(umem, descs, False)
    assert len(red0) == 0 and ((act0 == 1) == ((act == 1) | (act == 4))).all()
    # every frame of >= 34 B the echo transform would accept is one the filter redirects; the filter
    # drops 20..33-B frames (inner_xdp.c:41-42) that process_packet's len >= 20 gate would accept
    v, _, _ = oracle.echo_batch(umem.copy(), descs)
    assert (act[(v == 0) & (descs["len"] >= 34)] == 4).all()
    assert (act[(v == 0) & (descs["len"] < 34)] == 1).all()


# ---- wire-format widening (xsk_gpu_echo_dev_opts) -------------------------------
def _wire_golden():
    import json
    import os
    from tests.conftest import ROOT
    with open(os.path.join(ROOT, "tests", "golden", "wire.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("off", [0, 1, 3, 16])
def test_wire_oracle_matches_golden(off):
    """The C oracle's wire mode against the independent Python restatement's vectors (all 7 option sets)."""
    for case in _wire_golden():
        fr = bytes.fromhex(case["frame"])
        L = case["len"]
        for opts, exp in case["results"].items():
            umem = np.zeros(2048, np.uint8)
            umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
            d = np.zeros(1, oracle.DESC_DTYPE)
            d[0] = (off, L, 0)
            v, r, s = oracle.echo_batch_opts(umem, d, int(opts))
            assert v[0] == exp["verdict"], (case["name"], L, opts)
            assert {k: int(r[0][k]) for k in r.dtype.names} == exp["rec"], (case["name"], L, opts)
            assert umem[off:off + max(L, 1)].tobytes().hex() == exp["out"], (case["name"], L, opts)
            assert int(s["tx_packets"]) == (1 if exp["verdict"] == 0 else 0)


def test_wire_opts_zero_is_reference_mode():
    umem = np.zeros(300 * 2048, np.uint8)
    descs = oracle.synth_batch(umem, 300, 0, 2048, seed=0x5EED0B0B, mode=1, len_lo=20, len_hi=1500)
    a, b = umem.copy(), umem.copy()
    va, ra, sa = oracle.echo_batch(a, descs)
    vb, rb, sb = oracle.echo_batch_opts(b, descs, 0)
    assert (va == vb).all() and (ra == rb).all() and (a == b).all() and sa == sb


@pytest.mark.parametrize("opts", [1, 2, 3, 4, 5, 6, 7])
def test_wire_oracle_matches_python_spec_on_random_traffic(opts):
    """Two independent restatements of the wire spec agree on random mixed traffic."""
    from tests.wire_frames import G, mixed_batch
    umem, descs = mixed_batch(600, 2048, seed=opts, offsets=True)
    work = umem.copy()
    v, r, s = oracle.echo_batch_opts(work, descs, opts)
    tx = 0
    for i, d in enumerate(descs):
        a, L = int(d["addr"]), int(d["len"])
        frame = umem[a:a + 128 + L].tobytes()
        ev, erec, eout = G.expect(frame, L, opts)
        assert v[i] == ev, (i, opts)
        assert {k: int(r[i][k]) for k in r.dtype.names} == erec, (i, opts)
        assert work[a:a + L].tobytes() == eout[:L], (i, opts)
        tx += ev == 0
    assert int(s["tx_packets"]) == tx and int(s["rx_packets"]) == len(descs)
    # every reply of a verified request verifies again (the incremental update is exact)
    if opts & 4:
        for i in np.nonzero(v == 0)[0]:
            a = int(descs[i]["addr"])
            hl = 4 * (int(r[i]["ip_vihl"]) & 15) if opts & 1 else 20
            frame = work[a:a + int(descs[i]["len"])].tobytes()
            # locate l3 by skipping tags exactly like the spec
            l3, et = 14, (frame[12] << 8) | frame[13]
            while opts & 2 and l3 < 22 and et in (0x8100, 0x88A8):
                et = (frame[l3 + 2] << 8) | frame[l3 + 3]
                l3 += 4
            l4 = l3 + hl
            end = l3 + ((frame[l3 + 2] << 8) | frame[l3 + 3]) if opts & 1 else len(frame)
            assert G.csum16(frame[l4:end]) == 0xFFFF
