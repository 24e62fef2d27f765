"""Random mixed traffic for the wire-format widening tests (xsk_gpu_echo_dev_opts).

Frames come from tests/golden/make_wire_golden.py's builder (an independent restatement of the
spec), with random VLAN stacks, IHL / options, fragments, tot_len errors, Ethernet padding, bad
checksums, non-ICMP / non-echo messages and truncations, placed in a UMEM at a fixed stride with
optional start offsets.
"""
import importlib.util
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("make_wire_golden", os.path.join(_HERE, "golden", "make_wire_golden.py"))
G = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(G)


def random_frame(rng: np.random.Generator, max_payload: int = 1400):
    r = rng.random
    vlan = []
    nv = rng.choice([0, 0, 0, 1, 2, 3], p=[0.4, 0.1, 0.1, 0.2, 0.15, 0.05])
    for _ in range(nv):
        vlan.append((int(rng.choice([0x8100, 0x88A8])), int(rng.integers(0, 4096))))
    ihl = 5 if r() < 0.7 else int(rng.integers(3, 16))
    opts = bytes(rng.integers(0, 256, max(0, 4 * ihl - 20), dtype=np.uint8)) if ihl > 5 else b""
    payload = bytes(rng.integers(0, 256, int(rng.integers(0, max_payload + 1)), dtype=np.uint8))
    kw = dict(
        vlan=vlan, ihl=ihl, options=opts, payload=payload,
        ethertype=0x0800 if r() < 0.9 else int(rng.choice([0x86DD, 0x0806, 0x8100])),
        version=4 if r() < 0.95 else int(rng.integers(0, 16)),
        frag=0x4000 if r() < 0.85 else int(rng.choice([0x2000, 0x0001, 0x3FFF, 0x0000, 0x8000])),
        proto=1 if r() < 0.9 else int(rng.choice([6, 17, 58])),
        itype=8 if r() < 0.85 else int(rng.choice([0, 13, 3])),
        code=0 if r() < 0.9 else int(rng.integers(1, 16)),
        ident=int(rng.integers(0, 65536)), seq=int(rng.integers(0, 65536)),
        pad=int(rng.integers(0, 40)) if r() < 0.2 else 0,
        bad_ip=r() < 0.08, bad_icmp=r() < 0.08,
        src_mac=bytes(rng.integers(0, 256, 6, dtype=np.uint8)), dst_mac=bytes(rng.integers(0, 256, 6, dtype=np.uint8)),
        saddr=bytes(rng.integers(0, 256, 4, dtype=np.uint8)), daddr=bytes(rng.integers(0, 256, 4, dtype=np.uint8)),
    )
    if r() < 0.05:
        kw["tot_len"] = int(rng.integers(0, 2000))
    f = G.build(**kw)
    L = len(f)
    if r() < 0.1:
        L = int(rng.integers(0, L + 1))
    return f, L


def mixed_batch(n: int, stride: int = 2048, seed: int = 1, offsets: bool = True, max_payload: int = 1400):
    """(umem, descs): n random frames at addr = i*stride + (i % 16 if offsets), window padding random."""
    rng = np.random.default_rng(seed)
    umem = rng.integers(0, 256, n * stride + 256, dtype=np.uint8)  # garbage around the frames
    descs = np.zeros(n, G_DESC)
    for i in range(n):
        f, L = random_frame(rng, max_payload)
        off = (i % 16) if offsets else 0
        a = i * stride + off
        assert off + len(f) <= stride
        umem[a:a + len(f)] = np.frombuffer(f, np.uint8)
        descs[i] = (a, L, 0)
    return umem, descs


G_DESC = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
