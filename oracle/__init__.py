"""CPU oracle (ctypes over oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker or the CPU baseline; the product path never does.

The C restatement (``echo_oracle.c``) follows ``/root/reference/src/lib/xsk_receive.c:101-157`` and
the batch loop ``:220-233``.  Parity pinning: the reference itself is unbuildable in this image
(``src/lib/xsk_utils.h:3`` needs ``<xdp/xsk.h>`` from libxdp, absent; stand-ins are not allowed),
so the oracle is pinned by the RFC 1071/1624 published vectors, the reference-run facts recorded
in SURVEY.md §8a, and golden frames produced by an independent restatement
(``tests/golden/make_golden.py``).  See DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

DESC_DTYPE = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
REC_DTYPE = np.dtype([
    ("verdict", "u1"), ("flags", "u1"), ("ip_proto", "u1"), ("icmp_type", "u1"),
    ("icmp_code", "u1"), ("ip_vihl", "u1"), ("eth_proto", "<u2"), ("icmp_csum_in", "<u2"),
    ("icmp_csum_out", "<u2"), ("ip_sum", "<u2"), ("icmp_sum", "<u2"),
])
STATS_DTYPE = np.dtype([("timestamp", "<u8"), ("rx_packets", "<u8"), ("rx_bytes", "<u8"),
                        ("tx_packets", "<u8"), ("tx_bytes", "<u8")])

_lib = None
_P = C.c_void_p


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def cpu_threads() -> int:
    """Worker threads for the oracle on this host: the CPUs this process may run on (the GPU box's share
    of a large machine is smaller than os.cpu_count())."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        sigs = {
            "oracle_csum_replace2": ([C.POINTER(C.c_uint16), C.c_uint16, C.c_uint16], None),
            "oracle_process_packet": ([_P, C.c_uint32], C.c_int),
            "oracle_fold_sum": ([_P, C.c_uint32, C.c_uint32], C.c_uint16),
            "oracle_echo_batch": ([_P, C.c_uint64, _P, C.c_uint32, _P, _P, _P], None),
            "oracle_echo_batch_mt": ([_P, C.c_uint64, _P, C.c_uint32, _P, _P, _P, C.c_int], None),
            "oracle_echo_batch_opts": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint32, _P, _P, _P], None),
            "oracle_echo_batch_opts_mt": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_int], None),
            "oracle_echo_batch_hdr": ([_P, _P, C.c_uint32, _P, _P], None),
            "oracle_echo_batch_hdr_mt": ([_P, _P, C.c_uint32, _P, _P, C.c_int], None),
            "oracle_synth_frame": ([C.c_uint64, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, _P, C.c_uint32],
                                   C.c_uint32),
            "oracle_synth_batch": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                    C.c_uint64, C.c_int, C.c_uint32, C.c_uint32], C.c_int),
            "oracle_synth_batch_mt": ([_P, C.c_uint64, _P, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                       C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, C.c_int], C.c_int),
            "oracle_rearm": ([_P, _P, _P, C.c_uint32], None),
            "oracle_mix64": ([C.c_uint64], C.c_uint64),
            "oracle_xdp_classify": ([_P, C.c_uint32, C.c_int], C.c_int),
            "oracle_xdp_classify_batch": ([_P, C.c_uint64, _P, C.c_uint32, C.c_int, _P, _P], C.c_uint32),
        }
        for name, (args, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def csum_replace2(field_le: int, old: int, new: int) -> int:
    v = C.c_uint16(field_le)
    lib().oracle_csum_replace2(C.byref(v), old, new)
    return v.value


def process_packet(frame: np.ndarray, length: int) -> int:
    return lib().oracle_process_packet(frame.ctypes.data, length)


def fold_sum(frame: np.ndarray, lo: int, hi: int) -> int:
    return lib().oracle_fold_sum(frame.ctypes.data, lo, hi)


def echo_batch(umem: np.ndarray, descs: np.ndarray, threads: int = 1):
    """Full contract on host arrays (umem modified in place). Returns verdicts, recs, stats."""
    n = len(descs)
    verdicts = np.zeros(n, np.uint8)
    recs = np.zeros(n, REC_DTYPE)
    stats = np.zeros(1, STATS_DTYPE)
    if threads > 1:
        lib().oracle_echo_batch_mt(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, verdicts.ctypes.data,
                                   recs.ctypes.data, stats.ctypes.data, threads)
    else:
        lib().oracle_echo_batch(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, verdicts.ctypes.data,
                                recs.ctypes.data, stats.ctypes.data)
    return verdicts, recs, stats[0]


def echo_batch_opts(umem: np.ndarray, descs: np.ndarray, opts: int, threads: int = 1):
    """xsk_gpu_echo_dev_opts' contract (wire-format widening for opts != 0) on host arrays."""
    n = len(descs)
    descs = np.ascontiguousarray(descs, DESC_DTYPE)
    verdicts = np.zeros(n, np.uint8)
    recs = np.zeros(n, REC_DTYPE)
    stats = np.zeros(1, STATS_DTYPE)
    if threads > 1:
        lib().oracle_echo_batch_opts_mt(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, opts,
                                        verdicts.ctypes.data, recs.ctypes.data, stats.ctypes.data, threads)
    else:
        lib().oracle_echo_batch_opts(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, opts, verdicts.ctypes.data,
                                     recs.ctypes.data, stats.ctypes.data)
    return verdicts, recs, stats[0]


def synth_batch(umem: np.ndarray, n: int, base_off: int, stride: int, seed: int, first: int = 0, step: int = 1,
                mode: int = 0, len_lo: int = 1500, len_hi: int = 1500, threads: int = 1) -> np.ndarray:
    descs = np.zeros(n, DESC_DTYPE)
    if threads > 1:
        rc = lib().oracle_synth_batch_mt(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, base_off, stride, seed,
                                         first, step, mode, len_lo, len_hi, threads)
    else:
        rc = lib().oracle_synth_batch(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, base_off, stride, seed,
                                      first, step, mode, len_lo, len_hi)
    if rc != 0:
        raise ValueError("oracle_synth_batch: frames do not fit the UMEM")
    return descs


def synth_frame(seed: int, gidx: int, mode: int, len_lo: int, len_hi: int, cap: int = 4096):
    buf = np.zeros(cap, np.uint8)
    L = lib().oracle_synth_frame(seed, gidx, mode, len_lo, len_hi, buf.ctypes.data, cap)
    return L, buf


def rearm(umem: np.ndarray, descs: np.ndarray, verdicts: np.ndarray) -> None:
    lib().oracle_rearm(umem.ctypes.data, descs.ctypes.data, verdicts.ctypes.data, len(descs))


def mix64(x: int) -> int:
    return lib().oracle_mix64(x)


XDP_DROP, XDP_PASS, XDP_REDIRECT = 1, 2, 4


def xdp_classify(frame: np.ndarray, length: int, target_bound: bool = True) -> int:
    return lib().oracle_xdp_classify(frame.ctypes.data, length, 1 if target_bound else 0)


def xdp_classify_batch(umem: np.ndarray, descs: np.ndarray, target_bound: bool = True):
    """inner_xdp.c:26-61 over a batch: (actions, redirected descriptors in order)."""
    n = len(descs)
    actions = np.zeros(n, np.uint8)
    out = np.zeros(max(n, 1), DESC_DTYPE)
    k = lib().oracle_xdp_classify_batch(umem.ctypes.data, umem.nbytes, descs.ctypes.data, n, 1 if target_bound else 0,
                                        actions.ctypes.data, out.ctypes.data)
    return actions, out[:k]
