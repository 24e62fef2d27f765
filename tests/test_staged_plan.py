"""STAGED chunking (CPU): the graduated tail of xsk_gpu_host.c's stage_chunk covers every frame once, ends in chunks
of at most TAIL_FRAMES, and never needs more chunk slots than stage_chunks_max() gives a context at init."""
import numpy as np

from tests.staged_plan import CHUNK_FRAMES, TAIL_FRAMES, stage_chunks, stage_chunks_max


def test_chunks_cover_the_batch_and_fit_the_slots():
    rng = np.random.default_rng(3)
    ns = list(range(1, 70000, 97)) + [int(x) for x in rng.integers(1, 1 << 22, 400)] + \
        [CHUNK_FRAMES, CHUNK_FRAMES + 1, 2 * CHUNK_FRAMES, 2 * CHUNK_FRAMES - 1, 262144, 1 << 20]
    for n in ns:
        ch = stage_chunks(n)
        assert sum(ch) == n and min(ch) > 0, n
        assert len(ch) <= stage_chunks_max(n), (n, len(ch))
        assert all(m <= CHUNK_FRAMES for m in ch), n
        if n > CHUNK_FRAMES:
            assert ch[-1] <= TAIL_FRAMES, (n, ch[-4:])
            assert all(m % 16 == 0 for m in ch[:-1]), n  # (a chunk boundary keeps 16-frame alignment)
        else:
            assert ch == [n]


def test_host_inclusive_shape():
    """262 144 frames (the bench's host-inclusive call): seven full chunks, then 16 384, 8 192, 4 096, 4 096."""
    assert stage_chunks(262144) == [CHUNK_FRAMES] * 7 + [16384, 8192, 4096, 4096]


# ---- the copy-in planner (xsk_stage_plan.h) ---------------------------------------------------------------------------
import ctypes as C  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402
import tempfile  # noqa: E402

import pytest  # noqa: E402

from tests.conftest import ROOT  # noqa: E402
from tests import staged_plan as SP  # noqa: E402

DESC = np.dtype([("addr", "<u8"), ("len", "<u4"), ("options", "<u4")])
SRC = os.path.join(ROOT, "tests", "c", "test_stage_plan.c")


def test_stage_plan_c_unit():
    """The planner's decisions on hand-built layouts (tests/c/test_stage_plan.c)."""
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-I", "/opt/rocm/include", "-o", exe, SRC],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=60).stdout
    assert "stage plan ok" in out


@pytest.fixture(scope="module")
def cplan():
    td = tempfile.mkdtemp()
    so = os.path.join(td, "libplan.so")
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-DSHIM", "-shared", "-fPIC", "-I", "/opt/rocm/include",
                    "-o", so, SRC], check=True)
    L = C.CDLL(so)
    L.xsk_test_stage_plan.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                      C.POINTER(C.c_uint64)]

    def plan(d, umem_size, wire=False, have_alias=True, prefix=True):
        d = np.ascontiguousarray(d, DESC)
        out = (C.c_uint64 * 9)()
        L.xsk_test_stage_plan(d.ctypes.data, len(d), umem_size, int(wire), int(have_alias), int(prefix), out)
        kind, n = int(out[0]), len(d)
        moved = {SP.TWO_D: n * int(out[7]), SP.SPAN: int(out[4]) - int(out[3])}.get(kind, int(out[8]))
        return kind, bool(out[1]), bool(out[2]), int(out[8]), (moved if int(out[8]) else 0)
    return plan


def _descs(addrs, lens):
    d = np.zeros(len(addrs), DESC)
    d["addr"] = addrs
    d["len"] = lens
    return d


def test_stage_plan_matches_restatement(cplan):
    """The C planner and the Python restatement agree on random layouts: strided, scrambled, packed, mixed alignment,
    wire and reference mode, with and without a mapped alias, any call prefix."""
    rng = np.random.default_rng(11)
    U = 1 << 28
    for t in range(400):
        n = int(rng.choice([1, 2, 7, 64, 500, 1024, 1025, 3000]))
        kind = t % 4
        if kind == 0:  # uniform stride, ragged or uniform lengths
            s = int(rng.choice([64, 128, 1024, 2048, 4096]))
            addrs = int(rng.integers(0, 64)) * 16 + np.arange(n, dtype=np.int64) * s
            lens = rng.integers(20, s + 1, n) if rng.random() < 0.5 else np.full(n, int(rng.integers(14, s + 1)))
        elif kind == 1:  # scrambled 2 KiB slots
            addrs = rng.permutation(n * 2)[:n].astype(np.int64) * 2048 + int(rng.choice([0, 0, 256, 3]))
            lens = rng.integers(0, 1600, n)
        elif kind == 2:  # packed back to back
            lens = rng.integers(int(rng.choice([14, 64, 1537])), 1552, n)
            addrs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        else:  # packed, then reordered
            lens = rng.integers(60, 200, n)
            addrs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)[rng.permutation(n)]
        d = _descs(addrs, lens)
        for wire in (False, True):
            for alias in (True, False):
                for prefix in (True, False):
                    want = SP.stage_plan(d, U, wire, alias, prefix)
                    assert cplan(d, U, wire, alias, prefix) == want, (t, kind, n, wire, alias, prefix)


def packed_reordered(n, seed=77):
    """frames packed back to back at odd lengths (1537..1551 B), descriptors reordered so that the
    call's first chunks hold every unaligned-start frame and its last chunks every aligned-start one."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1537, 1552, n).astype(np.int64)
    addrs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    order = np.concatenate([np.flatnonzero(addrs & 15), np.flatnonzero((addrs & 15) == 0)])
    return _descs(addrs[order], lens[order])


def test_plan_packed_reordered_aligned_tail_not_contained(cplan):
    """The aligned-start frames at the end of the call read spans whose last 16-B block reaches into an unaligned
    neighbour that an earlier chunk rewrites: every chunk after the first unaligned one is ordered (not contained),
    although its own frames are all aligned."""
    n = 3 * SP.CHUNK_FRAMES + 777
    d = packed_reordered(n)
    U = int(d["addr"][-1]) + 4096 * 4
    plans = SP.call_plans(d, U)
    chunks = SP.stage_chunks(n)
    assert plans[-1][2] and plans[-2][2], "the tail chunks hold only aligned-start frames"
    assert not any(p[1] for p in plans), plans
    # the same chunk judged alone (round 4's per-chunk rule) would have been contained
    i0 = sum(chunks[:-1])
    assert cplan(d[i0:], U, prefix=True)[1] and not cplan(d[i0:], U, prefix=False)[1]


def two_d_with_gap_frames(seed=9):
    """chunk 0 holds small frames placed in the stride gaps of later chunks' shorter frames; the
    later chunks are 1500-B frames at a 2 KiB stride, one in ten of them 150 B shorter (one 2-D copy each)."""
    C0 = SP.CHUNK_FRAMES
    n_str = 2 * C0
    base = 1 << 22  # (chunk 0's other frames lie below it)
    addrs = base + np.arange(n_str, dtype=np.int64) * 2048
    lens = np.full(n_str, 1500, np.int64)
    short = np.arange(0, n_str, 10)
    lens[short] = 1350
    gap = addrs[short] + 1360  # a 64-B frame in the gap [1350, 1504) of each short frame's row
    other = np.arange(C0 - len(gap), dtype=np.int64) * 64  # the rest of chunk 0 below `base`
    a0 = np.concatenate([gap, other])
    l0 = np.full(len(a0), 64, np.int64)
    rng = np.random.default_rng(seed)
    p = rng.permutation(len(a0))
    return _descs(np.concatenate([a0[p], addrs]), np.concatenate([l0[p], lens])), base + n_str * 2048 + 4096


def test_plan_2d_rows_past_short_frames_not_contained():
    d, U = two_d_with_gap_frames()
    plans = SP.call_plans(d, U)
    assert plans[0][0] == SP.GATHER and plans[0][1]  # chunk 0: aligned 64-B frames, contained
    assert all(p[0] == SP.TWO_D and not p[1] for p in plans[1:]), plans  # rows reach the gap frames
    # the gap frames lie inside the 2-D rows: the copy writes bytes of another chunk's frames
    assert (d["addr"][:SP.CHUNK_FRAMES] % 2048 == 1360).sum() > 0


def test_plan_wire_64b_pitch():
    """wire mode's read span of a 64-B frame.  Since round 4 every wire kernel reads the reference
    mode's 64-B window (xsk_gpu__read_span), so aligned 64-B frames at a 64-B pitch, interleaved over chunks, copy
    exactly their own bytes: contained in both modes (round 4's 128-B span reached into the next frame)."""
    n = SP.CHUNK_FRAMES + 5000
    addrs = np.arange(n, dtype=np.int64) * 64
    order = np.concatenate([np.arange(c, n, 3) for c in range(3)])
    d = _descs(addrs[order], np.full(n, 64))
    U = n * 64 + 4096
    for wire in (True, False):
        plans = SP.call_plans(d, U, wire=wire)
        assert all(p[1] for p in plans) and sum(p[3] for p in plans) == 64 * n, plans


def test_plan_no_alias_bounded():
    """Without a mapped alias a scattered chunk takes the host pack: the bytes it moves are its spans (plus 4 B of
    offset per frame), never the span [lo, hi) that round 4's fallback copied."""
    rng = np.random.default_rng(4)
    for n in (64, 1024, SP.CHUNK_FRAMES):
        addrs = 256 + rng.permutation(4 * n)[:n].astype(np.int64) * 4096
        d = _descs(addrs, rng.integers(20, 1500, n))
        kind, contained, aligned, total, _ = SP.stage_plan(d, 16 * n * 4096, have_alias=False)
        assert kind == SP.HOSTPACK and contained and aligned
        owned = int((((np.maximum(d["len"].astype(np.int64), 64) + 15) // 16) * 16).sum())
        assert total + 4 * n <= 1.1 * owned
