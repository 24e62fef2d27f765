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
