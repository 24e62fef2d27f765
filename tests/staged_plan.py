"""The STAGED host mode's chunking restated (xsknet_amd/csrc/xsk_gpu_host.c: stage_chunk, stage_chunks_max), for the
GPU tests' expected copy-in records and the CPU test of the chunk-count bound."""
CHUNK_FRAMES = 32768
TAIL_FRAMES = 4096


def stage_chunk(n, rem):
    """Frames in the next chunk of an n-frame batch with `rem` frames left."""
    if n <= CHUNK_FRAMES or rem <= TAIL_FRAMES:
        return rem
    if rem >= 2 * CHUNK_FRAMES:
        return CHUNK_FRAMES
    half = ((rem // 2) + 15) & ~15
    return TAIL_FRAMES if half < TAIL_FRAMES else half


def stage_chunks(n):
    """The chunk sizes of an n-frame batch, in order."""
    out, i0 = [], 0
    while i0 < n:
        m = stage_chunk(n, n - i0)
        out.append(m)
        i0 += m
    return out


def stage_chunks_max(n):
    return (n + CHUNK_FRAMES - 1) // CHUNK_FRAMES + 5
