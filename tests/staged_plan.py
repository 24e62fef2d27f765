"""The STAGED host mode's chunking (xsknet_amd/csrc/xsk_gpu_host.c: stage_chunk, stage_chunks_max) and copy-in planner
(xsknet_amd/csrc/xsk_stage_plan.h) restated, for the GPU tests' expected copy-in records and the CPU tests of the
chunk-count bound and of the planner's containment decision."""
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


# ---- the copy-in planner (xsknet_amd/csrc/xsk_stage_plan.h: xsk_gpu__stage_plan) --------------------------------------
LOWLAT_MAX = 1024
NONE, TWO_D, SPAN, GATHER, HOSTPACK = 0, 1, 2, 3, 4


def read_span(addr, length, umem_size, wire=False):
    """xsk_gpu__read_span (xsk_gpu_internal.h): (a16, bytes) the transform reads of one frame."""
    a16 = addr & ~15
    need = length if wire else (max(length, 38) if length >= 20 else length)
    if length > (1 << 30) or addr > umem_size or need > umem_size - addr or length < (14 if wire else 20):
        return a16, 0
    lim = max((addr & 15) + length, min(umem_size - a16, 64))
    return a16, (lim + 15) & ~15


def uniform_stride(addrs):
    n = len(addrs)
    if n < 2 or addrs[1] <= addrs[0]:
        return 0
    s = addrs[1] - addrs[0]
    if s < 64 or s & 15:
        return 0
    return s if all(addrs[i] == addrs[0] + i * s for i in range(n)) else 0


def stage_plan(descs, umem_size, wire=False, have_alias=True, prefix_aligned=True):
    """Returns (kind, contained, aligned, sum, moved): which path copies chunk `descs` into the device mirror (sum: the
    frames' read spans; moved: the frame bytes that path copies -- n x width for the 2-D copy, the span for the span
    copy, the spans otherwise; the host pack adds its offset tables), and whether the
    copy writes only mirror bytes of the chunk's own frames -- [addr, align16(addr + max(len, 64))) of each -- while
    every frame of the call so far (earlier chunks included) starts 16-B aligned, so that no earlier chunk's frame can
    be overwritten while its transform and header pack are in flight."""
    addrs = [int(a) for a in descs["addr"]]
    lens = [int(x) for x in descs["len"]]
    n = len(addrs)
    aligned = all(a & 15 == 0 for a in addrs)
    prefix = prefix_aligned and aligned
    lo, hi, width, total, spans_own = None, 0, 0, 0, True
    min_own = min((((max(ln, 64) + 15) // 16) * 16 for ln in lens), default=0)
    for a, ln in zip(addrs, lens):
        a16, sp = read_span(a, ln, umem_size, wire)
        if not sp:
            continue
        spans_own &= sp <= ((max(ln, 64) + 15) // 16) * 16
        lo = a16 if lo is None else min(lo, a16)
        hi = max(hi, a16 + sp)
        width = max(width, sp)
        total += sp
    if not total:
        return NONE, True, aligned, 0, 0
    budget = total + total // 10
    s = uniform_stride(addrs)
    base = addrs[0] & ~15
    small = n <= LOWLAT_MAX and have_alias
    if not small and s and width <= s and n * width <= budget and base + (n - 1) * s + width <= umem_size:
        return TWO_D, prefix and width <= min_own, aligned, total, n * width
    if not small and hi - lo <= budget:
        return SPAN, False, aligned, total, hi - lo
    return (GATHER if have_alias else HOSTPACK), prefix and spans_own, aligned, total, total


def call_plans(descs, umem_size, wire=False, have_alias=True):
    """The plan of every chunk of one STAGED call, the call-prefix alignment carried from chunk to chunk."""
    out, i0, prefix = [], 0, True
    n = len(descs)
    for m in stage_chunks(n):
        p = stage_plan(descs[i0:i0 + m], umem_size, wire, have_alias, prefix)
        prefix = prefix and p[2]
        out.append(p)
        i0 += m
    return out
