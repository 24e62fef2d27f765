"""Multi-GPU sharding of an echo batch: frames are independent
(``/root/reference/src/lib/xsk_receive.c:113-190`` reads only its own frame), so a step's global batch
of ``n_per_rank * world`` frames is split round-robin — global frame ``g`` goes to rank ``g % world``
— and every rank transforms its own sub-batch with no data-path collective.  The only cross-rank
steps are the max of the per-rank wall times and the sum of the ``stats_record`` counters
(``xsk_utils.h:17-23``), done with ``torch.distributed`` (RCCL on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

COUNTERS = ("rx_packets", "rx_bytes", "tx_packets", "tx_bytes")


def shard_range(batch: int, n_per_rank: int, rank: int, world: int) -> Tuple[int, int]:
    """(first, step) of the global frame indices rank ``rank`` owns in batch ``batch``: local frame j is
    global frame ``first + j * step`` (the generator's round-robin arguments)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return batch * n_per_rank * world + rank, world


def global_indices(batch: int, n_per_rank: int, rank: int, world: int) -> range:
    first, step = shard_range(batch, n_per_rank, rank, world)
    return range(first, first + n_per_rank * step, step)


def reduce_run(wall_s: float, counters: Dict[str, int], world: int, device=None):
    """Max of the wall times and sum of the counters over ranks (identity at world == 1)."""
    if world == 1:
        return wall_s, dict(counters)
    import torch
    import torch.distributed as dist
    t = torch.tensor([wall_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([int(counters[k]) for k in COUNTERS], dtype=torch.int64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), {k: int(v) for k, v in zip(COUNTERS, c.tolist())}


def sum_counters(parts: Sequence[Dict[str, int]]) -> Dict[str, int]:
    return {k: sum(int(p[k]) for p in parts) for k in COUNTERS}
