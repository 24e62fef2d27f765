"""N > 1 path on CPU: round-robin sharding and the cross-rank reduction over gloo, world size 2.

Each rank builds its sub-batch with the generator's (first, step) arguments from
``xsknet_amd.shard`` and transforms it (the CPU oracle stands in for the GPU kernel here: this test
is about the sharding and the collectives, the kernel has its own parity tests); the reduced counters
and every rank's frames must equal a single-process run over the whole global batch.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from xsknet_amd import shard

N_PER_RANK, STRIDE, SEED = 512, 2048, 0x5EED0005


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, batches, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = []
        for b in range(batches):
            first, step = shard.shard_range(b, N_PER_RANK, rank, world)
            umem = np.zeros(N_PER_RANK * STRIDE, np.uint8)
            descs = oracle.synth_batch(umem, N_PER_RANK, 0, STRIDE, SEED, first=first, step=step, mode=1,
                                       len_lo=20, len_hi=1500)
            v, _, st = oracle.echo_batch(umem, descs)
            counters = {k: int(st[k]) for k in shard.COUNTERS}
            wall, tot = shard.reduce_run(float(rank + 1), counters, world)
            res.append((b, wall, tot, umem[:64 * STRIDE].tobytes(), v[:64].tobytes()))
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_every_frame_once():
    for world in (1, 2, 4, 8):
        for b in range(3):
            seen = sorted(g for r in range(world) for g in shard.global_indices(b, 100, r, world))
            assert seen == list(range(b * 100 * world, (b + 1) * 100 * world))
    with pytest.raises(ValueError):
        shard.shard_range(0, 10, 2, 2)


def test_reduce_run_identity_world1():
    c = {"rx_packets": 3, "rx_bytes": 4, "tx_packets": 5, "tx_bytes": 6}
    assert shard.reduce_run(1.5, c, 1) == (1.5, c)


def test_gloo_world2_matches_single_process():
    world, batches = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batches, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for b in range(batches):
        # single process over the whole global batch
        n = N_PER_RANK * world
        umem = np.zeros(n * STRIDE, np.uint8)
        descs = oracle.synth_batch(umem, n, 0, STRIDE, SEED, first=b * n, step=1, mode=1, len_lo=20,
                                   len_hi=1500)
        v, _, st = oracle.echo_batch(umem, descs)
        ref = {k: int(st[k]) for k in shard.COUNTERS}
        for r in range(world):
            bb, wall, tot, frames, verd = got[r][b]
            assert bb == b and wall == float(world)  # max over ranks of (rank + 1)
            assert tot == ref
            # rank r's local frame j is global frame r + j*world
            for j in range(64):
                g = r + j * world
                assert frames[j * STRIDE:(j + 1) * STRIDE] == umem[g * STRIDE:(g + 1) * STRIDE].tobytes()
                assert verd[j] == v[g]
