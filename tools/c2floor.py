#!/usr/bin/env python3
"""Driver for tools/c2floor.hip (GPU box): c2-shaped batches (1 M packed 64-B frames), a pool of sets larger than
the 256 MiB Infinity Cache, each set launched once per pass so every launch is cold.  Prints per mode the median
launch time (HIP events), next to the shipped round kernel on the same sets (re-armed before each pass).

    python tools/c2floor.py [modes=0,1,2,3] [passes=5]
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import xsknet_amd as X  # noqa: E402
from bench import CONFIGS  # noqa: E402

SO = os.path.join(HERE, "libc2floor.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "c2floor.hip")], check=True)
L = C.CDLL(SO)
L.c2floor_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]


def main():
    modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n, lo, hi, stride, seed, _ = CONFIGS["c2"]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    sets = []
    for k in range(8):
        umem = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        descs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        X.synth_dev(umem, descs, n, 0, stride, seed + k, 0, 1, 0, lo, hi)
        sets.append((umem, descs, torch.zeros(n, dtype=torch.uint8, device=dev),
                     torch.zeros(n * 16, dtype=torch.uint8, device=dev)))
    stats = torch.zeros(32, dtype=torch.uint8, device=dev)
    fverd = torch.zeros(n, dtype=torch.uint8, device=dev)
    frecs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    flush = torch.zeros(1 << 30, dtype=torch.uint8, device=dev) if os.environ.get("C2F_FLUSH", "1") == "1" else None
    torch.cuda.synchronize()
    # "b2b": one event pair around the pool's launches (the bench's regime), else events around each launch
    keys = [(m, b2b) for m in modes + ["echo"] for b2b in (False, True)]
    times = {k: [] for k in keys}
    for p in range(passes + 1):
        for (m, b2b) in keys:
            if m == "echo":
                for (umem, descs, verd, recs) in sets:
                    X.rearm_dev(umem, descs, verd, n, stream)
                if flush is not None:
                    flush.add_(1)  # 1 GiB read and written: the re-armed sets leave the Infinity Cache
                torch.cuda.synchronize()
            evs = []
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(stream)
            for (umem, descs, verd, recs) in sets:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if not b2b:
                    e0.record(stream)
                if m == "echo":
                    X.echo_dev(umem, descs, n, verd, recs, stats, ws, stream)
                else:
                    # the floors leave the frames as they were and write their own verdict / record buffers, so that
                    # the echo's re-arm (which restores each frame from its verdict) still sees the echo's outputs
                    rc = L.c2floor_run(m, umem.data_ptr(), descs.data_ptr(), fverd.data_ptr(), frecs.data_ptr(), n, sp)
                    assert rc == 0, rc
                if not b2b:
                    e1.record(stream)
                    evs.append((e0, e1))
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record(stream)
            torch.cuda.synchronize()
            if m == "echo":  # every frame answered: the timing is of the full transform
                assert all(bool((s[2] == 0).all().item()) for s in sets), "echo verdicts"
            if p:
                times[(m, b2b)] += [a.elapsed_time(b) * 1e3 for a, b in evs] if not b2b else \
                    [t0.elapsed_time(t1) * 1e3 / len(sets)]
    for (m, b2b) in keys:
        t = float(np.median(times[(m, b2b)]))
        print(json.dumps({"mode": m, "b2b": b2b, "us": round(t, 2), "launches": len(times[(m, b2b)]),
                          "traffic_tbs": round((n * (64 + 64) + (0 if m == 2 else n * 33)) / (t * 1e-6) / 1e12, 3)}),
              flush=True)
    per_set = [float(np.median(times[("echo", False)][i::len(sets)])) for i in range(len(sets))]
    print(json.dumps({"echo_per_set_us": [round(t, 2) for t in per_set]}), flush=True)


if __name__ == "__main__":
    main()
