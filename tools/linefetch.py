#!/usr/bin/env python3
"""Driver for tools/linefetch.hip: cold 4 GiB buffers (a pool larger than the 256 MiB Infinity Cache), each mode
launched once per buffer per pass, HIP-event timed; prints per mode the median launch time and the rate of the
bytes the mode needs (its useful bytes) and of the lines it touches.  Run under `rocprofv3 --pmc FETCH_SIZE`
for the counter side (one pass per counter)."""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liblinefetch.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "linefetch.hip")], check=True)
L = C.CDLL(SO)
L.linefetch_run.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p]


def useful_bytes(mode, nbytes):
    if mode == 0:
        return nbytes
    if mode == 1:
        return nbytes // 2
    if mode == 2:
        return nbytes // 8
    if mode == 7:
        return nbytes
    import numpy as np
    j = np.arange(nbytes // 2048, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = j * np.uint64(0x9E3779B97F4A7C15) + np.uint64(0x5EED0004)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    ln = 64 + (z % np.uint64(1437)).astype(np.int64)
    if mode == 4:
        ln = (ln + 127) // 128 * 128
    if mode in (5, 6, 8):  # whole 16-B blocks of each frame
        ln = (ln + 15) // 16 * 16
    return int(ln.sum())


def main():
    modes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4").split(",")]
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    nbytes = 1 << 31  # 2 GiB = 1 M frames at 2 KiB (c4's slab)
    free, _ = torch.cuda.mem_get_info(dev)
    pool = max(2, min(8, int(free * 0.7) // nbytes))
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev) for _ in range(pool)]
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    res = {}
    for p in range(passes + 1):
        for m in modes:
            for b in bufs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.linefetch_run(m, b.data_ptr(), nbytes, out.data_ptr(), 256 * 4, sp) == 0
                e1.record()
                if p:
                    res.setdefault(m, []).append((e0, e1))
        torch.cuda.synchronize()
    for m, evs in sorted(res.items()):
        ts = sorted(a.elapsed_time(b) for a, b in evs)
        med = ts[len(ts) // 2] / 1e3
        ub = useful_bytes(m, nbytes)
        print(json.dumps({"mode": m, "us_med": round(med * 1e6, 1), "useful_bytes": ub,
                          "useful_gbs": round(ub / med / 1e9, 1), "n": len(ts)}), flush=True)


if __name__ == "__main__":
    main()
