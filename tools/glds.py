#!/usr/bin/env python3
"""Driver for tools/glds.hip (register loads vs LDS-DMA read ceiling, GPU box)."""
import ctypes as C
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libglds.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "glds.hip")], check=True)
L = C.CDLL(SO)
L.glds_run.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                       C.c_void_p]

NAMES = {0: "reg U4", 1: "reg U8", 2: "glds U4 nt", 3: "glds U8 nt", 4: "glds U4 default", 5: "glds U8 default",
         6: "glds U16 nt", 7: "per-WG contiguous reg U4", 8: "per-WG contiguous reg U8", 9: "per-WG contiguous reg U2"}
KINDS = [int(k) for k in os.environ.get("GLDS_KINDS", ",".join(map(str, NAMES))).split(",")]
GRIDS = {k: ((256,) if k >= 7 else (1024, 2048)) for k in NAMES}


def main():
    dev = torch.device("cuda:0")
    n, stride, ln = 1 << 20, 4096, 1500
    slabs = [torch.randint(0, 255, (n * stride,), dtype=torch.uint8, device=dev) for _ in range(2)]
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    rows = (ln + 255) // 256
    cases = [("contig_1.5GB", 0, n * ln // 1024), ("c3_rows_s4096", 1, n // 4 * rows),
             ("c3_framemajor_s4096", 2, n * 2), ("c3_rows128_s4096", 3, n // 8 * ((ln + 127) // 128)),
             ("c4like_rows_s2048", 4, n // 4 * rows)]
    only = os.environ.get("GLDS_CASES")
    if only:
        cases = [c for c in cases if c[0] in only.split(",")]
    res = {}
    for rep in range(8):
        for cname, layout, npieces in cases:
            for kind in KINDS:
                for grid in GRIDS[kind]:
                    for s in slabs:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        st = 2048 if layout == 4 else stride
                        assert L.glds_run(kind, s.data_ptr(), npieces, layout, ln, st, grid, out.data_ptr(), sp) == 0
                        e1.record()
                        if rep:
                            res.setdefault((cname, kind, grid), []).append((e0, e1))
        torch.cuda.synchronize()
    for (cname, kind, grid), evs in res.items():
        ts = sorted(a.elapsed_time(b) for a, b in evs)
        med = ts[len(ts) // 2] * 1e3
        fb = 820_000_000 if cname.startswith("c4like") else n * ln  # c4-like: ~782 B mean
        print(json.dumps({"case": cname, "kind": NAMES[kind], "grid": grid, "us_med": round(med, 1),
                          "us_min": round(ts[0] * 1e3, 1), "tbs_frame_bytes": round(fb / med / 1e6, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
