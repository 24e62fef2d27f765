#!/usr/bin/env python3
"""Driver for tools/wexp.hip (write-pattern micro-experiment, GPU box).  Cold-batch regime: a pool of
distinct 4 GiB slabs launched back to back, each launch timed with HIP events."""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libwexp.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", SO,
                    os.path.join(HERE, "wexp.hip")], check=True)
L = C.CDLL(SO)
L.wexp_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                       C.c_void_p]


def main():
    n, stride, ln = 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 1500
    modes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3,4,5,6").split(",")]
    grids = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "4096,1536").split(",")]
    dev = torch.device("cuda:0")
    free, _ = torch.cuda.mem_get_info(dev)
    pool = max(1, min(int(os.environ.get("WEXP_POOL", "10")), int(free * 0.8) // (n * stride)))
    bufs = [torch.randint(0, 255, (n * stride,), dtype=torch.uint8, device=dev) for _ in range(pool)]
    out = torch.zeros(8 + 2 * 4096, dtype=torch.int64, device=dev)
    side = torch.zeros(n * 64, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    res = {}
    for rep in range(4):
        for m in modes:
            for g in grids:
                for b in bufs:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    assert L.wexp_run(m, b.data_ptr(), n, stride, ln, out.data_ptr(), g, sp, side.data_ptr()) == 0
                    e1.record()
                    if rep:
                        res.setdefault((m, g), []).append((e0, e1))
                    if rep == 3 and b is bufs[-1] and m in (15, 16, 19, 20, 21, 22) and os.environ.get("WEXP_WG"):
                        torch.cuda.synchronize()
                        t = out[8:8 + 2 * g].cpu().view(g, 2).double() / 100.0  # wall_clock64: 100 MHz -> us
                        t0 = t[:, 0].min()
                        st, en = (t[:, 0] - t0), (t[:, 1] - t0)
                        xcd = [round(float(en[x::8].mean()), 1) for x in range(8)]
                        print(json.dumps({"mode": m, "grid": g, "start_max": round(float(st.max()), 1),
                                          "end_min": round(float(en.min()), 1), "end_med": round(float(en.median()), 1),
                                          "end_max": round(float(en.max()), 1), "end_mean_per_xcd": xcd}), flush=True)
        torch.cuda.synchronize()
    for (m, g), evs in sorted(res.items()):
        ts = sorted(a.elapsed_time(b) for a, b in evs)
        med = ts[len(ts) // 2]
        print(json.dumps({"stride": stride, "mode": m, "grid": g, "us_med": round(med * 1e3, 1),
                          "gbs_frame": round(n * ln / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
