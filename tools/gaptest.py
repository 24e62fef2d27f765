import os, sys, json, time
sys.path.insert(0, os.getcwd())
import torch
import xsknet_amd as X
dev = torch.device("cuda:0")
n, stride = 1 << 20, 4096
pool = 16
umems = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(pool)]
descs = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(pool)]
for b in range(pool):
    X.synth_dev(umems[b], descs[b], n, 0, stride, 0x5EED0003, b * n, 1, 0, 1500, 1500)
verd = torch.empty(n, dtype=torch.uint8, device=dev)
recs = torch.empty(n * 16, dtype=torch.uint8, device=dev)
stats = torch.zeros(40, dtype=torch.uint8, device=dev)
ws = torch.zeros(X.workspace_size(0, n), dtype=torch.uint8, device=dev)
for rep in range(6):
    for timing in (False, True):
        for b in range(pool):
            X.rearm_dev(umems[b], descs[b], verd, n)
        torch.cuda.synchronize()
        X.timing_enable(timing)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for b in range(pool):
            X.echo_dev(umems[b], descs[b], n, verd, recs, stats, ws)
        e1.record()
        torch.cuda.synchronize()
        km, la = X.timing_read()
        X.timing_enable(False)
        print(json.dumps({"rep": rep, "kernel_timer": timing, "us_per_step": round(e0.elapsed_time(e1) / pool * 1e3, 1),
                          "kernel_avg_us": round(km / la * 1e3, 1) if timing and la else None}), flush=True)
