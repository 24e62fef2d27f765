#!/usr/bin/env python3
"""Per-call latency of the host-UMEM drop-in (xsk_gpu_process) at RX-loop batch sizes: the C1 shape
(4096 x 64-B frames in a 16 MiB UMEM of 4 KiB chunks, 256-B headroom) processed in batches of
64 (RX_BATCH_SIZE, xsk_utils.h:8) up to 4096 frames, zerocopy and staged.  Prints one JSON line per
(mode, batch): microseconds per call and Mframes/s.  Frames are re-armed (untimed) between passes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle  # noqa: E402  (frame generator + re-arm only)
import xsknet_amd as X  # noqa: E402


def main():
    n, chunk = 4096, 4096
    for flen in (64, 1500):
        umem = np.zeros(n * chunk, np.uint8)
        descs = oracle.synth_batch(umem, n, 256, chunk, seed=0x5EED0001, mode=0, len_lo=flen, len_hi=flen)
        for name, mode in (("zerocopy", X.MODE_ZEROCOPY), ("staged", X.MODE_STAGED)):
            for batch in (64, 256, 1024, 4096):
                with X.EchoContext(umem, 0, max_batch=batch, mode=mode) as ctx:
                    for i in range(0, n, batch):  # warm
                        ctx.process(descs[i:i + batch], want_recs=False)
                    oracle.rearm(umem, descs, np.zeros(n, np.uint8))
                    calls, t = 0, 0.0
                    while t < 1.0:
                        t0 = time.perf_counter()
                        for i in range(0, n, batch):
                            ctx.process(descs[i:i + batch], want_recs=False)
                        t += time.perf_counter() - t0
                        calls += n // batch
                        oracle.rearm(umem, descs, np.zeros(n, np.uint8))
                print(json.dumps({"frame_len": flen, "mode": name, "batch": batch, "us_per_call": round(t / calls * 1e6, 1),
                                  "mframes_s": round(calls * batch / t / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
