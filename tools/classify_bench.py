#!/usr/bin/env python3
"""Time the device XDP ingress filter (xsk_gpu_classify_dev, inner_xdp.c:26-61) and the filter ->
echo pipeline on a 1 M mixed-traffic batch (GPU box).  Prints one JSON line.

--lib PATH times the xsk_gpu_classify_dev of another build of xsk_classify.hip (same C signature; e.g. round 1's
three-launch filter, `git show <rev>:xsknet_amd/csrc/xsk_classify.hip` built with hipcc -shared -I xsknet_amd/csrc)
against the same batch, for A/B; its workspace is the larger of the two builds'.

Algorithmic bytes per frame of the filter: 16-B descriptor read, the frame bytes the eBPF program
reads (12-13 and 23: one 64-B sector per frame in practice), 1-B action written, 16-B descriptor
written per redirected frame.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import xsknet_amd as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    args = ap.parse_args()
    n, stride, reps = 1 << 20, 2048, 20
    dev = torch.device("cuda:0")
    classify = X.classify_dev
    if args.lib:
        L = C.CDLL(os.path.abspath(args.lib))
        L.xsk_gpu_classify_dev.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_int, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.xsk_gpu_classify_dev.restype = C.c_int
        L.xsk_gpu_classify_workspace_size.argtypes = [C.c_uint32]
        L.xsk_gpu_classify_workspace_size.restype = C.c_size_t

        def classify(umem, descs, n, bound, act, out, nout, ws):
            rc = L.xsk_gpu_classify_dev(umem.data_ptr(), umem.numel(), descs.data_ptr(), n, 1 if bound else 0,
                                        act.data_ptr(), out.data_ptr(), nout.data_ptr(), ws.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
    umem = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    descs = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    X.synth_dev(umem, descs, n, 0, stride, 0x5EED0E0E, 0, 1, 1, 20, 1500)  # mixed traffic
    act = torch.empty(n, dtype=torch.uint8, device=dev)
    red = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    nred = torch.zeros(1, dtype=torch.int64, device=dev)
    wsz = int(X.lib().xsk_gpu_classify_workspace_size(n))
    if args.lib:
        wsz = max(wsz, int(L.xsk_gpu_classify_workspace_size(n)))
    ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
    for _ in range(3):
        classify(umem, descs, n, True, act, red, nred, ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        classify(umem, descs, n, True, act, red, nred, ws)
    e1.record()
    torch.cuda.synchronize()
    t_cls = e0.elapsed_time(e1) / reps / 1e3
    k = int(nred.cpu().view(torch.int32)[0].item())
    # filter -> echo on the redirected frames (echo re-armed between reps, untimed)
    verd = torch.empty(max(k, 1), dtype=torch.uint8, device=dev)
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ews = torch.zeros(X.workspace_size(0, k), dtype=torch.uint8, device=dev)
    t_pipe = 0.0
    for _ in range(reps):
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        classify(umem, descs, n, True, act, red, nred, ws)
        X.echo_dev(umem, red, k, verd, None, stats, ews)
        a1.record()
        X.rearm_dev(umem, red, verd, k)
        torch.cuda.synchronize()
        t_pipe += a0.elapsed_time(a1) / 1e3
    t_pipe /= reps
    algo = n * (16 + 64 + 1) + k * 16
    print(json.dumps({"lib": args.lib or "libxsknet_amd.so", "frames": n, "redirected": k, "classify_us": round(t_cls * 1e6, 2),
                      "classify_mframes_s": round(n / t_cls / 1e6, 1),
                      "classify_gbs_algorithmic": round(algo / t_cls / 1e9, 1),
                      "filter_plus_echo_us": round(t_pipe * 1e6, 2),
                      "filter_plus_echo_mframes_s": round(n / t_pipe / 1e6, 1)}))


if __name__ == "__main__":
    main()
