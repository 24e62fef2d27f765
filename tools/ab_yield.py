"""A/B of the LOWLAT leader's yield word (round 6) on the RX loop: the product library built with
XSK_LL_YIELD = 0 (the round-5 poll: an 8-B load of the command word, no yield) and 1 (shipped: one 16-B load of the
command word and the yield word), each driving tools/rxring (64-frame steps plain and pipelined at depth 4, 1024-frame steps;
LOWLAT, 64-B frames, burst NIC, huge pages, every reply checked) in turn, round after round, on one box.

    python tools/ab_yield.py --build          # here: tools/ab_yield/v{0,1}/libxsknet_amd.so
    python tools/ab_yield.py [--rounds 3]     # on the GPU box: one JSON line per run, then a summary
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "xsknet_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "ab_yield")
POLICIES = (0, 1)
RUNS = (("step64", ["64"], [], {}), ("step64_pipe4", ["64"], ["pipe=4"], {}), ("step1024", ["1024"], [], {}),
        ("step64_pipe8_hwq8", ["64"], ["pipe=8"], {"GPU_MAX_HW_QUEUES": "8"}))


def build():
    objs = [os.path.join(CSRC, f) for f in ("xsk_echo.o", "xsk_aux.o", "xsk_classify.o", "xsk_gpu_host.o",
                                             "xsk_gpu_mem.o", "xsk_gpu_rx.o", "xsk_gpu_multi.o", "xsk_gpu_pipe.o",
                                             "xsk_gpu_umem.o")]
    subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True, stdout=subprocess.DEVNULL)
    for pol in POLICIES:
        d = os.path.join(OUT, f"v{pol}")
        os.makedirs(d, exist_ok=True)
        o = os.path.join(d, "xsk_lowlat.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wall",
                        f"-DXSK_LL_YIELD={pol}", "-c", "-o", o, os.path.join(CSRC, "xsk_lowlat.hip")],
                       check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(d, "libxsknet_amd.so")] + objs + [o, "-pthread",
                                                                      "-Wl,-soname,libxsknet_amd.so"], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--runs", default="step64,step64_pipe4,step1024,step64_pipe8_hwq8")
    args = ap.parse_args()
    if args.build:
        build()
        return 0
    exe = os.path.join(ROOT, "tools", "rxring")
    res = {}
    for rnd in range(args.rounds):
        for pol in POLICIES:
            for name, step, extra, xenv in [r for r in RUNS if r[0] in args.runs.split(",")]:
                env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(OUT, f"v{pol}"), **xenv)
                cmd = [exe] + step + ["lowlat", str(args.seconds), "len=64", "huge=1", "ring=16384", "frames=16384",
                                      "nic=burst"] + extra
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
                d = json.loads(r.stdout.strip().splitlines()[-1])
                q = d["per_queue"][0]
                line = {"round": rnd, "policy": pol, "run": name, "mframes_s": q["mframes_s"],
                        "us_per_step": q["us_per_step"], "p50_us": q["p50_us"], "failures": d["failures"],
                        "mode": q["mode"]}
                res.setdefault((name, pol), []).append((q["mframes_s"], q["p50_us"]))
                print(json.dumps(line), flush=True)
    summary = {f"{n} policy {p}": {"median_mframes_s": sorted(x[0] for x in v)[len(v) // 2],
                                   "median_p50_us": sorted(x[1] for x in v)[len(v) // 2],
                                   "all_mframes_s": [x[0] for x in v]} for (n, p), v in res.items()}
    print(json.dumps({"tool": "ab_yield", "summary": summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
