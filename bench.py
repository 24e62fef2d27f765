#!/usr/bin/env python3
"""Bench of the MI355X ICMP-echo frame transform (BASELINE.json metric).

One step = one pass of the transform (xsk_gpu_echo_dev: parse + full-payload checksums + echo-reply
rewrite + records + stats counters) over one batch of frames already resident in HBM.  Each step
gets a fresh, never-transformed batch (a pool of pre-generated batches), so no step sees replies.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5|p98] [--no-cpu] [--host-inclusive]

Multi-GPU: one process per GPU.  Run as `python bench.py --gpus N` (no launcher) the script starts
`torch.distributed.run --nproc-per-node N` itself as a child process before anything touches a GPU, and
exits with its status; under an external torch.distributed.run it is one of the ranks and checks that
WORLD_SIZE == N.  Frame i of a step's global batch goes to GPU i mod N (round-robin sharding, no
data-path collective): c2/c3/c4/p98 keep the per-GPU work fixed (weak scaling), c5 splits a fixed 64 M
frames per step over the N GPUs (strong scaling).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Mframes/s + GiB/s device-resident, 1500B ICMP echo batch, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# the transform kernel xsk_gpu_echo_dev launches for a large batch (the name rocprofv3 reports)
KERNEL = "echo_round_kernel<false, false, 6, true, true, 2, true>"
# xsk_gpu_echo_dev_opts, nonzero --opts
WIRE_KERNEL = "echo_round_kernel<true, false, 6, true, true, 2, true>"
CONFIGS = {
    # name: (frames per GPU, len_lo, len_hi, stride, seed, description)
    "c2": (1 << 20, 64, 64, 64, 0x5EED0002, "c2: 1M x 64B minimum-size ICMP echo frames, packed 64-B stride"),
    "c3": (1 << 20, 1500, 1500, 4096, 0x5EED0003,
           "c3: 1M x 1500B ICMP echo frames, 4 KiB UMEM-chunk stride, full-payload checksum"),
    "c4": (1 << 20, 64, 1500, 2048, 0x5EED0004, "c4: 1M x U{64..1500}B ICMP echo frames, 2 KiB stride"),
    # not a BASELINE config: the frame a default `ping` sends (56-B payload), for the RX-loop case
    "p98": (1 << 20, 98, 98, 2048, 0x5EED0098, "p98: 1M x 98B default-ping ICMP echo frames, 2 KiB stride"),
    # C5 is a STRONG-scaling config: 64 M frames in total per step, frame i on GPU i mod N
    "c5": (1 << 26, 1500, 1500, 2048, 0x5EED0005,
           "c5: 64M x 1500B ICMP echo frames per step in total, round-robin over the GPUs, 2 KiB stride"),
}
STRONG = {"c5"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# Rehearsal of the N > 1 path on a one-GPU box (never used by the driver): every rank on cuda:0 and a
# gloo process group (RCCL refuses two ranks on one device).
SHARE_GPU = os.environ.get("XSK_BENCH_SHARE_GPU") == "1"


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpu_count(nodes=KFD_NODES, env=None):
    """GPUs this process would see, counted WITHOUT any GPU library (the launcher parent must not touch the
    GPU: it spawns the ranks that do).  GPU agents are the KFD topology nodes whose `gpu_id` is nonzero (CPU
    nodes have 0); HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES narrow them as the HIP
    runtime does (comma lists; an empty list hides every GPU).  Returns None when the topology cannot be
    read (not a ROCm host, or sysfs hidden), so the caller can leave the decision to the ranks."""
    env = os.environ if env is None else env
    try:
        names = os.listdir(nodes)
    except OSError:
        return None
    n = 0
    for name in names:
        try:
            gid = int(open(os.path.join(nodes, name, "gpu_id")).read().strip() or "0")
        except (OSError, ValueError):
            continue
        n += 1 if gid != 0 else 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None:
            continue
        ids = [x.strip() for x in v.split(",") if x.strip()]
        # numeric ids past the last GPU select nothing (HIP stops at the first invalid one)
        ok = 0
        for x in ids:
            if x.isdigit() and int(x) >= n:
                break
            ok += 1
        n = min(n, ok)
    return n


def launch_ranks(gpus):
    """Start `torch.distributed.run` with one rank per GPU as a child process (this process has not
    touched a GPU and never will) and return its exit status; rank 0's JSON line reaches our stdout."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[launcher] {gpus} ranks: {' '.join(cmd[1:5])} ...")
    return subprocess.run(cmd).returncode


def dist_setup(gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if SHARE_GPU else int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: run `python bench.py --gpus {gpus}` "
                         f"(it starts its own ranks) or launch {gpus} ranks")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if SHARE_GPU:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:  # "nccl" is RCCL on ROCm; it only carries the barrier and the timing/counter reductions
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    return rank, world, local


def allreduce(vals, op, world, dev):
    if world == 1:
        return vals
    import torch.distributed as dist
    t = torch.tensor(vals, dtype=torch.float64, device="cpu" if SHARE_GPU else dev)
    dist.all_reduce(t, op=op)
    return t.tolist()


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def cpu_share():
    """CPUs this process may use: the affinity mask, bounded by the cgroup CPU quota (on the GPU box the
    machine's nproc is many times the box's share), and never above 16 (the pool's worker-pool rule)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    share = min(n, quota) if quota else n
    return max(1, min(16, share)), n, quota


def _read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def cpu_baseline(cfg, budget_s=8.0):
    """The oracle's C restatement timed on this host's cores on a bounded sample of the same workload:
    full contract (gates, rewrite, RFC 1071 full-payload sums, records, counters) and the reference-
    equivalent header-only transform (process_packet without logging / sendto), each at 1 thread and
    at the box's CPU share, plus BASELINE config 1 (4096 x 64 B, one UMEM) replayed in-process."""
    import oracle
    n_total, lo, hi, stride, seed, _ = CONFIGS[cfg]
    share, affinity, quota = cpu_share()
    n = min(n_total, 1 << 17)  # 131072 frames
    umem = np.zeros(n * stride, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed, mode=0, len_lo=lo, len_hi=hi, threads=share)
    nbytes = int(descs["len"].sum())

    def run(fn, budget, um=umem, ds=descs):
        done, t_tot = 0, 0.0
        while t_tot < budget:
            t0 = time.perf_counter()
            v = fn(um, ds)
            t_tot += time.perf_counter() - t0
            done += len(ds)
            oracle.rearm(um, ds, v)  # untimed: restore requests for the next pass
        return done / t_tot / 1e6

    def full(threads):
        return lambda um, ds: oracle.echo_batch(um, ds, threads=threads)[0]

    def hdr(threads):
        def f(um, ds):
            verd = np.zeros(len(ds), np.uint8)
            st = np.zeros(1, oracle.STATS_DTYPE)
            oracle.lib().oracle_echo_batch_hdr_mt(um.ctypes.data, ds.ctypes.data, len(ds), verd.ctypes.data,
                                                  st.ctypes.data, threads)
            return verd
        return f

    full_n = run(full(share), budget_s)
    full_1 = run(full(1), budget_s / 2)
    hdr_n = run(hdr(share), budget_s / 4)
    hdr_1 = run(hdr(1), budget_s / 4)
    # BASELINE config 1: 4096 x 64 B in one 16 MiB UMEM of 4 KiB chunks (256-B headroom), in-process
    c1_umem = np.zeros(4096 * 4096, np.uint8)
    c1_descs = oracle.synth_batch(c1_umem, 4096, 256, 4096, 0x5EED0001, mode=0, len_lo=64, len_hi=64)
    c1_hdr = run(hdr(1), budget_s / 4, c1_umem, c1_descs)
    c1_full = run(full(1), budget_s / 4, c1_umem, c1_descs)
    gib = nbytes / n / 2**30
    return {
        "value": round(full_n, 3), "unit": "Mframes/s", "cores": share, "kind": "port",
        "gib_per_s": round(full_n * 1e6 * gib, 3),
        "sample": f"{n} frames of {cfg} ({lo}-{hi} B, stride {stride}), full contract (gates, rewrite, RFC 1071 "
                  f"full-payload sums, records, counters) of oracle/echo_oracle.c, {share} pthreads over contiguous "
                  f"frame ranges",
        "full_contract_1core": round(full_1, 3),
        "reference_equivalent": {"cores": share, "value": round(hdr_n, 3), "value_1core": round(hdr_1, 3),
                                 "unit": "Mframes/s",
                                 "sample": "header-only transform exactly as process_packet (no logging, no sendto, "
                                           "no payload sums)"},
        "c1_in_process": {"workload": "BASELINE configs[0]: 4096 x 64 B ICMP echo requests, one per 4 KiB chunk of a "
                                      "16 MiB UMEM (256-B headroom), replayed in-process (no veth / XDP / sendto)",
                          "reference_equivalent_1core": round(c1_hdr, 3), "full_contract_1core": round(c1_full, 3),
                          "unit": "Mframes/s"},
        "host": {"cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": affinity,
                 "cgroup_cpu_quota": quota, "smt_active": _read("/sys/devices/system/cpu/smt/active"),
                 "threads_used": share,
                 "note": "threads = this box's CPU share (affinity / cgroup quota, at most 16: the GPU pool's "
                         "worker rule), not the machine's nproc"},
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def traffic_from_profiles(cfg, kernel, build_id, path=None):
    """PMC-derived HBM bytes per launch from the committed rocprofv3 --pmc summary of this config
    (tools/pmc_summary.py: separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled on gfx950).
    Returns (bytes or None, source): the summary counts only when it names exactly the kernel that ran
    (full demangled template string) AND the build id of the running library (xsk_gpu_build_id(): a hash
    of the kernel sources and flags), so a stale summary is never attached to a different kernel."""
    p = path or os.path.join(ROOT, "profiles", f"traffic_{cfg}.json")
    rel = os.path.relpath(p, ROOT)
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None, f"none: no summary at {rel}"
    if d.get("kernel") != kernel:
        return None, f"none: {rel} profiles kernel {d.get('kernel')!r}, not the one that ran"
    if not build_id or d.get("build_id") != build_id:
        return None, f"none: {rel} is of build {d.get('build_id')!r}, the running library is {build_id!r}"
    b = d.get("hbm_bytes_per_launch")
    return (int(b), f"{rel} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this build)") if b else \
        (None, f"none: {rel} has no byte count")


def host_inclusive(cfg, dev_index):
    """Rate including PCIe: host UMEM -> staged H2D copy -> kernel -> header write-back -> host."""
    import oracle
    import xsknet_amd as X
    n_total, lo, hi, stride, seed, _ = CONFIGS[cfg]
    n = min(n_total, 1 << 18)
    umem = np.zeros(n * stride, np.uint8)
    descs = oracle.synth_batch(umem, n, 0, stride, seed, mode=0, len_lo=lo, len_hi=hi)
    out = {}
    ndev = torch.cuda.device_count()
    runs = [("staged", X.MODE_STAGED, None), ("zerocopy", X.MODE_ZEROCOPY, None)]
    for g in (1, 2):  # xsk_gpu_multi over G contexts: distinct GPUs when there are, else G on this one
        devs = list(range(dev_index, dev_index + g)) if dev_index + g <= ndev else [dev_index] * g
        runs.append((f"staged_multi_g{g}", X.MODE_STAGED, devs))
    for name, mode, devs in runs:
        work = X.umem_copy(umem)  # page-aligned, as xsk_gpu_init requires
        mk = (lambda: X.EchoContext(work, dev_index, max_batch=n, mode=mode)) if devs is None else \
            (lambda: X.MultiContext(work, devs, max_batch=n, mode=mode))
        with mk() as ctx:
            ctx.process(descs, want_recs=False)  # warm
            v = None
            reps, t = 0, 0.0
            while t < 3.0:
                oracle.rearm(work, descs, np.zeros(n, np.uint8) if v is None else v)
                t0 = time.perf_counter()
                v, _, _ = ctx.process(descs, want_recs=False)
                t += time.perf_counter() - t0
                reps += 1
        out[name] = {"mframes_per_s": round(reps * n / t / 1e6, 3),
                     "gib_per_s": round(reps * int(descs["len"].sum()) / t / 2**30, 3), "frames_per_call": n}
        if devs is not None:
            out[name]["devices"] = devs
    return out


def rx_loop(seconds=2.0):
    """The AF_XDP RX loop per queue, measured by tools/rxring in a child process: one LOWLAT queue
    against a simulated kernel side whose RX ring holds every frame of a burst (nic=burst: the application + GPU
    alone), 64-B requests on a huge-page UMEM, every reply checked.  The reference's 64-frame step plain and pipelined
    (xsk_gpu_rx_pipe_*, depth 4), 1024-frame steps, and the depth-8 pipe of a process started with
    GPU_MAX_HW_QUEUES=8 (eight resident kernels: the deployment setting include/xsk_gpu.h names)."""
    exe = os.path.join(ROOT, "tools", "rxring")
    if not os.path.exists(exe):
        return {"skipped": "tools/rxring not built (make)"}
    out = {"tool": "tools/rxring", "timing": "burst", "frame_len": 64, "umem": "xsk_gpu_umem_alloc (huge pages)"}
    for name, step, extra, env in (("step64", 64, [], {}), ("step64_pipe4", 64, ["pipe=4"], {}),
                                   ("step1024", 1024, [], {}),
                                   ("step64_pipe8_hwq8", 64, ["pipe=8"], {"GPU_MAX_HW_QUEUES": "8"})):
        cmd = [exe, str(step), "lowlat", str(seconds), "len=64", "huge=1", "ring=16384", "frames=16384",
               "nic=burst"] + extra
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=60 + 4 * seconds,
                               env=dict(os.environ, **env))
            d = json.loads(r.stdout.strip().splitlines()[-1])
            q = d["per_queue"][0]
            out[name] = {"mframes_per_s": q["mframes_s"], "us_per_step": q["us_per_step"], "p50_us": q["p50_us"],
                         "p99_us": q["p99_us"], "frames": d["frames"], "checked": d["checked"],
                         "failures": d["failures"], "tx_full": d.get("tx_full"), "mode": q["mode"]}
            if env:
                out[name]["env"] = env
        except Exception as e:  # a measurement leg: report, never fail the bench line
            out[name] = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    return out


def multi_devices(world, share_gpu=False):
    """The GPUs of the multi-GPU host-inclusive leg: one context per rank's GPU (LOCAL_RANK r = cuda:r), or every
    context on cuda:0 in the one-GPU rehearsal."""
    return [0] * world if share_gpu else list(range(world))


def host_inclusive_multi(cfg, world, budget_s=2.0, n=1 << 18):
    """The PCIe-inclusive rate of ONE host UMEM served by all of this node's ranks' GPUs (N > 1 runs: the driver's
    scaling curve), measured by rank 0 after the timed region and every collective: xsk_gpu_multi_* in STAGED mode,
    descriptor i of a call on GPU i mod G, each GPU copying its share's frames in over its own PCIe link and only the
    rewritten header bytes back, one host thread per GPU (the reference's one UMEM,
    xsk_utils.c:132-135).  G = 1 on the same UMEM beside it.  Never the bench value; any failure is recorded, not
    raised."""
    import oracle
    import xsknet_amd as X
    _, lo, hi, stride, seed, _ = CONFIGS[cfg]
    devs = multi_devices(world, SHARE_GPU)
    out = {"frames_per_call": n, "frame_len": [lo, hi], "stride": stride, "mode": "staged", "devices": devs,
           "note": "one host UMEM, xsk_gpu_multi_process over G GPUs (descriptor i on GPU i mod G), measured by rank "
                   "0 after the timed region; PCIe-inclusive, never the bench value"
                   + ("; rehearsal: every context on cuda:0" if SHARE_GPU else "")}
    try:
        umem = np.zeros(n * stride, np.uint8)
        descs = oracle.synth_batch(umem, n, 0, stride, seed, mode=0, len_lo=lo, len_hi=hi, threads=cpu_share()[0])
        nbytes = int(descs["len"].sum())
        for g in sorted({1, len(devs)}):
            work = X.umem_copy(umem)  # page-aligned, as xsk_gpu_init requires
            with X.MultiContext(work, devs[:g], max_batch=n, mode=X.MODE_STAGED) as ctx:
                v, _, _ = ctx.process(descs, want_recs=False)  # warm
                ok = bool((v == X.TX_REPLY).all())
                reps, t = 0, 0.0
                while t < budget_s:
                    oracle.rearm(work, descs, v)  # untimed: the frames are requests again
                    t0 = time.perf_counter()
                    v, _, st = ctx.process(descs, want_recs=False)
                    t += time.perf_counter() - t0
                    reps += 1
                    ok = ok and bool((v == X.TX_REPLY).all()) and int(st["tx_packets"]) == n
                # every context's copy-in record (xsk_gpu__staged_stats): bytes moved host -> device and the path
                # each chunk took -- a context without a device alias of the UMEM shows up as host-pack chunks
                staged = ctx.staged_stats()
            out[f"g{g}"] = {"gpus": g, "mframes_per_s": round(reps * n / t / 1e6, 3),
                            "gib_per_s": round(reps * nbytes / t / 2**30, 3), "calls": reps, "verified": ok,
                            "staged_stats": staged,
                            "h2d_per_frame_byte": round(sum(x["h2d_bytes"] for x in staged) / ((reps + 1) * nbytes), 4)}
    except Exception as e:  # noqa: BLE001 -- context only: the bench line must not depend on it
        out["error"] = f"{type(e).__name__}: {e}"
    return out


def reduce_ranks(rank, world, local, *, wall, ev_ms, ok, frames, frame_bytes, kern_avg_ms, launch_bytes, reduce):
    """The cross-rank step of the bench: max of the timed region (wall clock, events), sums of the frames, bytes
    and verification flags, and every rank's own figures gathered into rank 0's line (slot r of a zeroed vector,
    summed).  `reduce(vals, op)` all-reduces a list of floats ("max" / "sum"); the only collectives in the bench
    (no data-path collective: frames are independent, xsk_receive.c:113-190)."""
    import torch.distributed as _d  # noqa
    op_max = _d.ReduceOp.MAX if world > 1 else None
    op_sum = _d.ReduceOp.SUM if world > 1 else None
    wall_max, ev_max = reduce([float(wall), float(ev_ms)], op_max)
    ok_all, frames_all, bytes_all = reduce([1.0 if ok else 0.0, float(frames), float(frame_bytes)], op_sum)
    achieved = launch_bytes / (kern_avg_ms / 1e3) / 1e9 if kern_avg_ms > 0 else 0.0
    mine = [0.0] * (5 * world)
    mine[5 * rank:5 * rank + 5] = [kern_avg_ms * 1e3, achieved, float(wall), float(frames), float(local)]
    flat = reduce(mine, op_sum)
    per_rank = [{"rank": r, "device": int(flat[5 * r + 4]), "kernel_avg_us": round(flat[5 * r], 2),
                 "achieved_gbs": round(flat[5 * r + 1], 1), "frac": round(flat[5 * r + 1] / HBM_PEAK_GBS, 4),
                 "wall_ms": round(flat[5 * r + 2] * 1e3, 3), "frames": int(flat[5 * r + 3])} for r in range(world)]
    return {"wall_max": wall_max, "ev_max": ev_max, "ok_ranks": ok_all, "frames": frames_all, "bytes": bytes_all,
            "per_rank": per_rank}


def frac_of_ceiling(achieved, read_ceiling):
    """roofline.frac_of_read_ceiling: the kernel's algorithmic GB/s over the measured plain-read ceiling of the same
    slab (None when the ceiling was not measured)."""
    return round(achieved / read_ceiling, 4) if read_ceiling and read_ceiling > 0 else None


def pool_plan(n, stride, free, warmup, steps, cap=0):
    """Batches in the pool (each: n frames at `stride` + n descriptors) and whether a step must re-arm its
    batch inside the timed loop: one fresh batch per step while W + K batches fit in 85 % of the free HBM
    (less one batch of headroom for the outputs), else the largest pool that does, re-armed from its own
    verdicts when reused.  c5 per rank: 64 M / N frames at 2 KiB = 128 GiB / N per batch."""
    per_batch = n * stride + n * 16
    pool = max(1, min(warmup + steps, int(free * 0.85) // per_batch - 1))
    if cap:
        pool = min(pool, cap)
    return pool, pool < warmup + steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--host-inclusive", action="store_true", help="also measure the PCIe-inclusive rate")
    ap.add_argument("--no-rx-loop", action="store_true", help="skip the RX-loop leg (tools/rxring, N = 1 only)")
    ap.add_argument("--no-host-multi", action="store_true",
                    help="N > 1: skip rank 0's multi-GPU host-inclusive leg after the timed region")
    ap.add_argument("--pool-cap", type=int, default=0, help="cap the batch pool (rehearsals on a shared GPU)")
    ap.add_argument("--alloc", default="slab", choices=("slab", "separate"),
                    help="batch pool as one device allocation (slab, like one UMEM region) or one per batch")
    ap.add_argument("--variant", type=int, default=-1,
                    help="A/B only: time the product kernel at tuning switch N (tune/xsk_tune_product.hip, "
                         "xsk_gpu__product_variant) instead of the shipped entry point; the line is marked and is never "
                         "the bench value")
    ap.add_argument("--opts", type=int, default=0,
                    help="wire-format options (XSK_GPU_OPT_*, xsk_gpu_echo_dev_opts); 0 = the reference's gates")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the parent never touches a GPU library: it counts GPUs in the KFD topology and spawns the ranks
        ngpu = None if SHARE_GPU else kfd_gpu_count()
        if ngpu is not None and ngpu < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but {ngpu} GPU(s) visible "
                             "(XSK_BENCH_SHARE_GPU=1 rehearses N ranks on one GPU)")
        sys.exit(launch_ranks(args.gpus))

    import xsknet_amd as X
    from xsknet_amd import shard
    X.lib()  # fail loudly if the HIP library is missing

    rank, world, local = dist_setup(args.gpus)
    dev = torch.device("cuda", local)
    n, lo, hi, stride, seed, desc = CONFIGS[args.config]
    if args.config in STRONG:  # fixed total work split over the ranks
        if n % world:
            raise SystemExit(f"{args.config}: {n} frames do not split over {world} ranks")
        n //= world
    kernel = KERNEL if args.opts == 0 else WIRE_KERNEL
    if args.opts:
        desc += f"; wire-format options {args.opts:#x} (xsk_gpu_echo_dev_opts)"
    K, W = args.steps, args.warmup

    # ---- batch pool: one fresh batch per step (generated on the GPU, bit-identical to the oracle) ----
    batch_bytes = n * stride
    free, _ = torch.cuda.mem_get_info(dev)
    pool, rearm_in_loop = pool_plan(n, stride, free, W, K, args.pool_cap)
    log(f"[rank {rank}] {desc}; world {world}; pool {pool} batches of {batch_bytes / 2**30:.2f} GiB"
        + (" (re-arm inside timed loop)" if rearm_in_loop else ""))
    umems, descss = [], []
    t0 = time.perf_counter()
    # one allocation for the whole pool (the UMEM is one region in an AF_XDP client); separately
    # allocated 4 GiB batches land on increasingly fragmented physical memory and read up to 10 %
    # slower late in the pool
    slab = torch.empty(pool * batch_bytes, dtype=torch.uint8, device=dev) if args.alloc == "slab" else None
    for b in range(pool):
        u = slab[b * batch_bytes:(b + 1) * batch_bytes] if slab is not None else \
            torch.empty(batch_bytes, dtype=torch.uint8, device=dev)
        d = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        # round-robin shard: local frame j of batch b is global frame first + j*step
        first, gstep = shard.shard_range(b, n, rank, world)
        X.synth_dev(u, d, n, 0, stride, seed, first, gstep, 0, lo, hi)
        umems.append(u)
        descss.append(d)
    torch.cuda.synchronize()
    log(f"[rank {rank}] generated {pool} batches in {time.perf_counter() - t0:.1f} s")
    frame_bytes = int(descss[0].view(torch.int32).view(-1, 4)[:, 2].to(torch.int64).sum().item())

    # outputs: one verdict and one record buffer per step, so that every step's outputs are checked after the timed
    # region; when batches are re-armed inside the loop (c5: the pool is smaller than W + K), one verdict
    # buffer per pooled batch instead -- a re-arm restores batch b from ITS verdicts of its previous use -- and the
    # records of the last use of each
    per_step = not rearm_in_loop
    verds = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(W + K if per_step else pool)]
    recss = [torch.empty(n * 16, dtype=torch.uint8, device=dev) for _ in range(W + K if per_step else 1)]
    stats = torch.zeros(40, dtype=torch.uint8, device=dev)
    ws = torch.zeros(max(16, X.workspace_size(local, n)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    tune = X.tune_lib() if args.variant >= 0 else None
    wsv = torch.zeros(1 << 20, dtype=torch.uint8, device=dev) if args.variant >= 0 else None

    def step(s):
        b = s % pool
        verd = verds[s if per_step else b]
        recs = recss[s if per_step else 0]
        if rearm_in_loop and s >= pool:
            X.rearm_dev(umems[b], descss[b], verd, n, stream)  # conservative: counted inside the timing
        if args.variant >= 0:  # A/B timing of a tuning switch (counters as per-workgroup partials in ws)
            rc = tune.xsk_gpu__product_variant(args.variant, 0, umems[b].data_ptr(), umems[b].numel(),
                                               descss[b].data_ptr(), n, verd.data_ptr(), recs.data_ptr(),
                                               wsv.data_ptr(), stream.cuda_stream)
            assert rc == 0, rc
        else:
            X.echo_dev(umems[b], descss[b], n, verd, recs, stats, ws, stream, opts=args.opts)

    for s in range(W):
        step(s)
    torch.cuda.synchronize()

    # ---- timed region: exactly K steps between barrier + synchronize ----
    # One step is one kernel launch (the counters go out by device atomics, no fold launch), so the stream
    # events around the K back-to-back launches give the kernel's average launch duration (gaps included).
    # Per-launch events cost ~7 us per step at c3 (tools/gaptest.py), so the per-launch timer is only used
    # when a re-arm kernel shares the timed loop.
    per_launch_timer = rearm_in_loop
    X.timing_enable(per_launch_timer)
    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in range(W, W + K):
        step(s)
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    wall = t1 - t0
    ev_ms = ev0.elapsed_time(ev1)
    if per_launch_timer:
        kern_ms, launches = X.timing_read()
        X.timing_enable(False)
        timer_src = "HIP events around each launch (the timed loop also re-arms batches)"
    else:
        kern_ms, launches = ev_ms, K
        timer_src = "HIP events on the launch stream around the K back-to-back launches (one launch per step)"

    # ---- correctness of what was timed: every frame of every step accepted and counted, every step's verdicts
    # TX_REPLY and records carrying both verified input checksums (checked on the device after the timed region) ----
    st = stats.cpu().numpy().view(X.STATS_DTYPE)[0]
    ok = args.variant >= 0 or (int(st["rx_packets"]) == (W + K) * n and int(st["tx_packets"]) == (W + K) * n)
    ok = ok and all(bool((v == 0).all().item()) for v in verds)
    ok = ok and all(bool((r.view(-1, 16)[:, 1] == 3).all().item()) for r in recss)  # xsk_gpu_rec.flags
    checked = {"steps_with_outputs_checked": (W + K) if per_step else pool,
               "verdicts": "every step" if per_step else "the last use of each pooled batch",
               "records": "every step" if per_step else "the last step",
               "counters": "every step (rx / tx packets == steps x frames)"}

    # read-only streaming ceiling over one batch slab (context for the roofline)
    out = torch.zeros(1, dtype=torch.int64, device=dev)
    X.stream_read_dev(umems[0], batch_bytes, out, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(5):
        X.stream_read_dev(umems[0], batch_bytes, out, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    read_ceiling = batch_bytes * 5 / (e0.elapsed_time(e1) / 1e3) / 1e9

    kern_avg_ms = kern_ms / max(launches, 1)
    agg = reduce_ranks(rank, world, local, wall=wall, ev_ms=ev_ms, ok=ok, frames=K * n, frame_bytes=K * frame_bytes,
                       kern_avg_ms=kern_avg_ms, launch_bytes=frame_bytes,
                       reduce=lambda vals, op: allreduce(vals, op, world, dev))
    wall_max, ev_max, ok_all = agg["wall_max"], agg["ev_max"], agg["ok_ranks"]
    frames_all, bytes_all, per_rank = agg["frames"], agg["bytes"], agg["per_rank"]
    achieved = frame_bytes / (kern_avg_ms / 1e3) / 1e9

    if rank == 0:
        value = frames_all / wall_max / 1e6
        traffic, traffic_src = traffic_from_profiles(args.config + (f"_opts{args.opts}" if args.opts else ""), kernel,
                                                     X.build_id())
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mframes/s",
            "gib_per_s": round(bytes_all / wall_max / 2**30, 2),
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(wall_max / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config in STRONG else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded counter-based ICMP echo requests generated on-GPU, bit-identical "
                    "to oracle/echo_oracle.c)",
            "config": {"workload": desc, "frames_per_gpu": n, "frame_len": [lo, hi], "stride": stride,
                       "frame_bytes_per_gpu_step": frame_bytes, "parallelism": f"shard{world}:round-robin",
                       "layout": "device-resident UMEM slab + xdp_desc array", "pool_alloc": args.alloc,
                       "rearm_in_timed_region": rearm_in_loop},
            "verified": bool(ok_all == world),
            "verification": checked,
            **({"ab_variant": args.variant, "note": "A/B timing of a tuning variant, not the shipped kernel"}
               if args.variant >= 0 else {}),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "build_id": X.build_id(),
                         "kernel": kernel, "kernel_avg_us": round(kern_avg_ms * 1e3, 2), "kernel_timer": timer_src,
                         "algorithmic_bytes_per_launch": frame_bytes,
                         "read_ceiling_gbs": round(read_ceiling, 1),
                         # context for frac: a plain 16-B read of the same slab on this GPU (xsk_gpu_stream_read_dev);
                         # read kernels reach 0.90 of spec only as an asymptote of multi-GiB slabs
                         "frac_of_read_ceiling": frac_of_ceiling(achieved, read_ceiling),
                         "note": "rank 0's kernel; every rank's in per_rank"},
            "per_rank": per_rank,
            "event_ms_per_step": round(ev_max / K, 4),
        }
        if world == 1 and not args.no_cpu:
            log("[rank 0] CPU baseline ...")
            res["cpu_baseline"] = cpu_baseline(args.config)
        if world == 1 and not args.no_rx_loop:
            log("[rank 0] RX loop (tools/rxring) ...")
            res["rx_loop"] = rx_loop()
        if args.host_inclusive and world == 1:
            log("[rank 0] host-inclusive ...")
            res["host_inclusive"] = host_inclusive(args.config, local)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()  # the other ranks leave here: their GPUs are free for rank 0's multi leg
    if rank == 0:
        if world > 1 and not args.no_host_multi:
            log(f"[rank 0] host-inclusive over {world} GPUs ...")
            del slab, umems, descss  # the batch pool: HBM for the STAGED mirrors
            torch.cuda.empty_cache()
            res["host_inclusive_multi"] = host_inclusive_multi(args.config, world)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
