"""bench.py's multi-GPU launch (no GPU needed): `python bench.py --gpus N` without a launcher starts
`torch.distributed.run --nproc-per-node N` as a child before anything touches a GPU, forwards the same
arguments, and exits with the child's status; a rank whose WORLD_SIZE differs from --gpus refuses to run."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_launcher_spawns_n_ranks(monkeypatch):
    bench = _bench()
    seen = {}

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 7)

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    import xsknet_amd

    def no_gpu(*a, **k):
        raise AssertionError("the launcher must not load the HIP library")

    monkeypatch.setattr(xsknet_amd, "lib", no_gpu)
    # the parent counts GPUs in the KFD topology only: every torch / HIP device query must stay untouched
    for fn in ("device_count", "is_available", "init", "set_device", "mem_get_info", "synchronize"):
        monkeypatch.setattr(bench.torch.cuda, fn, no_gpu)
    monkeypatch.setattr(bench, "kfd_gpu_count", lambda *a, **k: 8)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5", "--config", "c5"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7  # the children's status
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-6:] == ["--gpus", "8", "--steps", "5", "--config", "c5"]
    assert os.path.samefile(cmd[-7], os.path.join(ROOT, "bench.py"))


def test_rank_refuses_world_size_mismatch(monkeypatch):
    bench = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(SystemExit) as e:
        bench.dist_setup(8)
    assert "WORLD_SIZE=2" in str(e.value)


def test_launch_command_runs_ranks_with_gloo(tmp_path):
    """The launch line bench.py builds really starts N ranks that see RANK / WORLD_SIZE (a stand-in
    script in place of bench.py, over gloo, world size 2)."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "import torch\n"
        "t = torch.ones(1) * (dist.get_rank() + 1)\n"
        "dist.all_reduce(t)\n"
        "if dist.get_rank() == 0: print('world', dist.get_world_size(), 'sum', int(t.item()))\n"
        "dist.destroy_process_group()\n")
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(script)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    # own process group: a hung launch is killed with all its ranks
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=180)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)
        p.communicate()
        raise
    r = subprocess.CompletedProcess(cmd, p.returncode, out, err)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "world 2 sum 3" in r.stdout


def test_launcher_refuses_more_ranks_than_gpus(monkeypatch):
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "SHARE_GPU", False)
    monkeypatch.setattr(bench, "kfd_gpu_count", lambda *a, **k: 1)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: (_ for _ in ()).throw(AssertionError("GPU query")))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "1 GPU(s) visible" in str(e.value)


def test_launcher_without_kfd_leaves_it_to_the_ranks(monkeypatch):
    """No readable KFD topology: the parent launches anyway (a rank without a GPU fails loudly itself)."""
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "SHARE_GPU", False)
    monkeypatch.setattr(bench, "KFD_NODES", "/nonexistent/kfd/nodes")
    monkeypatch.setattr(bench, "kfd_gpu_count", lambda *a, **k: None)
    monkeypatch.setattr(bench, "launch_ranks", lambda g: 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0


def _fake_kfd(root, gpu_ids):
    for i, g in enumerate(gpu_ids):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(f"{g}\n")
        (d / "properties").write_text(f"cpu_cores_count {0 if g else 64}\nsimd_count {0 if not g else 1024}\n")
    return str(root)


def test_kfd_parser_counts_gpu_nodes(tmp_path):
    """The KFD topology of an 8-GPU node: 2 CPU nodes (gpu_id 0) + 8 GPU nodes; visibility lists narrow it."""
    bench = _bench()
    nodes = _fake_kfd(tmp_path / "nodes", [0, 0, 41234, 52345, 63456, 7456, 8567, 9678, 10789, 11890])
    assert bench.kfd_gpu_count(nodes, env={}) == 8
    assert bench.kfd_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.kfd_gpu_count(nodes, env={"ROCR_VISIBLE_DEVICES": "3"}) == 1
    assert bench.kfd_gpu_count(nodes, env={"CUDA_VISIBLE_DEVICES": ""}) == 0
    assert bench.kfd_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": "0,9,1"}) == 1  # stops at the invalid id
    assert bench.kfd_gpu_count(nodes, env={"HIP_VISIBLE_DEVICES": "0,1,2,3", "ROCR_VISIBLE_DEVICES": "0,1"}) == 2
    # a node without gpu_id (a partially populated topology) is skipped
    os = __import__("os")
    os.remove(os.path.join(nodes, "2", "gpu_id"))
    assert bench.kfd_gpu_count(nodes, env={}) == 7
    assert bench.kfd_gpu_count(str(tmp_path / "missing"), env={}) is None


def test_traffic_provenance(tmp_path):
    """roofline.traffic is attached only when the summary names the kernel that ran AND the running build."""
    import json
    bench = _bench()
    k = bench.KERNEL
    p = tmp_path / "traffic_c3.json"
    p.write_text(json.dumps({"kernel": k, "build_id": "abc", "hbm_bytes_per_launch": 1714382400}))
    assert bench.traffic_from_profiles("c3", k, "abc", str(p))[0] == 1714382400
    t, src = bench.traffic_from_profiles("c3", k, "other", str(p))
    assert t is None and "build" in src
    t, src = bench.traffic_from_profiles("c3", k + " ", "abc", str(p))
    assert t is None and "kernel" in src
    p.write_text(json.dumps({"kernel": k, "hbm_bytes_per_launch": 1}))  # no build id recorded
    assert bench.traffic_from_profiles("c3", k, "abc", str(p))[0] is None
    assert bench.traffic_from_profiles("c3", k, "abc", str(tmp_path / "none.json"))[0] is None


def test_frac_of_read_ceiling_on_a_fake_line():
    """roofline.frac_of_read_ceiling = achieved / read_ceiling_gbs: on round 3's driver line (c3, 5 655 GB/s
    of frame bytes per kernel time, the read ceiling 6 960 GB/s measured beside it) it is 0.8125, against 0.707 of the
    8 TB/s spec; no ceiling -> None."""
    bench = _bench()
    line = {"roofline": {"achieved": 5655.0, "peak": bench.HBM_PEAK_GBS, "read_ceiling_gbs": 6960.0}}
    r = line["roofline"]
    r["frac_of_read_ceiling"] = bench.frac_of_ceiling(r["achieved"], r["read_ceiling_gbs"])
    assert r["frac_of_read_ceiling"] == 0.8125
    assert r["frac_of_read_ceiling"] > r["achieved"] / r["peak"]
    assert bench.frac_of_ceiling(5655.0, 0.0) is None and bench.frac_of_ceiling(5655.0, None) is None
    # the 0.90-of-spec target sits above the ceiling itself: 0.90 x 8000 > 6960
    assert 0.90 * bench.HBM_PEAK_GBS > r["read_ceiling_gbs"]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_c5_pool_plan(world):
    """c5 splits 64 M x 1500-B frames (2 KiB stride) over the ranks: the per-rank batch, the pool that fits a
    288 GB MI355X (about 280 GiB free after the runtime) and the re-arm decision for the driver's K=20, W=5."""
    bench = _bench()
    n_total, lo, hi, stride = bench.CONFIGS["c5"][:4]
    assert n_total % world == 0
    n = n_total // world
    free = 280 * 2**30
    pool, rearm = bench.pool_plan(n, stride, free, 5, 20)
    per = n * stride + n * 16
    assert pool >= 1 and (pool + 1) * per <= free * 0.85 or pool == 1
    assert rearm == (pool < 25)
    # the pool's outputs (verdicts per pooled batch when re-arming, records, stats) still fit beside it
    outputs = (pool if rearm else 1) * n + n * 16 + 40
    assert pool * per + outputs < free
    if world == 1:
        assert pool == 1 and rearm  # 128 GiB: one batch, re-armed every step
    if world == 8:
        assert pool >= 10  # 16 GiB batches


def _reduce_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def reduce(vals, op):
            t = torch.tensor(vals, dtype=torch.float64)
            dist.all_reduce(t, op=op)
            return t.tolist()
        agg = bench.reduce_ranks(rank, world, local=rank, wall=0.1 * (rank + 1), ev_ms=50.0 + rank, ok=True,
                                 frames=20 * (1 << 20), frame_bytes=20 * 1572864000, kern_avg_ms=0.275 + 0.01 * rank,
                                 launch_bytes=1572864000, reduce=reduce)
        q.put((rank, agg))
    finally:
        dist.destroy_process_group()


def test_reduce_ranks_gloo_world2():
    """bench.py's cross-rank step over gloo at world size 2 (the driver's N > 1 runs use RCCL): the slowest rank's
    wall time, summed frames / bytes / verification, and every rank's kernel time, GB/s and frac in rank 0's line."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_reduce_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = got[0]
    assert a == got[1]  # every rank sees the same reduction
    assert abs(a["wall_max"] - 0.2) < 1e-12 and a["ev_max"] == 51.0 and a["ok_ranks"] == 2.0
    assert a["frames"] == 2 * 20 * (1 << 20) and a["bytes"] == 2 * 20 * 1572864000
    pr = a["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1] and [r["device"] for r in pr] == [0, 1]
    assert [r["kernel_avg_us"] for r in pr] == [275.0, 285.0]
    assert pr[0]["achieved_gbs"] == round(1572864000 / 275e-6 / 1e9, 1)
    assert pr[1]["frac"] == round(1572864000 / 285e-6 / 1e9 / 8000.0, 4)
    assert [r["wall_ms"] for r in pr] == [100.0, 200.0] and pr[1]["frames"] == 20 * (1 << 20)


def test_host_inclusive_multi_devices_and_failure_is_recorded():
    """N > 1 runs: rank 0's multi-GPU host-inclusive leg uses one context per rank's GPU (every one on cuda:0 in the
    one-GPU rehearsal) and records a failure in its own field instead of raising -- here there is no GPU, so
    xsk_gpu_multi_init fails and the bench line would still print."""
    import bench
    assert bench.multi_devices(4) == [0, 1, 2, 3]
    assert bench.multi_devices(3, share_gpu=True) == [0, 0, 0]
    out = bench.host_inclusive_multi("c3", 2, budget_s=0.05, n=256)
    assert out["devices"] == [0, 1] and out["frames_per_call"] == 256 and out["mode"] == "staged"
    assert "error" in out and "g2" not in out


def test_rx_loop_leg_parses_rxring_and_never_fails_the_line(tmp_path, monkeypatch):
    """bench.py's RX-loop leg: each tools/rxring run's JSON line becomes a record; a missing tool or a run that prints
    no JSON is reported in the record, never raised (a measurement leg must not cost the bench line)."""
    bench = _bench()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert "skipped" in bench.rx_loop(0.1)
    (tmp_path / "tools").mkdir()
    exe = tmp_path / "tools" / "rxring"
    line = ('{"tool": "rxring", "per_queue": [{"mode": 2, "mframes_s": 28.7, "us_per_step": 4.2, "p50_us": 3.1, '
            '"p99_us": 9.0}], "frames": 1000, "checked": 1000, "tx_full": 0, "failures": 0, "rc": 0}')
    exe.write_text("#!/bin/sh\ncase \"$*\" in *1024*) echo nothing; exit 1;; esac\necho '" + line + "'\n")
    exe.chmod(0o755)
    r = bench.rx_loop(0.1)
    assert r["step64"] == {"mframes_per_s": 28.7, "us_per_step": 4.2, "p50_us": 3.1, "p99_us": 9.0, "frames": 1000,
                           "checked": 1000, "failures": 0, "tx_full": 0, "mode": 2}
    assert r["step64_pipe4"]["mframes_per_s"] == 28.7
    assert "error" in r["step1024"]
    assert r["step64_pipe8_hwq8"]["env"] == {"GPU_MAX_HW_QUEUES": "8"}
