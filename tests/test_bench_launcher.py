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
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
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
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "1 GPU(s) visible" in str(e.value)
