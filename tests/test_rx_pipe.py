"""The pipelined RX loop's host logic (xsknet_amd/csrc/xsk_gpu_pipe.c, with xsk_gpu_rx.c's shared helpers) against fake
contexts and a simulated AF_XDP kernel side: compiled C unit test, no GPU (tests/c/test_rx_pipe.c)."""
import os
import subprocess
import tempfile

from tests.conftest import ROOT


def test_rx_pipe_c_unit():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-I", "/opt/rocm/include", "-o", exe,
                        os.path.join(ROOT, "tests", "c", "test_rx_pipe.c")], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=300).stdout
    assert "rx pipe ok" in out
