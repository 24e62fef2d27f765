"""The LOWLAT doorbell protocol's host state machine (xsknet_amd/csrc/xsk_lowlat_proto.h) on the CPU: a
compiled C unit test drives it against a simulated resident grid, including the timeout and recovery
paths that a real GPU run reaches only when the kernel hangs."""
import os
import subprocess
import tempfile

from tests.conftest import ROOT


def test_lowlat_protocol_c_unit():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-o", exe,
                        os.path.join(ROOT, "tests", "c", "test_lowlat_proto.c")], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=60).stdout
    assert "lowlat proto ok" in out
