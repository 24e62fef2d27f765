"""The host memory bookkeeping (xsknet_amd/csrc/xsk_gpu_mem.c): the counted UMEM registrations and the buffers kept while
a resident grid runs, against stub runtime calls that behave as the HIP runtime was measured to -- compiled C unit test,
no GPU (tests/c/test_mem.c)."""
import os
import subprocess
import tempfile

from tests.conftest import ROOT


def test_mem_c_unit():
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "t")
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-pthread", "-I", "/opt/rocm/include",
                        "-o", exe, os.path.join(ROOT, "tests", "c", "test_mem.c")], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=300).stdout
    assert "mem ok" in out
