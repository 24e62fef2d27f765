"""Test configuration: `gpu` marker, repo on sys.path, native libraries built on demand."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session", autouse=True)
def _native_libs():
    """Build oracle/liboracle.so and the product library if they are missing (no-op otherwise)."""
    need = [os.path.join(ROOT, "oracle", "liboracle.so"), os.path.join(ROOT, "xsknet_amd", "libxsknet_amd.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-s", "-C", ROOT, "xsknet_amd/libxsknet_amd.so", "oracle"], check=True)
    yield


def golden_frames():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "frames.json")) as f:
        return json.load(f)


def golden_kat():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)


@pytest.fixture(autouse=True)
def _no_resident_grid_outlives_its_channel(request):
    """After every GPU test, once its contexts are collected, no LOWLAT resident grid may still run on cuda:0
    (xsk_gpu__lowlat_live): a grid that outlived its channel would keep polling memory a later channel reuses."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    try:
        import torch
        if not torch.cuda.is_available():
            return
    except ImportError:
        return
    import gc
    import xsknet_amd as X
    gc.collect()
    live = X.lowlat_live(0)
    assert live == 0, f"{live} resident LOWLAT workgroups still running after {request.node.nodeid}"
