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
