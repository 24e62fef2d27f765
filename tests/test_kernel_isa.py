"""The shipped transform kernels' instruction streams, pinned (no GPU).

tools/isa_manifest.py disassembles the gfx950 code objects of libxsknet_amd.so and hashes each kernel's instruction
text; tests/golden/kernel_isa.json holds the hashes of the transform kernels -- echo_round_kernel x 4 (reference and wire
mode, large and small batches) and lowlat_kernel x 2.  A source change meant to leave them alone (round 5 pruned 367
lines of losing switches from xsk_echo_device.h with every hash unchanged: profiles/r05/prune_isa.txt) fails here if
it does not; a change meant to alter them re-pins with `python tools/isa_manifest.py --write` in the same commit, so
the manifest always names the kernels the profiles of that build measured."""
import json
import os

import pytest

from tests.conftest import ROOT
from tests.test_lowlat_isa import LLVM

pytestmark = pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-objdump"), reason="llvm-objdump not installed")


def test_shipped_kernels_match_the_manifest():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_manifest as M
    want = json.load(open(M.MANIFEST))
    got = M.pinned(M.kernel_hashes())
    assert len(want) == 6 and sorted(want) == sorted(got), (sorted(want), sorted(got))
    for k in want:
        assert want[k] == got[k], (k, want[k], got[k])
