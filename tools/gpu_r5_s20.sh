#!/bin/bash
# Round 5: which earlier test makes test_lowlat_timeout_exactly_once / fuzz[5] fail after the submit / complete split.
set -o pipefail
O=gpurun_out/s20
mkdir -p $O
T="timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread"
$T tests/test_gpu_staged.py::test_lowlat_timeout_exactly_once > $O/a_alone.log 2>&1; echo "alone rc=$?"
$T tests/test_gpu_rxloop.py tests/test_gpu_staged.py::test_lowlat_timeout_exactly_once > $O/b_rxloop.log 2>&1; echo "rxloop+ rc=$?"
$T tests/test_gpu_host.py tests/test_gpu_staged.py::test_lowlat_timeout_exactly_once > $O/c_host.log 2>&1; echo "host+ rc=$?"
$T tests/test_gpu_staged.py > $O/d_staged.log 2>&1; echo "staged rc=$?"
for f in $O/*.log; do echo "== $f"; grep -E "^E .*(differ|Error)|passed|failed" $f | cut -c1-700 | head -6; done
