#!/bin/bash
# Round 5: address-reuse stress of registered UMEMs, then s19's sequence as the control on the same box.
set -o pipefail
O=gpurun_out/s24
mkdir -p $O
timeout -k 10 120 python -u tools/vareuse_stress.py --mode 2 --iters 400 --seconds 40 > $O/stress_lowlat.json 2>&1; echo "stress lowlat rc=$?"; cut -c1-600 $O/stress_lowlat.json
timeout -k 10 120 python -u tools/vareuse_stress.py --mode 0 --iters 400 --seconds 40 > $O/stress_zc.json 2>&1; echo "stress zc rc=$?"; cut -c1-600 $O/stress_zc.json
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_rxloop.py tests/test_gpu_host.py tests/test_gpu_staged.py > $O/seq.log 2>&1; echo "seq rc=$? $(tail -1 $O/seq.log)"
