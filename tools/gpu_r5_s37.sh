#!/bin/bash
# (This session staged doorbell batches of small frames through slots in pinned memory; the A/B below lost and the
# staging was reverted -- DESIGN.md §3.3.  tools/layout_lat.py and echo_replay no longer take stage=.)
# Round 5: staged doorbell batches of small frames -- host + staged + fuzz + pipe GPU tests, then the layout A/B.
set -o pipefail
O=gpurun_out/s37
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_host.py tests/test_gpu_fuzz.py \
    tests/test_gpu_rxloop.py tests/test_gpu_staged.py tests/test_gpu_zpipe.py > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" $O/tests.log | cut -c1-600 | tail -6
[ $rc -eq 0 ] || exit $rc
for len in 64 98; do
  timeout -k 10 200 python -u tools/layout_lat.py --reps 400 --len $len >> $O/layout.jsonl 2>&1 || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/s37/layout.jsonl'):
    d=json.loads(l); print(d['layout'], d['frame_len'], d['us_per_call'], d.get('gpu_us',{}).get('transform'), d.get('gpu_us',{}).get('host_doorbell_to_done'))
"
