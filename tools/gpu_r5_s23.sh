#!/bin/bash
# Round 5: are the misdirected / lost GPU writes to host memory (s22) tied to transparent huge pages?
set -o pipefail
O=gpurun_out/s23
mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag \
    /sys/kernel/mm/transparent_hugepage/khugepaged/defrag /sys/kernel/mm/transparent_hugepage/khugepaged/pages_to_scan \
    /sys/kernel/mm/transparent_hugepage/khugepaged/scan_sleep_millisecs 2>&1 | tee $O/thp.txt
grep -E "thp_|compact_" /proc/vmstat | head -30 > $O/vmstat_before.txt
T="timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread"
S="tests/test_gpu_rxloop.py::test_rx_pipe_end_to_end[2-2-64] tests/test_gpu_host.py tests/test_gpu_staged.py"
XSK_TEST_NO_THP=1 $T $S > $O/nothp1.log 2>&1; echo "nothp1 rc=$? $(tail -1 $O/nothp1.log)"
XSK_TEST_NO_THP=1 $T $S > $O/nothp2.log 2>&1; echo "nothp2 rc=$? $(tail -1 $O/nothp2.log)"
$T $S > $O/thp1.log 2>&1; echo "thp1 rc=$? $(tail -1 $O/thp1.log)"
XSK_TEST_NO_THP=1 $T $S > $O/nothp3.log 2>&1; echo "nothp3 rc=$? $(tail -1 $O/nothp3.log)"
$T $S > $O/thp2.log 2>&1; echo "thp2 rc=$? $(tail -1 $O/thp2.log)"
grep -E "thp_|compact_" /proc/vmstat | head -30 > $O/vmstat_after.txt
