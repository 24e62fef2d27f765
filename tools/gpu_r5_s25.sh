#!/bin/bash
# Round 5: NUMA balancing (PROT_NONE hinting of the UMEM's pages -> MMU-notifier eviction of the GPU queues) as the
# trigger of the misdirected host-memory writes?  Box settings, then the failing sequence with and without it.
set -o pipefail
O=gpurun_out/s25
mkdir -p $O
{ echo "numa_balancing $(cat /proc/sys/kernel/numa_balancing 2>&1)"; lscpu | grep -i "numa node" ; uname -r;
  cat /sys/module/amdgpu/parameters/noretry 2>&1; cat /proc/cmdline; } > $O/box.txt 2>&1; cat $O/box.txt
grep -E "^numa_" /proc/vmstat > $O/vmstat0.txt
S="tests/test_gpu_rxloop.py tests/test_gpu_host.py tests/test_gpu_staged.py tests/test_gpu_fuzz.py"
T="timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread"
$T $S > $O/ctl1.log 2>&1; echo "ctl1 rc=$? $(tail -1 $O/ctl1.log)"
grep -E "^numa_" /proc/vmstat > $O/vmstat1.txt
XSK_TEST_NO_NUMA_BALANCING=1 $T $S > $O/nonuma1.log 2>&1; echo "nonuma1 rc=$? $(tail -1 $O/nonuma1.log)"
grep -E "^numa_" /proc/vmstat > $O/vmstat2.txt
$T $S > $O/ctl2.log 2>&1; echo "ctl2 rc=$? $(tail -1 $O/ctl2.log)"
XSK_TEST_NO_NUMA_BALANCING=1 $T $S > $O/nonuma2.log 2>&1; echo "nonuma2 rc=$? $(tail -1 $O/nonuma2.log)"
paste $O/vmstat0.txt $O/vmstat1.txt $O/vmstat2.txt | awk '{print $1, $4-$2, $6-$4}'
