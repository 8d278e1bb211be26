#!/bin/bash
# k_msd_local's small-bucket list with bounds in the entries and the next entry prefetched (in-tree, C)
# against the list of bucket ids (B: tools/abtest/libs/libddshe_msdb1.so) and the bucket ranges per wave
# (A: tools/abtest/libs/libddshe_swar4.so), same box: order tests on C, the skew probe (uniform 54-bit keys:
# every bucket small and multi-key) and the order line per build (A B C, twice), a trace of C.
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
A="env DDSHE_LIB=$L/libddshe_swar4.so"
B1="env DDSHE_LIB=$L/libddshe_msdb1.so"
exec tools/gpurun/steps.sh "300 mq_tC $T" \
  "200 mq_pAa $A $P" "200 mq_pBa $B1 $P" "200 mq_pCa $P" "200 mq_pAb $A $P" "200 mq_pBb $B1 $P" "200 mq_pCb $P" \
  "200 mq_bAa $A $B" "200 mq_bBa $B1 $B" "200 mq_bCa $B" "200 mq_bAb $A $B" "200 mq_bBb $B1 $B" "200 mq_bCb $B" \
  "200 mq_kC rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/order_mqC -o run -- $B --steps 10"
