#!/bin/bash
# k_msd_local_blk whose large entries carry the bucket's bounds (in-tree, B: 768 blocks, block j entries j,
# j + 768, ...) against the bucket ranges per wave (A: tools/abtest/libs/libddshe_swar4.so), same box: order
# tests on B, the order line (A B, three times) and the skew probe per build, a trace of B.
# (Earlier run: block j reading segment j % 64's entries j / 64, j / 64 + 12, ...: k_msd_local_blk 21.5 us
# against 16.3 for one entry per block by the global index: segments of > 12 entries serialise.)
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
A="env DDSHE_LIB=$L/libddshe_swar4.so"
exec tools/gpurun/steps.sh "300 ms_tB $T" \
  "200 ms_bAa $A $B" "200 ms_bBa $B" "200 ms_bAb $A $B" "200 ms_bBb $B" "200 ms_bAc $A $B" "200 ms_bBc $B" \
  "200 ms_pA $A $P" "200 ms_pB $P" \
  "200 ms_kB rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/order_msB -o run -- $B --steps 10"
