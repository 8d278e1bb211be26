#!/bin/bash
# OrderLS dictionary codes (B: DDSHE_ORDER_DICT=1, default) against the key passes (A: 0), same box: the
# order tests both ways, the order bench line and the skew probe per build (A B, twice), a kernel trace of B.
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
exec tools/gpurun/steps.sh \
  "300 dt_B $T" \
  "300 dt_A env DDSHE_ORDER_DICT=0 $T" \
  "200 db_Aa env DDSHE_ORDER_DICT=0 $B" "200 db_Ba $B" \
  "200 db_Ab env DDSHE_ORDER_DICT=0 $B" "200 db_Bb $B" \
  "200 dp_A env DDSHE_ORDER_DICT=0 $P" "200 dp_B $P" \
  "200 dk_B rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dict/order_B -o run -- $B --steps 10"
