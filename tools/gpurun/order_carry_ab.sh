#!/bin/bash
# OrderLS carried-plan A/B on one box: the order tests, then the order line with the
# min / max pass every call (DDSHE_ORDER_CARRY=0) and with the carried plan (1), alternating; then the
# kernel trace and the FETCH_SIZE / WRITE_SIZE passes of the carried form (tools/order_call_traffic.py
# cuts them per call).
export TMPDIR=/tmp
P=gpurun_out/prof6
B="python3 -u bench.py --workload order --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 oc_tests python -u -m pytest tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread" \
  "150 oc_0a env DDSHE_ORDER_CARRY=0 $B --steps 20" \
  "150 oc_1a env DDSHE_ORDER_CARRY=1 $B --steps 20" \
  "150 oc_0b env DDSHE_ORDER_CARRY=0 $B --steps 20" \
  "150 oc_1b env DDSHE_ORDER_CARRY=1 $B --steps 20" \
  "240 oc_ks rocprofv3 --kernel-trace --stats --output-format csv -d $P/order -o run -- $B --steps 10" \
  "240 oc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_order_fetch -o run -- $B --steps 2 --warmup 1 --verify 0" \
  "240 oc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_order_write -o run -- $B --steps 2 --warmup 1 --verify 0"
