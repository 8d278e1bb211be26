#!/bin/bash
# k_msd_local with 8 buckets per wave (DDSHE_ORDER_MSDWAVE=8, default) against one wave per bucket (1,
# round 5), same box: order tests under both, the skew probe (bench column, uniform 54-bit keys: every
# bucket multi-key, three keys) and the order line, alternating.
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 mw_t8 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "300 mw_t64 env DDSHE_ORDER_MSDWAVE=64 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 mw_p1a env DDSHE_ORDER_MSDWAVE=1 python3 -u tools/order_skew_probe.py" \
  "200 mw_p8a env DDSHE_ORDER_MSDWAVE=8 python3 -u tools/order_skew_probe.py" \
  "200 mw_b1a env DDSHE_ORDER_MSDWAVE=1 $B" \
  "200 mw_b8a env DDSHE_ORDER_MSDWAVE=8 $B" \
  "200 mw_p1b env DDSHE_ORDER_MSDWAVE=1 python3 -u tools/order_skew_probe.py" \
  "200 mw_p8b env DDSHE_ORDER_MSDWAVE=8 python3 -u tools/order_skew_probe.py" \
  "200 mw_b1b env DDSHE_ORDER_MSDWAVE=1 $B" \
  "200 mw_b8b env DDSHE_ORDER_MSDWAVE=8 $B" \
  "200 mw_ks rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/order_mw -o run -- $B --steps 10"
