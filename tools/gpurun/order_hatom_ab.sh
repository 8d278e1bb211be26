#!/bin/bash
# OrderLS digit counts: per-row LDS atomics (DDSHE_ORDER_HATOM=1) against per-distinct-digit ballots, same
# box: order tests under the atomics, then the skew probe and the order bench line under both.
cd "$(dirname "$0")/../.." || exit 1
tools/gpurun/steps.sh \
  "300 t env DDSHE_ORDER_HATOM=1 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 p0 python3 -u tools/order_skew_probe.py" "200 p1 env DDSHE_ORDER_HATOM=1 python3 -u tools/order_skew_probe.py" \
  "200 b0 python3 -u bench.py --workload order --steps 20 --no-cpu-baseline" \
  "200 b1 env DDSHE_ORDER_HATOM=1 python3 -u bench.py --workload order --steps 20 --no-cpu-baseline" \
  "200 p0b python3 -u tools/order_skew_probe.py" "200 p1b env DDSHE_ORDER_HATOM=1 python3 -u tools/order_skew_probe.py"
