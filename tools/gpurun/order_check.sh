#!/bin/bash
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 oc2_t python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 oc2_b $B" \
  "200 oc2_ks rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/order_c -o run -- python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
