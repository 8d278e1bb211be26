#!/bin/bash
# k_msd_local: the multi-key buckets' id copy fused into the first partition round (DDSHE_ORDER_FUSECOPY=1,
# default) against the separate copy loop (0), one box: order tests under both, the order line and the skew
# probe alternating, kernel traces under both.
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
K="python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 fc_t1 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_mutations.py" \
  "300 fc_t0 env DDSHE_ORDER_FUSECOPY=0 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 fc_b0a env DDSHE_ORDER_FUSECOPY=0 $B" "200 fc_b1a $B" "200 fc_b0b env DDSHE_ORDER_FUSECOPY=0 $B" "200 fc_b1b $B" \
  "200 fc_p0 env DDSHE_ORDER_FUSECOPY=0 python3 -u tools/order_skew_probe.py" "200 fc_p1 python3 -u tools/order_skew_probe.py" \
  "200 fc_k0 env DDSHE_ORDER_FUSECOPY=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/fc_k0 -o run -- $K" \
  "200 fc_k1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/fc_k1 -o run -- $K"
