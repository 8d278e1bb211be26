#!/bin/bash
# k_msd_local: the partition's first round keyed by the smallest key of the bucket's first chunk
# (DDSHE_ORDER_MINFIRST=1, default) against the first row's key (0), one box: order tests under both, the
# order line and the skew probe alternating, kernel traces under both.
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
K="python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 mf_t1 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_mutations.py" \
  "300 mf_t0 env DDSHE_ORDER_MINFIRST=0 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 mf_b0a env DDSHE_ORDER_MINFIRST=0 $B" "200 mf_b1a $B" "200 mf_b0b env DDSHE_ORDER_MINFIRST=0 $B" "200 mf_b1b $B" \
  "200 mf_p0 env DDSHE_ORDER_MINFIRST=0 python3 -u tools/order_skew_probe.py" "200 mf_p1 python3 -u tools/order_skew_probe.py" \
  "200 mf_k0 env DDSHE_ORDER_MINFIRST=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/mf_k0 -o run -- $K" \
  "200 mf_k1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/mf_k1 -o run -- $K"
