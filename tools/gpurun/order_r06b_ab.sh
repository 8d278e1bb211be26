#!/bin/bash
# OrderLS round-6b A/B on one box: the carried plan checked inside k_rs_scan_chunks (each histogram block
# keeps only its largest holder key; no k_rs_red launch) and the read-back words stored by k_msd_big's last
# block (no k_rs_publish launch), against the previous build (tools/abtest/libs/libddshe_r06a.so: bounds
# in the histogram, k_rs_red check, k_rs_publish). Order tests on the new build (also with the publish
# launch), then the order line and the skew probe alternating, then a kernel trace of the new build.
export TMPDIR=/tmp
OLD=tools/abtest/libs/libddshe_r06a.so
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 ob_t python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_mutations.py" \
  "300 ob_tp env DDSHE_ORDER_PUBLISH=1 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py" \
  "200 ob_old_a env DDSHE_LIB=$OLD $B" "200 ob_new_a $B" "200 ob_old_b env DDSHE_LIB=$OLD $B" "200 ob_new_b $B" \
  "200 ob_pold env DDSHE_LIB=$OLD python3 -u tools/order_skew_probe.py" "200 ob_pnew python3 -u tools/order_skew_probe.py" \
  "200 ob_pub1 env DDSHE_ORDER_PUBLISH=1 $B" "200 ob_pub0 $B" \
  "200 ob_ks rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/order_b -o run -- python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
