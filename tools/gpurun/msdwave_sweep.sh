#!/bin/bash
# k_msd_local buckets per wave (DDSHE_ORDER_MSDWAVE) sweep on one box: order line (resident device time)
# and the skew probe per setting, then the kernel traces (k_msd_local device time per call).
export TMPDIR=/tmp
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
K="python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "200 mw3_p2 env DDSHE_ORDER_MSDWAVE=2 python3 -u tools/order_skew_probe.py" \
  "200 mw3_p4 env DDSHE_ORDER_MSDWAVE=4 python3 -u tools/order_skew_probe.py" \
  "200 mw3_p1 env DDSHE_ORDER_MSDWAVE=1 python3 -u tools/order_skew_probe.py" \
  "200 mw3_k1 env DDSHE_ORDER_MSDWAVE=1 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/mw_k1 -o run -- $K" \
  "200 mw3_k2 env DDSHE_ORDER_MSDWAVE=2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/mw_k2 -o run -- $K" \
  "200 mw3_k4 env DDSHE_ORDER_MSDWAVE=4 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof6/mw_k4 -o run -- $K"
