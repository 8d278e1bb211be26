#!/bin/bash
# dense-rank ordering: parity tests, the hash-set microbench, then the order line both ways (same box)
tools/gpu_steps.sh \
 "60 hash tools/microbench/dr_hash_probe 10000000 10000" \
 "400 tests python3 -u -m pytest tests/test_gpu_order.py tests/test_gpu_routes.py -x -q --timeout 200 --timeout-method thread" \
 "300 order_dense python3 -u bench.py --workload order --no-cpu-baseline" \
 "300 order_bits env DDSHE_ORDER_DENSE=0 python3 -u bench.py --workload order --no-cpu-baseline" \
 "300 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/order -o run -- python3 bench.py --no-cpu-baseline --no-e2e --workload order --steps 5"
