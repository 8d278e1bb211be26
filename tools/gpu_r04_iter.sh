#!/bin/bash
# iteration pass: the tests of the paths changed since the last full run, then their bench lines
tools/gpu_steps.sh \
 "400 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_mutations.py tests/test_gpu_order.py tests/test_gpu_routes.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "240 bench_order python3 -u bench.py --workload order --no-cpu-baseline" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 bench_pf python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "240 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/order -o run -- python3 bench.py --no-cpu-baseline --workload order --steps 5"
