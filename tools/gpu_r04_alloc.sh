#!/bin/bash
# engine-allocated reply buffers: tests, then the product_filter line twice (search route into a
# dds_host_alloc buffer and into a registered numpy array, same process)
tools/gpu_steps.sh \
 "300 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_routes.py -x -q --timeout 120 --timeout-method thread" \
 "300 pf1 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf2 python3 -u bench.py --workload product_filter --no-cpu-baseline"
