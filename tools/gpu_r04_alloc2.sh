#!/bin/bash
# cached mapped addresses, workers created outside the context lock: tests, Search / Order lines, /Sum sweep
tools/gpu_steps.sh \
 "400 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_routes.py tests/test_gpu_order.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread" \
 "300 pf python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 order python3 -u bench.py --workload order --no-cpu-baseline" \
 "300 pairs env PAIR_SWEEP='0 4 64|0 4 64|0 2 64|0 8 64' bash tools/native/pairs_sweep.sh"
