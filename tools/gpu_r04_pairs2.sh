#!/bin/bash
# pairwise worker pool: route / concurrency tests, then /Sum under 64 and 128 native callers
tools/gpu_steps.sh \
 "300 tests python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_concurrency.py tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread" \
 "300 pairs env PAIR_SWEEP='0 4 64|0 4 64|0 4 64|0 2 64|0 4 128' bash tools/native/pairs_sweep.sh"
