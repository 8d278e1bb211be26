#!/bin/bash
# /Sum under 64 native callers: inside the bench (child of the bench process) and standalone, with the
# longest batch split into its GPU round trip
tools/gpu_steps.sh \
 "300 routes python3 -u -m pytest tests/test_gpu_routes.py -x -q --timeout 120 --timeout-method thread" \
 "400 bench python3 -u bench.py --no-cpu-baseline" \
 "300 pairs env PAIR_SWEEP='0 4 64|0 4 64|0 4 64' bash tools/native/pairs_sweep.sh"
