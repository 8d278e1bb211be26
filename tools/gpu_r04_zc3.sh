#!/bin/bash
# same-box A/B of the zero-copy Search count (host-summed tile counts vs device total + hand-off launch),
# and /Sum under 64 native callers with pre-sized batch buffers and a loaded warm-up
tools/gpu_steps.sh \
 "300 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_routes.py -x -q --timeout 120 --timeout-method thread" \
 "300 pf_tiles python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf_atomic env DDSHE_MASK_COUNT=atomic python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf_tiles2 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf_atomic2 env DDSHE_MASK_COUNT=atomic python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 t_atomic env DDSHE_MASK_COUNT=atomic python3 -u -m pytest tests/test_gpu_strtab.py -x -q --timeout 120 --timeout-method thread -k mask" \
 "300 pairs env PAIR_SWEEP='0 2 64|100 2 64|0 4 64|100 4 64|0 8 64|0 2 128' bash tools/native/pairs_sweep.sh"
