#!/bin/bash
# 16-byte non-temporal zero-copy mask stores as the default: mask / route tests, then the product_filter
# line against one word per lane, twice each (same box)
tools/gpu_steps.sh \
 "300 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_routes.py tests/test_gpu_mutations.py -x -q --timeout 120 --timeout-method thread" \
 "300 pf16a python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf4a env DDSHE_MASK_STORE=4 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf16b python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf4b env DDSHE_MASK_STORE=4 python3 -u bench.py --workload product_filter --no-cpu-baseline"
