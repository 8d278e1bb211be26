#!/bin/bash
# zero-copy Search mask store width A/B (DDSHE_MASK_STORE 4 / 8 / 16): mask tests per width, then the
# product_filter line per width, twice (same box)
tools/gpu_steps.sh \
 "300 t8 env DDSHE_MASK_STORE=8 python3 -u -m pytest tests/test_gpu_strtab.py -x -q --timeout 120 --timeout-method thread -k mask" \
 "300 t16 env DDSHE_MASK_STORE=16 python3 -u -m pytest tests/test_gpu_strtab.py -x -q --timeout 120 --timeout-method thread -k mask" \
 "300 pf4a python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf8a env DDSHE_MASK_STORE=8 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf16a env DDSHE_MASK_STORE=16 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf4b python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pf8b env DDSHE_MASK_STORE=8 python3 -u bench.py --workload product_filter --no-cpu-baseline"
