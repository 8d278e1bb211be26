#!/bin/bash
# zero-copy Search mask: its parity tests, then the product_filter line (route timing) both ways
tools/gpu_steps.sh \
 "300 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_mutations.py tests/test_gpu_routes.py -x -q --timeout 120 --timeout-method thread" \
 "300 bench_pf python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 bench_pf_dma env DDSHE_MASK_ZEROCOPY=0 python3 -u bench.py --workload product_filter --no-cpu-baseline"
