#!/bin/bash
# zero-copy Search mask and pairwise batches: their parity tests, the product_filter line (route timing)
# both ways, then /Sum under 64 native callers (sweep, and the staged pairwise path for A/B)
tools/gpu_steps.sh \
 "400 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_mutations.py tests/test_gpu_routes.py tests/test_gpu_parity.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread" \
 "300 bench_pf python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 bench_pf_dma env DDSHE_MASK_ZEROCOPY=0 python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "600 pairs_sweep bash tools/native/pairs_sweep.sh" \
 "300 pairs_staged env DDSHE_PAIR_ZEROCOPY=0 PAIR_SWEEP='100 2 64|20 4 64' bash tools/native/pairs_sweep.sh"
