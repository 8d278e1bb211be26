#!/bin/bash
# zero-copy Search bitmask with host-summed tile counts: parity tests, the product_filter line; then /Sum
# under 64 native callers by host wait mode (DDSHE_SYNC) and batches in flight
tools/gpu_steps.sh \
 "400 tests python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_mutations.py tests/test_gpu_routes.py tests/test_gpu_order.py -x -q --timeout 120 --timeout-method thread" \
 "300 bench_pf python3 -u bench.py --workload product_filter --no-cpu-baseline" \
 "300 pairs_auto env PAIR_SWEEP='0 2 64|0 4 64|100 2 64' bash tools/native/pairs_sweep.sh" \
 "300 pairs_block env DDSHE_SYNC=block PAIR_SWEEP='0 2 64|0 4 64|0 8 64' bash tools/native/pairs_sweep.sh" \
 "300 pairs_yield env DDSHE_SYNC=yield PAIR_SWEEP='0 2 64|0 4 64' bash tools/native/pairs_sweep.sh" \
 "300 pairs_spin env DDSHE_SYNC=spin PAIR_SWEEP='0 2 64|0 4 64' bash tools/native/pairs_sweep.sh"
