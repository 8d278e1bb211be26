#!/bin/bash
# Round-4 final validation on one box: the whole GPU suite, smoke, and the bench lines.
tools/gpu_steps.sh \
 "500 tests python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 bench_default python3 -u bench.py" \
 "240 bench_order python3 -u bench.py --workload order" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 bench_pf python3 -u bench.py --workload product_filter" \
 "300 pairs env PAIR_SWEEP='0 4 64|100 4 64|0 2 64|0 8 64|0 4 128' bash tools/native/pairs_sweep.sh"
