#!/bin/bash
# Round-4 validation pass on one box: k_fold1 A/B, the whole GPU suite, smoke, and the bench lines.
export AB_NAME0=fold1_committed AB_NAME1=fold1_r01loop AB_NAME2=fold1_committed AB_NAME3=fold1_r01loop
tools/gpu_steps.sh \
 "120 abfold1 ./tools/abtest/ab_fold1 10000000 9" \
 "500 tests python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 bench_default python3 -u bench.py" \
 "240 bench_order python3 -u bench.py --workload order" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 bench_pf python3 -u bench.py --workload product_filter"
