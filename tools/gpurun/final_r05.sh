#!/bin/bash
# Round-5 validation on one box: the GPU suite, smoke, and the bench lines of every workload.
tools/gpurun/steps.sh \
 "600 tests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 bench_default python3 -u bench.py" \
 "240 bench_order python3 -u bench.py --workload order" \
 "300 bench_pf python3 -u bench.py --workload product_filter" \
 "300 bench_es python3 -u bench.py --workload entry_search"
