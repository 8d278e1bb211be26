#!/bin/bash
# Round-6 validation on one box: the GPU suite, smoke, the bench lines of every workload, the launcher's
# refusal of --gpus 2 on a one-GPU box (exit 2 expected) and its two-rank gloo rehearsal.
export TMPDIR=/tmp
tools/gpurun/steps.sh \
 "600 tests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "400 bench_default python3 -u bench.py" \
 "240 bench_order python3 -u bench.py --workload order" \
 "300 bench_pf python3 -u bench.py --workload product_filter" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 bench_gloo2 env DDSHE_DIST_BACKEND=gloo python3 -u bench.py --gpus 2 --steps 5" \
 "120 nccl2_refused bash -c 'python3 bench.py --gpus 2 --steps 1; rc=\$?; echo rc=\$rc; test \$rc -eq 2'"
