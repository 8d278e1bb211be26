#!/bin/bash
# Round-6 closing bench lines on one box (the GPU suite + smoke ran in the call before): every workload's
# line, the launcher's refusal of --gpus 2 on a one-GPU box (exit 2 expected) and its two-rank gloo
# rehearsal, then kernel stats of the headline and OrderLS lines.
export TMPDIR=/tmp
tools/gpurun/steps.sh \
 "400 bench_default python3 -u bench.py" \
 "240 bench_order python3 -u bench.py --workload order" \
 "300 bench_pf python3 -u bench.py --workload product_filter" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 bench_gloo2 env DDSHE_DIST_BACKEND=gloo python3 -u bench.py --gpus 2 --steps 5" \
 "120 nccl2_refused bash -c 'python3 bench.py --gpus 2 --steps 1; rc=\$?; echo rc=\$rc; test \$rc -eq 2'" \
 "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6b/sum -o run -- python3 -u bench.py --no-extras --steps 10" \
 "240 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6b/order -o run -- python3 -u bench.py --workload order --steps 10 --no-cpu-baseline"
