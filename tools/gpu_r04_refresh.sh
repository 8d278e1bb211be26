#!/bin/bash
# Round-4 profile refresh with the final code: default and entry_search bench lines, and the kernel stats of
# the product_filter workload (the zero-copy Search route included)
export TMPDIR=/tmp
P=gpurun_out/prof
tools/gpu_steps.sh \
 "400 bench_default python3 -u bench.py" \
 "300 bench_es python3 -u bench.py --workload entry_search" \
 "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/product_filter -o run -- python3 bench.py --no-cpu-baseline --no-e2e --workload product_filter --steps 5"
