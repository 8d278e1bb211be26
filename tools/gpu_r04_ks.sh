#!/bin/bash
# Final kernel stats with the bench line of the SAME command (so the headline avg_launch_ms and the profile's
# k_fold Average come from one run): single-size sum, and the product_filter workload
export TMPDIR=/tmp
P=gpurun_out/prof
B="python3 bench.py --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
 "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d $P/sum -o run -- $B --no-extras --verify 0 --steps 5" \
 "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/product_filter -o run -- $B --workload product_filter --steps 5"
