#!/bin/bash
# final round-4 profiles: the fold's VALU PMC pass, kernel stats + PMC traffic passes, order bench line
export TMPDIR=/tmp
tools/gpu_steps.sh "240 bench_order python3 -u bench.py --workload order --no-cpu-baseline" && \
bash tools/pmc_valu.sh && bash tools/profile_r04.sh
