#!/bin/bash
# OrderLS A/B on one box: for each "name:VAR=VAL ..." argument, the order bench line (verified against
# numpy) and a rocprofv3 kernel trace (per-dispatch rows + stats) under those DDSHE_ORDER_* settings.
# usage (repo root, on the GPU box): tools/gpurun/order_ab.sh "base:DDSHE_ORDER_XCD=0" "xcd:DDSHE_ORDER_XCD=1"
export TMPDIR=/tmp
P=gpurun_out/prof
specs=()
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  specs+=("240 bench_$name $envs python3 -u bench.py --workload order --no-cpu-baseline --steps 10")
  specs+=("240 ks_$name $envs rocprofv3 --kernel-trace --stats --output-format csv -d $P/order_$name -o run -- python3 bench.py --workload order --no-cpu-baseline --steps 5 --verify 0")
done
exec tools/gpurun/steps.sh "${specs[@]}"
