#!/bin/bash
# The N > 1 bench flow rehearsed on one GPU through bench.py's own launcher (DDSHE_DIST_BACKEND=gloo: every
# rank on the box's GPU, partials gathered through host memory): each workload at 2 ranks (verified by the
# combined result, or by each rank checking its own shard and a min over ranks), the headline at 4 ranks,
# and the headline at 2 ranks with --no-extras (verification must not depend on the extras).
export TMPDIR=/tmp
G="env DDSHE_DIST_BACKEND=gloo python3 -u bench.py --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 dr_sum4 $G --gpus 4 --steps 3 --warmup 1" \
  "200 dr_sum2_noextras $G --gpus 2 --steps 3 --warmup 1 --no-extras" \
  "300 dr_pf2 $G --gpus 2 --workload product_filter --rows 2000000 --steps 3 --warmup 1" \
  "300 dr_enc2 $G --gpus 2 --workload encrypt_sum --rows 100000 --steps 1 --warmup 1" \
  "200 dr_order2 $G --gpus 2 --workload order --steps 3 --warmup 1" \
  "200 dr_order2_noextras $G --gpus 2 --workload order --steps 3 --warmup 1 --no-extras" \
  "300 dr_es2 $G --gpus 2 --workload entry_search --rows 2000000 --steps 3 --warmup 1"
