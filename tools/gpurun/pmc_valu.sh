#!/bin/bash
# VALU issue counters of the fold (one PMC pass, SQ + GRBM blocks only), plus the counter list.
# Run on the GPU box from the repo root: gpurun -- tools/gpurun/pmc_valu.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -s KILL 60 rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1 || true
EXTRA=""
for c in SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32; do
  if grep -q "$c" gpurun_out/prof/counters.txt; then EXTRA="$EXTRA $c"; fi
done
echo "extra counters:$EXTRA"
exec tools/gpurun/steps.sh \
  "200 pmc_valu rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY$EXTRA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc_valu -o run -- python3 bench.py --no-cpu-baseline --no-e2e --no-extras --steps 1 --warmup 0 --verify 0"
