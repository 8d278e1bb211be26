#!/bin/bash
# In-block level-1 tree A/B on one box: its parity tests, then the strong-split
# share probe and the headline line with DDSHE_FOLD_INBLOCK=0 (tail launches) and 1, alternating.
export TMPDIR=/tmp
B="python3 -u bench.py --no-cpu-baseline --no-e2e --no-extras --steps 20"
exec tools/gpurun/steps.sh \
  "300 ib_tests python -u -m pytest tests/test_gpu_inblock.py tests/test_gpu_rccl.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread" \
  "120 ib_probe0a env DDSHE_FOLD_INBLOCK=0 python3 tools/strong_split_probe.py" \
  "120 ib_probe1a env DDSHE_FOLD_INBLOCK=1 python3 tools/strong_split_probe.py" \
  "120 ib_probe0b env DDSHE_FOLD_INBLOCK=0 python3 tools/strong_split_probe.py" \
  "120 ib_probe1b env DDSHE_FOLD_INBLOCK=1 python3 tools/strong_split_probe.py" \
  "150 ib_sum0a env DDSHE_FOLD_INBLOCK=0 $B" \
  "150 ib_sum1a env DDSHE_FOLD_INBLOCK=1 $B" \
  "150 ib_sum0b env DDSHE_FOLD_INBLOCK=0 $B" \
  "150 ib_sum1b env DDSHE_FOLD_INBLOCK=1 $B"
