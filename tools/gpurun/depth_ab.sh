#!/bin/bash
# k_fold<148,4,28,QP> row-chain A/B (tools/abtest/make_depth_variant.py, tools/abtest/ab_fold.sh with OLD=HEAD):
# the committed build (2 blocks ahead, buffers rotated by register moves) against the working tree (ring of 3
# block buffers, loop unrolled by 3), depth 3 unrolled by 4, and the committed build again; outputs must agree.
export TMPDIR=/tmp
export AB_NAME0=head AB_NAME1=ring3 AB_NAME2=d3u AB_NAME3=head_again
tools/gpurun/steps.sh \
  "200 dab1 tools/abtest/ab_fold 10000000 9" \
  "200 dab2 tools/abtest/ab_fold 10000000 9"
