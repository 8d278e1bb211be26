#!/bin/bash
# fold A/B: round-1 kernel, HEAD kernel, and both with loop heads aligned to 64 B (-falign-loops=64)
export AB_NAME0=r01 AB_NAME1=head_r01loop AB_NAME2=head_r01loop_align64 AB_NAME3=r01_align64
tools/gpurun/steps.sh \
 "120 abfold_align1 ./tools/abtest/ab_fold 10000000 9" \
 "120 abfold_align2 ./tools/abtest/ab_fold 10000000 9"
