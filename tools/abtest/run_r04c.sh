#!/bin/bash
# fold A/B on one box, one process: round-1 kernel, HEAD (round-1 row loop restored), the round-3
# kernel (row-id loop for every fold), round-1 again
export AB_NAME0=r01 AB_NAME1=head_r04 AB_NAME2=r03_loop AB_NAME3=r01
tools/gpurun/steps.sh \
 "120 abfold_c1 ./tools/abtest/ab_fold 10000000 9" \
 "120 abfold_c2 ./tools/abtest/ab_fold 10000000 9"
