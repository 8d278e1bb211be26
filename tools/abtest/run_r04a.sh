#!/bin/bash
# round-4 first GPU pass: fold A/B (round-1 vs HEAD kernel, one process), the new string-table,
# mutation and tree-mode tests, and the HEAD / round-1 headline bench lines back to back on one box
export AB_NAME0=r01 AB_NAME1=head AB_NAME2=head AB_NAME3=r01
tools/gpurun/steps.sh \
 "120 abfold1 ./tools/abtest/ab_fold 10000000 9" \
 "60 mfma_probe ./tools/microbench/mfma_i8_probe" \
 "500 tests_new python3 -u -m pytest tests/test_gpu_strtab.py tests/test_gpu_mutations.py tests/test_gpu_strscan.py tests/test_gpu_tree_modes.py tests/test_gpu_order.py -x -v --timeout 120 --timeout-method thread" \
 "240 bench_head python3 -u bench.py --no-cpu-baseline --no-e2e --no-extras --steps 20 --warmup 3" \
 "240 bench_r01 cd tools/abtest/r01tree && python3 -u bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3" \
 "120 abfold2 ./tools/abtest/ab_fold 10000000 9"
