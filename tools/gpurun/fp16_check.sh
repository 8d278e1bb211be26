#!/bin/bash
# 16-bit element fingerprints (string scans): the string-table GPU tests, then the entry_search line
# against the previous build (DDSHE_LIB=tools/abtest/libs/libddshe_r06a.so, 32-bit fingerprints), and a
# kernel trace of the new build.
export TMPDIR=/tmp
OLD=tools/abtest/libs/libddshe_r06a.so
B="python3 -u bench.py --workload entry_search --no-cpu-baseline --steps 20"
exec tools/gpurun/steps.sh \
  "400 fp_t python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_strtab.py tests/test_gpu_strscan.py tests/test_gpu_mutations.py tests/test_gpu_routes.py" \
  "300 fp_old_a env DDSHE_LIB=$OLD $B" "300 fp_new_a $B" "300 fp_old_b env DDSHE_LIB=$OLD $B" "300 fp_new_b $B" \
  "300 fp_ks rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/es -o run -- $B"
