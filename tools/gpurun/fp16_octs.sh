#!/bin/bash
# k_str_any with 2 / 4 / 8 16-byte fingerprint loads per thread (tools/abtest/libs/libddshe_fp{2,4,8}.so),
# one box: the string-table tests on the 4-load build, the entry_search line per build (twice), traces.
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload entry_search --no-cpu-baseline --steps 20"
exec tools/gpurun/steps.sh \
  "300 oc_t env DDSHE_LIB=$L/libddshe_fp4.so python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_strtab.py tests/test_gpu_strscan.py tests/test_gpu_mutations.py" \
  "300 oc_2a env DDSHE_LIB=$L/libddshe_fp2.so $B" "300 oc_4a env DDSHE_LIB=$L/libddshe_fp4.so $B" "300 oc_8a env DDSHE_LIB=$L/libddshe_fp8.so $B" \
  "300 oc_2b env DDSHE_LIB=$L/libddshe_fp2.so $B" "300 oc_4b env DDSHE_LIB=$L/libddshe_fp4.so $B" "300 oc_8b env DDSHE_LIB=$L/libddshe_fp8.so $B" \
  "300 oc_k4 env DDSHE_LIB=$L/libddshe_fp4.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/es4 -o run -- $B" \
  "300 oc_k8 env DDSHE_LIB=$L/libddshe_fp8.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/es8 -o run -- $B"
