#!/bin/bash
# k_str_any zero-halfword fast path (in-tree build, 4 loads per thread) against the same loads without it
# (tools/abtest/libs/libddshe_fp4.so), one box: string-table tests on the in-tree build, the entry_search
# line per build (A B A B), a trace of the in-tree build.
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload entry_search --no-cpu-baseline --steps 20"
exec tools/gpurun/steps.sh \
  "300 sw_t python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_strtab.py tests/test_gpu_strscan.py tests/test_gpu_mutations.py tests/test_gpu_routes.py" \
  "300 sw_1a env DDSHE_LIB=$L/libddshe_fp4.so $B" "300 sw_1b $B" \
  "300 sw_2a env DDSHE_LIB=$L/libddshe_fp4.so $B" "300 sw_2b $B" \
  "300 sw_k rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/esw -o run -- $B"
