#!/bin/bash
# k_str_any grid-stride A/B (DDSHE_STR_GS=1: 2,048 blocks walking the octets, next chunk's loads in flight)
# against the one-chunk-per-block launch (0), same box: string tests with it on, the entry_search line per
# build twice, a kernel trace per build.
export TMPDIR=/tmp
B="python3 -u bench.py --workload entry_search --steps 20 --no-cpu-baseline"
exec tools/gpurun/steps.sh \
  "300 gt_B env DDSHE_STR_GS=1 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_strtab.py tests/test_gpu_mutations.py" \
  "200 ge_Aa env DDSHE_STR_GS=0 $B" "200 ge_Ba env DDSHE_STR_GS=1 $B" \
  "200 ge_Ab env DDSHE_STR_GS=0 $B" "200 ge_Bb env DDSHE_STR_GS=1 $B" \
  "200 gk_A env DDSHE_STR_GS=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gs/A -o run -- $B --steps 10" \
  "200 gk_B env DDSHE_STR_GS=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gs/B -o run -- $B --steps 10"
