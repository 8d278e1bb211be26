#!/bin/bash
# string-table scan before/after writes (plain, then under a kernel trace), then the round-4 profiles
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
tools/gpu_steps.sh \
 "200 strtab_probe python3 -u tools/strtab_probe.py 2000000" \
 "240 strtab_probe_trace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/strtab_probe -o run -- python3 -u tools/strtab_probe.py 2000000" && \
 bash tools/profile_r04.sh
