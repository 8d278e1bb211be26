#!/bin/bash
export TMPDIR=/tmp
P=gpurun_out/prof
B="python3 bench.py --no-cpu-baseline --no-e2e --workload order --steps 1 --warmup 0 --verify 0"
exec tools/gpurun/steps.sh \
  "240 pmck2_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmck2_order_fetch -o run -- $B" \
  "240 pmck2_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmck2_order_write -o run -- $B" \
  "240 pmck0_fetch DDSHE_ORDER_KEYS2=0 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmck0_order_fetch -o run -- $B" \
  "240 pmck0_write DDSHE_ORDER_KEYS2=0 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmck0_order_write -o run -- $B"
