#!/bin/bash
# rocprofv3 kernel statistics for every bench workload, then PMC HBM-traffic passes (one counter
# per pass) for the HBM-bound workloads. Run on the GPU box from the repo root:
#   gpurun -- tools/gpurun/profile_all.sh
# Outputs under gpurun_out/prof/<name>/ (CSV); copy the summaries to be judged into profiles/.
export TMPDIR=/tmp
P=gpurun_out/prof
B="python3 bench.py --no-cpu-baseline --no-e2e"
exec tools/gpurun/steps.sh \
  "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d $P/sum -o run -- $B --steps 5" \
  "300 ks_e2e rocprofv3 --kernel-trace --stats --output-format csv -d $P/e2e -o run -- python3 bench.py --no-cpu-baseline --no-extras --steps 1" \
  "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/product_filter -o run -- $B --workload product_filter --steps 5" \
  "400 ks_enc rocprofv3 --kernel-trace --stats --output-format csv -d $P/encrypt_sum -o run -- $B --workload encrypt_sum --steps 1 --warmup 1" \
  "300 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d $P/order -o run -- $B --workload order --steps 5" \
  "300 ks_es rocprofv3 --kernel-trace --stats --output-format csv -d $P/entry_search -o run -- $B --workload entry_search --steps 5" \
  "240 pmc_pf_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_pf_fetch -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0" \
  "240 pmc_pf_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_pf_write -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0" \
  "240 pmc_order_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_order_fetch -o run -- $B --workload order --steps 1 --warmup 0 --verify 0" \
  "240 pmc_order_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_order_write -o run -- $B --workload order --steps 1 --warmup 0 --verify 0" \
  "240 pmc_sum_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_sum_fetch -o run -- $B --steps 1 --warmup 0 --verify 0" \
  "240 pmc_sum_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_sum_write -o run -- $B --steps 1 --warmup 0 --verify 0"
