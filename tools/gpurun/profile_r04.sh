#!/bin/bash
# Round-4 profiles (run on the GPU box from the repo root: gpurun -- tools/gpurun/profile_r04.sh):
#   * rocprofv3 kernel stats of the headline with ONE fold size (10M rows: no strong-split share, no CPU
#     prefix fold), so the k_fold row's Average is the headline launch;
#   * kernel stats of the order, product_filter (Search route) and entry_search (string table) workloads;
#   * PMC HBM-traffic passes (one counter per pass) of the headline, order and product_filter.
# Outputs under gpurun_out/prof/<name>/ (CSV); the summaries to be judged are copied into profiles/.
export TMPDIR=/tmp
P=gpurun_out/prof
B="python3 bench.py --no-cpu-baseline --no-e2e"
exec tools/gpurun/steps.sh \
  "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d $P/sum -o run -- $B --no-extras --verify 0 --steps 5" \
  "300 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d $P/order -o run -- $B --workload order --steps 5" \
  "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/product_filter -o run -- $B --workload product_filter --steps 5" \
  "300 ks_es rocprofv3 --kernel-trace --stats --output-format csv -d $P/entry_search -o run -- $B --workload entry_search --steps 5" \
  "240 pmc_sum_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_sum_fetch -o run -- $B --no-extras --steps 1 --warmup 0 --verify 0" \
  "240 pmc_sum_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_sum_write -o run -- $B --no-extras --steps 1 --warmup 0 --verify 0" \
  "240 pmc_order_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_order_fetch -o run -- $B --workload order --steps 1 --warmup 0 --verify 0" \
  "240 pmc_order_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_order_write -o run -- $B --workload order --steps 1 --warmup 0 --verify 0" \
  "240 pmc_pf_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_pf_fetch -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0" \
  "240 pmc_pf_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_pf_write -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0"
