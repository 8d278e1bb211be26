#!/bin/bash
# Round-5 profiles (GPU box, repo root: gpurun -- tools/gpurun/profile_r05.sh):
#   * rocprofv3 kernel stats: the headline with ONE fold size (10M rows, --no-extras), order, product_filter
#     (Search route), encrypt_sum (config 4) and entry_search;
#   * PMC HBM-traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs) of sum, order, product_filter,
#     entry_search and encrypt_sum (the k_modexp_ladder traffic of config 4's roofline);
#   * the ladder's issue / wait counters (one SQ + GRBM pass) on encrypt_sum.
# Outputs under gpurun_out/prof/<name>/; tools/pmc_summary.py and tools/pmc_valu_summary.py make the
# profiles/ summaries.
export TMPDIR=/tmp
P=gpurun_out/prof
B="python3 bench.py --no-cpu-baseline --no-e2e"
# PART=ks: the kernel-stats runs only; PART=pmc: the PMC passes only (each fits one gpurun call)
KS=(
  "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d $P/sum -o run -- $B --no-extras --verify 0 --steps 5"
  "300 ks_order rocprofv3 --kernel-trace --stats --output-format csv -d $P/order -o run -- $B --workload order --steps 5"
  "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/product_filter -o run -- $B --workload product_filter --steps 5"
  "400 ks_enc rocprofv3 --kernel-trace --stats --output-format csv -d $P/encrypt_sum -o run -- $B --workload encrypt_sum --steps 1 --warmup 1"
  "300 ks_es rocprofv3 --kernel-trace --stats --output-format csv -d $P/entry_search -o run -- $B --workload entry_search --steps 5"
)
PMC=(
  "240 pmc_sum_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_sum_fetch -o run -- $B --no-extras --steps 1 --warmup 0 --verify 0"
  "240 pmc_sum_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_sum_write -o run -- $B --no-extras --steps 1 --warmup 0 --verify 0"
  "240 pmc_order_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_order_fetch -o run -- $B --workload order --steps 1 --warmup 0 --verify 0"
  "240 pmc_order_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_order_write -o run -- $B --workload order --steps 1 --warmup 0 --verify 0"
  "240 pmc_pf_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_pf_fetch -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0"
  "240 pmc_pf_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_pf_write -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0"
  "240 pmc_es_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_es_fetch -o run -- $B --workload entry_search --steps 1 --warmup 0 --verify 0"
  "240 pmc_es_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_es_write -o run -- $B --workload entry_search --steps 1 --warmup 0 --verify 0"
  "300 pmc_enc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_enc_fetch -o run -- $B --workload encrypt_sum --steps 1 --warmup 0 --verify 0"
  "300 pmc_enc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/pmc_enc_write -o run -- $B --workload encrypt_sum --steps 1 --warmup 0 --verify 0"
  "300 pmc_enc_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $P/pmc_enc_stall -o run -- $B --workload encrypt_sum --steps 1 --warmup 0 --verify 0"
)
case "${PART:-all}" in
  ks) exec tools/gpurun/steps.sh "${KS[@]}" ;;
  pmc) exec tools/gpurun/steps.sh "${PMC[@]}" ;;
  *) exec tools/gpurun/steps.sh "${KS[@]}" "${PMC[@]}" ;;
esac
