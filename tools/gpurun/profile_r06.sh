#!/bin/bash
# Round-6 roofline evidence, on one box (gpurun -- tools/gpurun/profile_r06.sh):
#   * the v_mad_u64_u32 issue-rate microbenchmark (tools/microbench/ubench);
#   * rocprofv3 kernel traces + stats of the headline (sum), product_filter (config 3) and encrypt_sum
#     (config 4) with their bench lines in the same run's log (the HIP-event launch time of a line and
#     the trace's dispatches of the same kernel come from one process);
#   * one SQ + GRBM PMC pass each for k_fold (sum), k_fold1 (product_filter) and k_modexp_ladder
#     (encrypt_sum): VALU / INT64 instruction counts, wave cycles, waits, and the clock.
# Summaries: tools/dispatch_stats.py, tools/pmc_valu_summary.py -> profiles/r06_*.
export TMPDIR=/tmp
P=gpurun_out/prof6
B="python3 bench.py --no-cpu-baseline --no-e2e"
V="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE"
KS=(
  "300 order_keys2_0 env DDSHE_ORDER_KEYS2=0 python -u -m pytest tests/test_gpu_order.py -x -q --timeout 200 --timeout-method thread"
  "120 ubench tools/microbench/ubench"
  "300 ks_sum rocprofv3 --kernel-trace --stats --output-format csv -d $P/sum -o run -- $B --no-extras --steps 10"
  "300 ks_pf rocprofv3 --kernel-trace --stats --output-format csv -d $P/pf -o run -- $B --workload product_filter --steps 10"
  "400 ks_enc rocprofv3 --kernel-trace --stats --output-format csv -d $P/enc -o run -- $B --workload encrypt_sum --steps 2 --warmup 1"
)
PMC=(
  "240 pmc_valu_sum rocprofv3 --pmc $V --output-format csv -d $P/pmc_valu_sum -o run -- $B --no-extras --steps 1 --warmup 0 --verify 0"
  "240 pmc_valu_pf rocprofv3 --pmc $V --output-format csv -d $P/pmc_valu_pf -o run -- $B --workload product_filter --steps 1 --warmup 0 --verify 0"
  "300 pmc_valu_enc rocprofv3 --pmc $V --output-format csv -d $P/pmc_valu_enc -o run -- $B --workload encrypt_sum --steps 1 --warmup 0 --verify 0"
)
case "${PART:-all}" in
  ks) exec tools/gpurun/steps.sh "${KS[@]}" ;;
  pmc) exec tools/gpurun/steps.sh "${PMC[@]}" ;;
  *) exec tools/gpurun/steps.sh "${KS[@]}" "${PMC[@]}" ;;
esac
