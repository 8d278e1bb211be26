#!/bin/bash
# Round-6 HBM-traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs, one bench step each) of sum,
# product_filter, entry_search, encrypt_sum and order on the round-6 build -> tools/pmc_summary.py ->
# profiles/r06_pmc.json; first, k_str_any with plain (temporal) fingerprint loads
# (tools/abtest/libs/libddshe_swar4t.so) against the in-tree non-temporal ones (A B A B).
export TMPDIR=/tmp
P=gpurun_out/prof6
B="python3 bench.py --no-cpu-baseline --no-e2e"
E="python3 -u bench.py --workload entry_search --no-cpu-baseline --steps 20"
L=tools/abtest/libs
S=()
for w in sum:--no-extras pf:"--workload product_filter" es:"--workload entry_search" order:"--workload order" enc:"--workload encrypt_sum"; do
  t=${w%%:*}; a=${w#*:}
  for c in FETCH_SIZE:fetch WRITE_SIZE:write; do
    S+=("300 pmc_${t}_${c#*:} rocprofv3 --pmc ${c%%:*} --output-format csv -d $P/pmc_${t}_${c#*:} -o run -- $B $a --steps 1 --warmup 0 --verify 0")
  done
done
exec tools/gpurun/steps.sh "300 tl_1a env DDSHE_LIB=$L/libddshe_swar4t.so $E" "300 tl_1b $E" \
  "300 tl_2a env DDSHE_LIB=$L/libddshe_swar4t.so $E" "300 tl_2b $E" "${S[@]}"
