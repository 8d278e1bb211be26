#!/bin/bash
# k_msd_local over lists of the multi-key buckets (k_msd_list, atomic-free: buckets of <= 512 rows by a
# 4-wave-per-SIMD launch with the memory rounds, larger ones one per 256-thread block partitioning from
# registers, k_msd_local_blk; B: in-tree
# build) against the bucket ranges per wave (A: tools/abtest/libs/libddshe_swar4.so), same box: order
# tests on B, then the skew probe and the order line per build (A B, three times), a trace of B.
# (Earlier runs, round 6: one list, one atomic counter, 2,048 waves: no faster than A; one atomic-free list
# with the register partition up to 3,072 rows: bench call 0.270 -> 0.262 ms but uniform 54-bit keys
# 0.67 -> 1.0 ms at one wave per SIMD; two lists, one wave per large bucket from registers up to 3,072
# rows: bench call -7 us, uniform +1 %, but a column with 4-key buckets of > 3,072 rows no faster.)
# (First run, round 6: one atomic counter for the list and 2,048 waves, list + register partition up to
# 2,048 rows / list + memory rounds: no faster than A, the list kernel 7.4 us.)
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
exec tools/gpurun/steps.sh \
  "300 ml_tB $T" \
  "200 ml_pAa env DDSHE_LIB=$L/libddshe_swar4.so $P" "200 ml_pBa $P" \
  "200 ml_bAa env DDSHE_LIB=$L/libddshe_swar4.so $B" "200 ml_bBa $B" \
  "200 ml_pAb env DDSHE_LIB=$L/libddshe_swar4.so $P" "200 ml_pBb $P" \
  "200 ml_bAb env DDSHE_LIB=$L/libddshe_swar4.so $B" "200 ml_bBb $B" \
  "200 ml_bAc env DDSHE_LIB=$L/libddshe_swar4.so $B" "200 ml_bBc $B" \
  "200 ml_ksB rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/order_mlB -o run -- $B --steps 10"
