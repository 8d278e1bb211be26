#!/bin/bash
# OrderLS scatter A/B (same box): A = committed build, B = 8 ballots on full tiles of a pass without the
# validity bucket, C = 3072-row tiles (kRsItems 12). Order tests on B and C, then the order line and the skew
# probe per build, twice.
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
exec tools/gpurun/steps.sh \
  "300 st_B env DDSHE_LIB=$L/libddshe_b8.so $T" \
  "300 st_C env DDSHE_LIB=$L/libddshe_i12.so $T" \
  "200 sb_Aa env DDSHE_LIB=$L/libddshe_head.so $B" "200 sb_Ba env DDSHE_LIB=$L/libddshe_b8.so $B" "200 sb_Ca env DDSHE_LIB=$L/libddshe_i12.so $B" \
  "200 sb_Ab env DDSHE_LIB=$L/libddshe_head.so $B" "200 sb_Bb env DDSHE_LIB=$L/libddshe_b8.so $B" "200 sb_Cb env DDSHE_LIB=$L/libddshe_i12.so $B" \
  "200 sp_A env DDSHE_LIB=$L/libddshe_head.so $P" "200 sp_B env DDSHE_LIB=$L/libddshe_b8.so $P" "200 sp_C env DDSHE_LIB=$L/libddshe_i12.so $P"
