#!/bin/bash
# Encrypt ladder A/B on one box: the encrypt tests on the current build, then the
# config-4 line (1M rows, 3072-bit key, CRT halves) with the two-wave build (tools/abtest/libs/
# libddshe_occ2.so: -DDDSHE_LADDER_OCC2) and the current one, alternating, twice each.
export TMPDIR=/tmp
OCC2=tools/abtest/libs/libddshe_occ2.so
exec tools/gpurun/steps.sh \
  "300 lad_tests python -u -m pytest tests/test_gpu_encrypt.py -x -q --timeout 200 --timeout-method thread" \
  "200 lad_occ2_a env DDSHE_LIB=$OCC2 python -u bench.py --workload encrypt_sum --no-cpu-baseline --steps 2 --warmup 1" \
  "200 lad_occ3_a python -u bench.py --workload encrypt_sum --no-cpu-baseline --steps 2 --warmup 1" \
  "200 lad_occ2_b env DDSHE_LIB=$OCC2 python -u bench.py --workload encrypt_sum --no-cpu-baseline --steps 2 --warmup 1" \
  "200 lad_occ3_b python -u bench.py --workload encrypt_sum --no-cpu-baseline --steps 2 --warmup 1"
