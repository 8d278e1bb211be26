#!/bin/bash
# k_msd_local_blk block shapes (threads x rows per lane; grid): 256 x 16 (768 blocks, in-tree),
# 512 x 8 (512), 1024 x 4 (256) from tools/abtest/libs/libddshe_blk{512,1024}.so, same box: order tests per
# build, then the order line (twice) and the skew probe per build, a trace per build.
export TMPDIR=/tmp
L=tools/abtest/libs
B="python3 -u bench.py --workload order --steps 20 --no-cpu-baseline"
P="python3 -u tools/order_skew_probe.py"
T="python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_order.py"
S=()
for v in 256 512 1024; do
  E=""; [ $v != 256 ] && E="env DDSHE_LIB=$L/libddshe_blk$v.so"
  S+=("300 mb_t$v $E $T")
done
for rep in a b; do
  for v in 256 512 1024; do
    E=""; [ $v != 256 ] && E="env DDSHE_LIB=$L/libddshe_blk$v.so"
    S+=("200 mb_b$v$rep $E $B")
  done
done
for v in 256 512 1024; do
  E=""; [ $v != 256 ] && E="env DDSHE_LIB=$L/libddshe_blk$v.so"
  S+=("200 mb_p$v $E $P" "200 mb_k$v $E rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6/order_mb$v -o run -- $B --steps 10")
done
exec tools/gpurun/steps.sh "${S[@]}"
