#!/bin/bash
# Build tools/abtest/ab_fold from up to four header directories (A/B tool, not product):
#   ./ab_dirs.sh <dir0> <dir1> [dir2] [dir3]   (each holding ddshe_device.hpp / ddshe_fold.hpp / ddshe_launch.hpp)
# then on the GPU box: AB_NAME0=.. AB_NAME1=.. ./tools/abtest/ab_fold 10000000 9
set -e
cd "$(dirname "$0")"
HIPCC=/opt/rocm/bin/hipcc
FL="--offload-arch=gfx950 -O3 -std=c++17"
mkdir -p abobj
objs=""
i=0
for d in "$@"; do
  $HIPCC $FL -I"$d" -DKNAME=k_ab$i -c ab_fold.hip -o abobj/ab$i.o &
  objs="$objs abobj/ab$i.o"; i=$((i+1))
done
while [ $i -lt 4 ]; do  # unused slots: copies of the first build
  $HIPCC $FL -I"$1" -DKNAME=k_ab$i -c ab_fold.hip -o abobj/ab$i.o &
  objs="$objs abobj/ab$i.o"; i=$((i+1))
done
$HIPCC $FL -c ab_fold_main.cpp -o abobj/main.o &
wait
$HIPCC --offload-arch=gfx950 abobj/main.o $objs -o ab_fold
echo built tools/abtest/ab_fold
