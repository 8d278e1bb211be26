#!/bin/bash
# Build tools/abtest/ab_fold: the production k_fold<148,4,28,QP> of an older commit (default: the end of
# round 1, cddbb2f) and of the working tree, timed interleaved in one process (run it on the GPU box:
# AB_NAME0=... ./tools/abtest/ab_fold 10000000 9). Extra builds: AB_V2 / AB_V3 = "-I<dir> [-D...]".
# Run here (needs git): the binary travels to the box with the snapshot.
set -e
cd "$(dirname "$0")"
OLD=${OLD:-cddbb2f}
CSRC=../../dependable-data-storage-csd2017_amd/csrc
HIPCC=/opt/rocm/bin/hipcc
FL="--offload-arch=gfx950 -O3 -std=c++17"
mkdir -p old abobj
for f in ddshe_device.hpp ddshe_fold.hpp ddshe_launch.hpp; do
  git show "$OLD:dependable-data-storage-csd2017_amd/csrc/$f" > old/$f
done
V2=${AB_V2:--I$CSRC}
V3=${AB_V3:--Iold}
$HIPCC $FL -Iold -DKNAME=k_ab0 -c ab_fold.hip -o abobj/ab0.o &
$HIPCC $FL -I$CSRC -DKNAME=k_ab1 -c ab_fold.hip -o abobj/ab1.o &
$HIPCC $FL $V2 -DKNAME=k_ab2 -c ab_fold.hip -o abobj/ab2.o &
$HIPCC $FL $V3 -DKNAME=k_ab3 -c ab_fold.hip -o abobj/ab3.o &
$HIPCC $FL -c ab_fold_main.cpp -o abobj/main.o &
wait
$HIPCC --offload-arch=gfx950 abobj/main.o abobj/ab0.o abobj/ab1.o abobj/ab2.o abobj/ab3.o -o ab_fold
echo built tools/abtest/ab_fold
