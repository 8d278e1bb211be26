#!/bin/bash
# Build tools/abtest/ab_fold1: the production k_fold1<74,28,false> (MultAll's one-bignum-per-lane fold) of the
# committed HEAD (before the working tree's edits) and of the working tree, twice each, interleaved in one
# process (AB_NAME0..3 label them). Run here (needs git); the binary travels with the snapshot.
set -e
cd "$(dirname "$0")"
CSRC=../../dependable-data-storage-csd2017_amd/csrc
HIPCC=/opt/rocm/bin/hipcc
FL="--offload-arch=gfx950 -O3 -std=c++17"
mkdir -p committed abobj1
for f in ddshe_device.hpp ddshe_fold.hpp ddshe_launch.hpp; do
  git show "HEAD:dependable-data-storage-csd2017_amd/csrc/$f" > committed/$f
done
$HIPCC $FL -Icommitted -DKNAME=k_ab0 -c ab_fold1.hip -o abobj1/ab0.o &
$HIPCC $FL -I$CSRC -DKNAME=k_ab1 -c ab_fold1.hip -o abobj1/ab1.o &
$HIPCC $FL -Icommitted -DKNAME=k_ab2 -c ab_fold1.hip -o abobj1/ab2.o &
$HIPCC $FL -I$CSRC -DKNAME=k_ab3 -c ab_fold1.hip -o abobj1/ab3.o &
$HIPCC $FL -DAB_FOLD1 -c ab_fold_main.cpp -o abobj1/main.o &
wait
$HIPCC --offload-arch=gfx950 abobj1/main.o abobj1/ab0.o abobj1/ab1.o abobj1/ab2.o abobj1/ab3.o -o ab_fold1
echo built tools/abtest/ab_fold1
