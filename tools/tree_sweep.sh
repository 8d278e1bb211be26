#!/bin/bash
# tail sweeps (tools/tree_ab.py, each variant in its own process): launch plan of the reduction tree
cd /root/repo
for v in "DDSHE_TREE_MID=0" "DDSHE_TREE_MID=256" "DDSHE_TREE_MID=0" "DDSHE_TREE_MID=256" "DDSHE_TREE_MID=128"; do
  echo "== $v"
  env $v timeout -k 5 120 python -u tools/tree_ab.py || exit 1
done
