#!/bin/bash
# tail sweeps: DDSHE_TREE_SWITCH and in-kernel levels (each variant in its own process)
cd /root/repo
for v in "DDSHE_TREE_SWITCH=1024" "DDSHE_TREE_SWITCH=2048" "DDSHE_TREE_SWITCH=4096" "DDSHE_TREE_SWITCH=512" "DDSHE_TREE_LEVELS=2 DDSHE_TREE_FENCE=2" "DDSHE_TREE_LEVELS=0 DDSHE_TREE_FENCE=2"; do
  echo "== $v"
  env $v timeout -k 5 120 python -u tools/tree_ab.py || exit 1
done
