#!/bin/bash
# strong-split share A/B: level-1 group caps (tools/strong_split_probe.py), one box
cd "$(dirname "$0")/../.." || exit 1
for g in 0 16384 8192 4096 0; do
  DDSHE_PARTIAL_GROUPS=$g timeout -k 5 120 python3 tools/strong_split_probe.py || exit 1
done
