#!/bin/bash
# The GPU suite, smoke and a short headline bench line (no extras) on one box.
cd "$(dirname "$0")/../.." || exit 1
tools/gpurun/steps.sh \
  "600 tests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "120 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "300 bench python3 -u bench.py --steps 5 --no-extras"
