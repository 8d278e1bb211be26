#!/bin/bash
# Binary host-boundary fold (dds_paillier_sum / fold_buffer) pipelined in pieces vs ingest-then-fold, same
# box: GPU tests of the paths first, then the default bench's end_to_end line under DDSHE_INGEST_PIECES.
cd "$(dirname "$0")/../.." || exit 1
tools/gpurun/steps.sh \
  "300 t python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_concurrency.py tests/test_gpu_parity.py" \
  "300 e1 python3 -u bench.py --steps 3 --no-extras --no-cpu-baseline" \
  "300 e0 env DDSHE_INGEST_PIECES=1 python3 -u bench.py --steps 3 --no-extras --no-cpu-baseline" \
  "300 e8 env DDSHE_INGEST_PIECES=8 python3 -u bench.py --steps 3 --no-extras --no-cpu-baseline"
