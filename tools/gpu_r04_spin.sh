#!/bin/bash
# fold finalize: spin on the root's completion word vs hipStreamSynchronize (DDSHE_FOLD_SPIN=0): parity
# tests, then the config-1 latency (fold_probe) both ways, twice
tools/gpu_steps.sh \
 "400 tests python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_columns.py tests/test_gpu_tree_modes.py tests/test_gpu_concurrency.py -x -q --timeout 200 --timeout-method thread" \
 "120 spin_a python3 tools/fold_probe.py paillier1024_seed1 10000 200" \
 "120 sync_a env DDSHE_FOLD_SPIN=0 python3 tools/fold_probe.py paillier1024_seed1 10000 200" \
 "120 spin_b python3 tools/fold_probe.py paillier1024_seed1 10000 200" \
 "120 sync_b env DDSHE_FOLD_SPIN=0 python3 tools/fold_probe.py paillier1024_seed1 10000 200" \
 "120 spin_1k python3 tools/fold_probe.py paillier1024_seed1 1000 200" \
 "120 sync_1k env DDSHE_FOLD_SPIN=0 python3 tools/fold_probe.py paillier1024_seed1 1000 200"
