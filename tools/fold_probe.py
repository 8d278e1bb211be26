#!/usr/bin/env python3
"""One fold size, repeated (tool, not product): run under rocprofv3 --kernel-trace to see the launch
sequence of a fold, e.g. config 1 (10k rows, 1024-bit key):
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ft -o run -- python3 tools/fold_probe.py paillier1024_seed1 10000 20
Prints the median wall time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]

import ddshe  # noqa: E402


def main(name, n, reps):
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    k = {a: int(b, 16) for a, b in keys[name].items()}
    eng = ddshe.Engine(0)
    col = eng.column(k["nsquare"], n)
    col.fill_paillier_synth(k["n"], k["g"], 3, 0, n, 64)
    col.fold()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        col.fold()
        ts.append(time.perf_counter() - t)
    ts.sort()
    print(json.dumps({"key": name, "rows": n, "median_ms": ts[len(ts) // 2] * 1e3}))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 20)
