#!/usr/bin/env python3
"""Fold latency probe (tool, not product): median wall time of resident-column folds at several row
counts, to A/B the reduction tree (DDSHE_TREE=1, default) against round 1's per-level launches
(DDSHE_TREE=0) in separate processes. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]

import ddshe  # noqa: E402


def main():
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    out = {"tree": os.environ.get("DDSHE_TREE", "1"), "direct": os.environ.get("DDSHE_TREE_DIRECT", "8192")}
    eng = ddshe.Engine(0)
    for name, sizes in (("paillier1024_seed1", [2, 100, 1000, 10000]),
                        ("paillier2048_committed", [2, 1000, 10000, 100000, 1000000, 10000000])):
        k = {a: int(b, 16) for a, b in keys[name].items()}
        col = eng.column(k["nsquare"], max(sizes))
        col.fill_paillier_synth(k["n"], k["g"], 3, 0, max(sizes), 64)
        res = {}
        for n in sizes:
            col.fold(0, n)
            reps = 30 if n <= 100000 else 5
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                col.fold(0, n)
                ts.append(time.perf_counter() - t)
            ts.sort()
            res[n] = round(ts[len(ts) // 2] * 1e3, 4)
        out[name] = res
        col.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
