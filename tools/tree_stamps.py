#!/usr/bin/env python3
"""Where a reduction-tree level's time goes (tool, not product; VERDICT r02 "next" 3).

Runs resident-column folds with DDSHE_TREE_STAMPS set (ddshe_tree.hip: thread 0 of the first and last
block of every k_tree launch records s_memtime after each barrier of its Montgomery product) and prints
one JSON line: per tree class S, the median shader cycles of each phase of a level launch (leaf load,
zeroing, T = a*b, split, m = d*n', split, V = T + m*N, carry + splits, hand-off store), their sum, the
launch's wall span from s_memrealtime (100 MHz), and the implied clock. Run on the GPU box:
    python tools/tree_stamps.py
"""
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
PATH = os.path.join(tempfile.gettempdir(), "ddshe_tree_stamps.txt")
os.environ["DDSHE_TREE_STAMPS"] = PATH

import ddshe  # noqa: E402

PHASES = ["load", "T=a*b", "split_T", "m=d*n'", "split_m", "V=T+m*N", "carry+split+norm", "handoff"]


def main():
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    eng = ddshe.Engine(0)
    out = {}
    for name, n in (("paillier2048_committed", 1024), ("paillier2048_committed", 10_000_000),
                    ("paillier1024_seed1", 10000), ("paillier1024_seed1", 1024)):
        k = {a: int(b, 16) for a, b in keys[name].items()}
        col = eng.column(k["nsquare"], n)
        col.fill_paillier_synth(k["n"], k["g"], 3, 0, n, 64)
        col.fold()
        if os.path.exists(PATH):
            os.remove(PATH)
        walls = []
        for _ in range(5):
            t = time.perf_counter()
            col.fold()
            walls.append(time.perf_counter() - t)
        col.close()
        rows = [ln.split() for ln in open(PATH)]
        per = {}
        for r in rows:
            S, nleaves, blocks, which = int(r[0]), int(r[1]), int(r[2]), r[3]
            rt0, rt1, nm = int(r[5]), int(r[6]), int(r[7])
            deltas = [int(x) for x in r[8:]]
            key = f"S{S}_{which}_{'root' if blocks == 1 else 'level'}"
            per.setdefault(key, []).append((deltas, (rt1 - rt0) / 100.0))  # realtime: 100 MHz -> us
        summ = {}
        for key, lst in per.items():
            ph = {}
            m = min(len(d) for d, _ in lst)
            for i in range(m):
                ph[PHASES[i] if i < len(PHASES) else f"p{i}"] = statistics.median(d[i] for d, _ in lst)
            cyc = sum(ph.values())
            span = statistics.median(w for _, w in lst)
            summ[key] = {"launches": len(lst), "phase_cycles": ph, "cycles": cyc, "span_us": span,
                         "clock_GHz": cyc / span / 1e3 if span else None}
        walls.sort()
        out[f"{name}_{n}"] = {"fold_ms_median": walls[2] * 1e3, "launch_phases": summ}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
