#!/usr/bin/env python3
"""Debug probe (tool, not product): the golden MultAll route cases, engine vs expected, printed."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402
from ddshe import routes  # noqa: E402


def main():
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
    eng = ddshe.Engine(0)
    rv = v["routes"]
    rows = rv["rows"]
    for c in rv["cases"]:
        if c["route"] != "MultAll":
            continue
        ops = [r[c["position"]] for r in routes._dedup(rows) if len(r) - 1 > c["position"]]
        got = routes.mult_all(eng, rows, c["position"], c["n"])
        n = int(c["n"])
        want = 1
        for x in ops:
            want = want * int(x) % n
        print("k", len(ops), "bits", n.bit_length(), "ok", got == c["result"], "py", str(want) == c["result"], flush=True)
        for k in range(2, len(ops) + 1):
            w = 1
            for x in ops[:k]:
                w = w * int(x) % n
            g = eng.mult_all_dec([str(x) for x in ops[:k]], str(n))
            b = eng.modmul_fold(n, [int(x) % n for x in ops[:k]])
            print("  prefix", k, g == str(w), b == w, flush=True)


if __name__ == "__main__":
    main()
