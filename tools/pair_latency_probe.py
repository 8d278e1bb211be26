#!/usr/bin/env python3
"""One /Sum caller, repeated (tool, not product): median latency of dds_pair_modmul_dec under the
committed key's n^2, through the Python binding. Prints one JSON line."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402

keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
m = int(keys["paillier2048_committed"]["nsquare"], 16)
rng = random.Random(5)
a, b = rng.randrange(m), rng.randrange(m)
eng = ddshe.Engine(0)
want = str(a * b % m)
ms = str(m)
for _ in range(20):
    assert eng.pair_modmul_dec(str(a), str(b), ms) == want
ts = []
sa, sb = str(a), str(b)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 500):
    t = time.perf_counter()
    r = eng.pair_modmul_dec(sa, sb, ms)
    ts.append(time.perf_counter() - t)
assert r == want
ts.sort()
print(json.dumps({"calls": len(ts), "median_ms": ts[len(ts) // 2] * 1e3, "p99_ms": ts[int(len(ts) * 0.99)] * 1e3}))
eng.close()
