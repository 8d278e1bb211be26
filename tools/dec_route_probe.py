#!/usr/bin/env python3
"""Config-1 String[] route probe (tool, not product): median wall time of dds_sum_all_dec over 10k
BigInteger.toString rows of the 1024-bit key (run under rocprofv3 --kernel-trace / --hip-trace to see
where a call's time goes). Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402


def main(reps=30, n=10000):
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    k = {a: int(b, 16) for a, b in keys["paillier1024_seed1"].items()}
    eng = ddshe.Engine(0)
    col = eng.column(k["nsquare"], n)
    col.fill_paillier_synth(k["n"], k["g"], 1, 0, n, 64)
    rows = [str(x) for x in col.read(0, n)]
    want = col.fold()
    arr = (C.c_char_p * n)(*[r.encode() for r in rows])
    cap = 4096
    obuf, olen, modb = C.create_string_buffer(cap), C.c_size_t(), str(k["nsquare"]).encode()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        st = ddshe._lib.dds_sum_all_dec(eng._h, arr, n, modb, obuf, cap, C.byref(olen))
        ts.append(time.perf_counter() - t)
        assert st == 0 and int(obuf.value.decode()) == want
    ts.sort()
    print(json.dumps({"rows": n, "chars": sum(map(len, rows)), "median_ms": ts[len(ts) // 2] * 1e3,
                      "min_ms": ts[0] * 1e3}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
