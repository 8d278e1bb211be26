#!/usr/bin/env python3
"""String[] route probe (tool, not product): median wall time of dds_sum_all_dec over
BigInteger.toString rows. Default: config 1 (10k rows of the 1024-bit key). `--big`: the end-to-end
shape of bench.py (1M rows of the committed 2048-bit key: 100k distinct rows tiled 10 times), the
String[] entry point beside the Arrow-style chars + offsets ingest of the same rows. Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402


def med(ts):
    ts = sorted(ts)
    return ts[len(ts) // 2] * 1e3, ts[0] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--big", action="store_true")
    a = ap.parse_args()
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    k = {x: int(y, 16) for x, y in keys["paillier2048_committed" if a.big else "paillier1024_seed1"].items()}
    u, rep = (100_000, 10) if a.big else (10_000, 1)
    n = u * rep
    eng = ddshe.Engine(0)
    col = eng.column(k["nsquare"], u)
    col.fill_paillier_synth(k["n"], k["g"], 1, 0, u, 64)
    rows = [str(x) for x in col.read(0, u)]
    want = pow(col.fold(), rep, k["nsquare"])
    enc = [r.encode() for r in rows]
    arr = (C.c_char_p * n)(*(enc * rep))
    cap = 4096
    obuf, olen, modb = C.create_string_buffer(cap), C.c_size_t(), str(k["nsquare"]).encode()
    ts = []
    for _ in range(a.reps):
        t = time.perf_counter()
        st = ddshe._lib.dds_sum_all_dec(eng._h, arr, n, modb, obuf, cap, C.byref(olen))
        ts.append(time.perf_counter() - t)
        assert st == 0 and int(obuf.value.decode()) == want
    out = {"rows": n, "chars": sum(map(len, rows)) * rep, "copy_threads": os.environ.get("DDSHE_COPY_THREADS", "8")}
    out["strings_median_ms"], out["strings_min_ms"] = med(ts)
    if a.big:  # the same rows as chars + offsets (bench.py end_to_end "decimal")
        chars = b"".join(enc) * rep
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.tile(np.array([len(r) for r in enc], dtype=np.uint64), rep), out=offs[1:])
        ts = []
        for _ in range(max(3, a.reps // 3)):
            t = time.perf_counter()
            dcol = eng.column(k["nsquare"], n)
            dcol.append_dec((chars, offs))
            got = dcol.fold()
            ts.append(time.perf_counter() - t)
            dcol.close()
            assert got == want
        out["chars_offsets_median_ms"], out["chars_offsets_min_ms"] = med(ts)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
