#!/usr/bin/env python3
"""Decimal route A/B across library builds (tool, not product): median wall time of dds_sum_all_dec over
the same String[] rows (10k rows under the 1024-bit key, and 1M rows under the committed 2048-bit key's
n^2 with 100k distinct values), through plain ctypes so that an older build (DDSHE_LIB path) loads too.
    python tools/route_ab.py <lib.so> ...   (one process per library)"""
import ctypes as C
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(paths):
    keys = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    out = {}
    for path in paths:
        lib = C.CDLL(path)
        ctx = C.c_void_p()
        assert lib.dds_ctx_create(0, C.byref(ctx)) == 0
        res = {}
        for name, n, distinct, reps in (("paillier1024_seed1", 10000, 10000, 20), ("paillier2048_committed", 1000000, 100000, 5)):
            nsq = int(keys[name]["nsquare"], 16)
            rng = random.Random(7)
            vals = [str(rng.randrange(nsq)).encode() for _ in range(distinct)]
            rows = [vals[i % distinct] for i in range(n)]
            arr = (C.c_char_p * n)(*rows)
            cap = 4 * len(str(nsq)) + 64
            obuf, olen = C.create_string_buffer(cap), C.c_size_t()
            modb = str(nsq).encode()
            ts = []
            for _ in range(reps + 1):
                t = time.perf_counter()
                assert lib.dds_sum_all_dec(ctx, arr, n, modb, obuf, cap, C.byref(olen)) == 0
                ts.append(time.perf_counter() - t)
            ts = sorted(ts[1:])
            res[f"{name}_{n}"] = {"median_ms": round(ts[len(ts) // 2] * 1e3, 4), "result_digits": olen.value}
        out[os.path.basename(path)] = res
        lib.dds_ctx_destroy(ctx)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1:])
