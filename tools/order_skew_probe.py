#!/usr/bin/env python3
"""OrderLS call time on key distributions that stress the digit counting (tool, not product): the bench's
OPE column, uniform 54-bit keys, and 3 distinct keys spread over a 2^50 span (every wave's digits equal).
Prints one JSON line of median ms per raw-array call (dds_ope_order_device) per distribution."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402


def main(n=10_000_000, reps=15):
    rng = np.random.default_rng(5)
    eng = ddshe.Engine(0)
    ope_map = np.cumsum(rng.integers(1, 1 << 40, size=10001, dtype=np.int64)) - (1 << 52)
    cols = {"ope_bench": ope_map[rng.integers(1, 10001, size=n)],
            "uniform_2p54": rng.integers(0, 1 << 54, size=n, dtype=np.int64),
            "three_keys_2p50": np.array([0, 1 << 49, (1 << 50) - 1], dtype=np.int64)[rng.integers(0, 3, size=n)]}
    valid = torch.from_numpy((rng.random(n) > 0.05).astype(np.uint8)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    res = {}
    for name, c in cols.items():
        d = torch.from_numpy(c).cuda()
        ts = []
        print(name, flush=True)
        for r in range(reps + 2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            eng.ope_order_device(d.data_ptr(), valid.data_ptr(), n, True, out.data_ptr())
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t) * 1e3)
        ts = sorted(ts[2:])
        res[name] = round(ts[len(ts) // 2], 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
