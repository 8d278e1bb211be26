#!/usr/bin/env python3
"""OPE filter probe (tool, not product): device time per dds_ope_filter_device call (HIP events on the
launch stream, the engine's timing counters) over a 10M-row int64 column + valid bytes, 50 %
selectivity, and the resident OPE column's search (host output). Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ddshe  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rng = np.random.default_rng(3)
    col = rng.integers(-2**62, 2**62, size=n, dtype=np.int64)
    bound = int(np.median(col))
    eng = ddshe.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    d_col = torch.from_numpy(col).cuda()
    d_valid = torch.ones(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n, dtype=torch.int32, device="cuda")
    got = eng.ope_filter_device(d_col.data_ptr(), d_valid.data_ptr(), n, bound, "gt", d_out.data_ptr())
    ok = got == int((col > bound).sum())
    reps = 40
    eng.set_timing(True)
    eng.reset_timing()
    t = time.perf_counter()
    for r in range(reps):
        eng.ope_filter_device(d_col.data_ptr(), d_valid.data_ptr(), n, bound, ("gt", "ge", "lt", "le")[r % 4],
                              d_out.data_ptr())
    call_ms = (time.perf_counter() - t) / reps * 1e3
    _, _, dev_ms, _ = eng.timing()
    eng.set_timing(False)
    eng.ope_filter_device(d_col.data_ptr(), d_valid.data_ptr(), n, bound, "gt", d_out.data_ptr())
    dev = dev_ms / reps
    alg = 9 * n + 4 * got
    ids = d_out[:got].cpu().numpy().view(np.uint32)
    ok = ok and bool(np.array_equal(ids, np.nonzero(col > bound)[0].astype(np.uint32)))
    oc = eng.opecol(n)
    oc.append(col)
    oc.search(str(bound), "gt")
    t = time.perf_counter()
    r2 = oc.search(str(bound), "gt")
    res_ms = (time.perf_counter() - t) * 1e3
    print(json.dumps({"rows": n, "matches": got, "device_ms": dev, "call_ms": call_ms, "GBps": alg / dev / 1e6,
                      "frac_of_8TBps": alg / dev / 1e6 / 8000, "resident_search_host_ms": res_ms,
                      "ok": ok and bool(np.array_equal(r2, ids))}))


if __name__ == "__main__":
    main()
