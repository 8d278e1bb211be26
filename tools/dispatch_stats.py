#!/usr/bin/env python3
"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV (tool, not product).

usage: tools/dispatch_stats.py <run_kernel_trace.csv> <kernel substring> [last_k] [out.json]
Prints every dispatch of the kernel in launch order (grid size, ns), then the mean over all dispatches,
over the last `last_k` (the bench's timed steps come last), min, max and where the max sits, so a bench
line's HIP-event launch time can be matched to the same run's trace."""
import csv
import json
import sys


def main(path, kern, last_k=None, out=None):
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
         for r in rows]
    if not d:
        sys.exit(f"no dispatch of {kern} in {path}")
    ns = [x for x, _ in d]
    res = {"kernel": rows[0]["Kernel_Name"][:160], "source": path, "dispatches": len(ns),
           "durations_ms": [x / 1e6 for x in ns], "grids": [g for _, g in d],
           "mean_all_ms": sum(ns) / len(ns) / 1e6, "min_ms": min(ns) / 1e6, "max_ms": max(ns) / 1e6,
           "max_index": ns.index(max(ns))}
    if last_k:
        k = int(last_k)
        res["last_k"] = k
        res["mean_last_k_ms"] = sum(ns[-k:]) / len(ns[-k:]) / 1e6
    print(json.dumps({k: v for k, v in res.items() if k != "durations_ms"}, indent=1))
    print("durations_ms:", [round(x, 4) for x in res["durations_ms"]])
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
