#!/usr/bin/env python3
"""HBM traffic per kernel from the rocprofv3 --pmc passes of tools/gpurun/profile_all.sh (tool, not product).

usage: tools/pmc_summary.py <prof dir> <out.json>
Reads <prof dir>/pmc_<workload>_{fetch,write}/**/*counter_collection.csv and writes, per
"<workload>:<kernel>", the dispatch count, FETCH_SIZE / WRITE_SIZE (KB, summed over the pass) and the
corrected HBM bytes per dispatch. gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
counts half the bytes of a coalesced stream, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024
as is."""
import csv
import glob
import json
import os
import re
import sys

WORKLOADS = {"pf": "product_filter", "order": "order", "sum": "sum", "enc": "encrypt_sum", "es": "entry_search"}


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("ddshe::", "")


def read_pass(d):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
            v = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
            disp = row.get("Dispatch_Id") or row.get("Correlation_Id") or ""
            e = acc.setdefault(k, {"value": 0.0, "dispatches": set(), "max": 0.0})
            e["value"] += v
            e["max"] = max(e["max"], v)
            e["dispatches"].add(disp)
    return acc


def main(prof, out):
    kernels = {}
    for tag, wl in WORKLOADS.items():
        fe = read_pass(os.path.join(prof, f"pmc_{tag}_fetch"))
        wr = read_pass(os.path.join(prof, f"pmc_{tag}_write"))
        for k in sorted(set(fe) | set(wr)):
            nd = max(len(fe.get(k, {}).get("dispatches", ())), len(wr.get(k, {}).get("dispatches", ())), 1)
            fkb = fe.get(k, {}).get("value", 0.0)
            wkb = wr.get(k, {}).get("value", 0.0)
            rb, wb = 2 * fkb * 1024, wkb * 1024
            kernels[f"{wl}:{k}"] = {"dispatches": nd, "FETCH_SIZE_KB": fkb, "read_bytes": rb / nd,
                                    "WRITE_SIZE_KB": wkb, "write_bytes": wb / nd,
                                    "hbm_bytes_per_dispatch": (rb + wb) / nd,
                                    # the largest dispatch (e.g. the 10M-row fold among the smaller folds of
                                    # the bench's extra lines)
                                    "hbm_bytes_max_dispatch": 2 * fe.get(k, {}).get("max", 0.0) * 1024
                                    + wr.get(k, {}).get("max", 0.0) * 1024}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, one bench step each "
                         "(tools/gpurun/profile_all.sh; tools/pmc_summary.py)",
               "correction": "gfx950 FETCH_SIZE counts half the bytes of a coalesced stream (MI355X_MICROARCH.md "
                             "HBM section): read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 as is",
               "rows_per_dispatch": 10000000, "kernels": kernels}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
