#!/usr/bin/env python3
"""HBM bytes of each OrderLS call from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of the order
bench (tool, not product).

usage: tools/order_call_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]
Dispatches in launch order are cut into calls after each k_msd_big (the last kernel of a call; k_rs_publish before round 6b); per
call: kernels, read bytes = 2 x FETCH_SIZE x 1024 and write bytes = WRITE_SIZE x 1024 (the gfx950
correction of MI355X_MICROARCH.md, as tools/pmc_summary.py)."""
import csv
import json
import re
import sys


def per_dispatch(path, counter):
    d = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        name = re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["Kernel_Name"])).replace("ddshe::", "")
        e = d.setdefault(k, [name, 0.0])
        e[1] += float(r["Counter_Value"])
    return d


def calls(d):
    out, cur = [], []
    for k in sorted(d):
        cur.append((k, d[k][0], d[k][1]))
        if d[k][0] in ("k_rs_publish", "k_msd_big"):
            out.append(cur)
            cur = []
    return out


def main(fetch, write, out=None):
    f, w = calls(per_dispatch(fetch, "FETCH_SIZE")), calls(per_dispatch(write, "WRITE_SIZE"))
    res = []
    for i, (cf, cw) in enumerate(zip(f, w)):
        kern = {}
        for (_, n, v) in cf:
            kern.setdefault(n, [0.0, 0.0])[0] += 2 * v * 1024
        for (_, n, v) in cw:
            kern.setdefault(n, [0.0, 0.0])[1] += v * 1024
        rb = sum(x[0] for x in kern.values())
        wb = sum(x[1] for x in kern.values())
        res.append({"call": i, "kernels": [n for (_, n, _) in cf], "read_bytes": rb, "write_bytes": wb,
                    "hbm_bytes": rb + wb, "per_kernel": {n: {"read": v[0], "write": v[1]} for n, v in kern.items()}})
        print(i, f"{(rb + wb) / 1e9:.4f} GB", " ".join(n for (_, n, _) in cf))
    if out:
        json.dump({"source": [fetch, write], "calls": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
