#!/usr/bin/env python3
"""k_msd_local (and every other order kernel) device time per call from rocprofv3 kernel traces (tool, not
product). usage: tools/msd_local_times.py <trace dir> [<trace dir> ...]"""
import csv
import glob
import re
import statistics
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
    per = {}
    for r in rows:
        n = re.sub(r"\(.*$", "", re.sub(r"^void ", "", r["Kernel_Name"])).replace("ddshe::", "").split("<")[0]
        per.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(d, {k: round(statistics.median(v), 1) for k, v in per.items() if k.startswith(("k_msd", "k_rs_sc", "k_rs_h"))})
