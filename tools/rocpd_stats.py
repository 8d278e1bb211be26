#!/usr/bin/env python3
"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.
usage: tools/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name_col = "display_name" if "display_name" in cols else "kernel_name"
    rows = c.execute(f"select s.{name_col}, d.end - d.start from {disp} d join {sym} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        agg.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        mean = sum(v) / len(v)
        sd = (sum((x - mean) ** 2 for x in v) / len(v)) ** 0.5
        out.append([name, len(v), sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd])
    return out


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(hdr)
            w.writerows(rows)
    for r in rows:
        print(f"{r[1]:6d} {r[3]/1e3:12.1f} us {r[4]:6.2f}%  {r[0][:110]}")
