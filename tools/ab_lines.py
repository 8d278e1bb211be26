#!/usr/bin/env python3
"""Print the key fields of bench lines in gpurun_out/<name>.log files (tool, not product).
usage: tools/ab_lines.py name [name ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for name in sys.argv[1:]:
    p = os.path.join(ROOT, "gpurun_out", name + ".log")
    if not os.path.exists(p):
        print(name, "missing")
        continue
    for line in open(p):
        if line.startswith('{"ope_bench"'):
            print(name, line.strip())
        elif line.startswith("{"):
            d = json.loads(line)
            ro = d.get("resident_opecol_order") or {}
            r = d.get("roofline") or {}
            print(name, f"ms/step {d['ms_per_step']:.4f}", f"verified {d.get('verified')}",
                  f"frac {r.get('frac', 0):.4f}", f"resident_dev_ms {ro.get('device_ms', 0):.4f}" if ro else "")
