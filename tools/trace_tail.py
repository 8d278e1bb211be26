#!/usr/bin/env python3
"""Print the last N dispatches of a rocprofv3 kernel trace with durations and gaps (tool, not product).
    python tools/trace_tail.py gpurun_out/ft1/run_kernel_trace.csv [N]"""
import csv
import sys


def main(path, n=25):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    for r in rows[-n:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{r['Kernel_Name'][:64]:64s} grid={r['Grid_Size_X']:>8} dur={(e - s) / 1e3:8.2f}us gap={gap:7.2f}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
