"""Print the end_to_end rates of bench logs under gpurun_out/ (tool, not product): e2e_summary.py TAG..."""
import json
import sys

for tag in sys.argv[1:]:
    d = None
    for line in open(f"gpurun_out/{tag}.log"):
        if line.startswith("{"):
            d = json.loads(line)
    e = d["end_to_end"]
    print(tag, {k: (round(v["rows_per_s"] / 1e6, 2), round(v["seconds"] * 1e3, 1),
                    v.get("matches", v.get("matches_resident_fold"))) for k, v in e.items()})
