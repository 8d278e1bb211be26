"""Summarise OrderLS A/B runs (tools/gpurun/order_ab.sh): the bench line of each variant and the
per-kernel device time of the last OrderLS call in its rocprofv3 kernel trace."""
import csv
import json
import sys


def last_call(trace):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"].split("(")[0].replace("ddshe::", ""), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
           for r in rows]
    # the last call starts at the last first-pass histogram kernel (or prep) after a large copy
    starts = [i for i, (k, _) in enumerate(seq) if k.startswith("k_rs_hist") or k.startswith("k_rs_glob")]
    i0 = starts[-2] if len(starts) >= 2 else 0
    for i in range(len(seq) - 1, 0, -1):
        if seq[i][0].startswith("k_msd_big") or seq[i][0].startswith("k_msd_local"):
            end = i
            break
    # walk back from the end to the first hist of that call
    j = end
    while j > 0 and not (seq[j][0].startswith("__amd_rocclr_copyBuffer") and seq[j][1] > 100):
        j -= 1
    return seq[j + 1:end + 1]


for name in sys.argv[1:]:
    line = None
    for l in open(f"bench_{name}.log"):
        if l.startswith("{"):
            line = json.loads(l)
    calls = last_call(f"prof/order_{name}/run_kernel_trace.csv")
    tot = sum(t for _, t in calls)
    print(f"{name}: ms/step {line['ms_per_step']:.4f} verified {line.get('verified')} resident device_ms "
          f"{line['resident_opecol_order'].get('device_ms', 0):.4f}  last-call kernels {tot:.1f} us")
    print("   " + "  ".join(f"{k[:14]}={t:.1f}" for k, t in calls))
