#!/usr/bin/env python3
"""VALU issue summary of one kernel's largest dispatch from the tools/gpurun/pmc_valu.sh pass (tool, not product).

usage: tools/pmc_valu_summary.py <counter_collection.csv> <kernel substring> <products> <S> <out.json>
<products> Montgomery products that dispatch ran, <S> its limb count: the expected mad count is
products x (2 S^2 + S) lane-ops. Clock from GRBM_GUI_ACTIVE (summed over the 8 XCDs) over the
dispatch's own start/end timestamps; v_mad_u64_u32 issues at half rate, 64 lane-ops/clk/CU peak."""
import csv
import json
import sys

N_CU, N_XCD, N_SIMD = 256, 8, 1024


def main(path, kern, products, s, out):
    per = {}
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        d = per.setdefault(r["Dispatch_Id"], {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                             "name": r["Kernel_Name"]})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not per:
        sys.exit(f"no dispatch of {kern} in {path}")
    c = max(per.values(), key=lambda d: d.get("SQ_INSTS_VALU", 0.0))
    dur = c["dur_ns"] / 1e9
    clk = c["GRBM_GUI_ACTIVE"] / N_XCD / dur
    cycles = clk * dur
    i64 = c.get("SQ_INSTS_VALU_INT64", 0.0)
    mad_ops = i64 * 64 / (cycles * N_CU)
    derived = {
        "clock_GHz_est": clk / 1e9,
        "expected_mad_wave_instr": products * (2 * s * s + s) / 64,
        "valu_int64_share_of_valu": i64 / c["SQ_INSTS_VALU"],
        "mad_lane_ops_per_clk_per_CU": mad_ops,
        "mad_issue_frac_of_half_rate_peak_at_measured_clock": mad_ops / 64,
        "int64_instr_per_expected_mad": i64 / (products * (2 * s * s + s) / 64),
        "valu_wave_instr_per_clk_per_SIMD": c["SQ_INSTS_VALU"] / (cycles * N_SIMD),
        "issue_stall_share": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
        "waitcnt_share": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
    }
    counters = {k: v for k, v in c.items() if k not in ("dur_ns", "name")}
    json.dump({"kernel": c["name"][:120], "source": "rocprofv3 --pmc (tools/gpurun/pmc_valu.sh), largest dispatch of the kernel",
               "products": products, "S": s, "counters": counters, "duration_s": dur, "derived": derived},
              open(out, "w"), indent=1)
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
