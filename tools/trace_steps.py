#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 --kernel-trace CSV of bench.py: wall time between consecutive
k_reset_table launches (one per step), the union of kernel busy time inside it, and the idle gaps.
usage: python3 tools/trace_steps.py <kernel_trace.csv> [--show N]"""
import json
import sys

import pandas as pd


def main():
    path = sys.argv[1]
    show = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--show" else 1
    df = pd.read_csv(path, usecols=["Kernel_Name", "Start_Timestamp", "End_Timestamp"]).sort_values("Start_Timestamp")
    starts = df[df["Kernel_Name"].str.contains("k_reset_table")]["Start_Timestamp"].tolist()
    out = {"steps": []}
    for i in range(max(0, len(starts) - 11), len(starts) - 1):
        s, e = starts[i], starts[i + 1]
        d = df[(df.Start_Timestamp >= s) & (df.Start_Timestamp < e)]
        iv = sorted(zip(d.Start_Timestamp, d.End_Timestamp))
        busy, gaps = 0, []
        cs, ce = iv[0]
        for a, b in iv[1:]:
            if a > ce:
                busy += ce - cs
                gaps.append((int(ce - s), int(a - ce)))
                cs, ce = a, b
            else:
                ce = max(ce, b)
        busy += ce - cs
        gaps.append((int(ce - s), int(e - ce)))
        out["steps"].append({"wall_ms": (e - s) / 1e6, "busy_ms": busy / 1e6, "kernels": int(len(d)),
                             "gaps_us": [(round(a / 1e3, 1), round(g / 1e3, 1)) for a, g in gaps if g > 2000]})
    last = starts[-2], starts[-1]
    d = df[(df.Start_Timestamp >= last[0]) & (df.Start_Timestamp < last[1])]
    out["last_step_kernels"] = [
        [round((r.Start_Timestamp - last[0]) / 1e3, 1), round((r.End_Timestamp - r.Start_Timestamp) / 1e3, 1),
         r.Kernel_Name.split("(")[0][-48:]] for r in d.itertuples()]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
