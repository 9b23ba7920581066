#!/usr/bin/env python3
"""Kernel timeline of one merge from a rocprofv3 --kernel-trace CSV of tools/time_merge.py: the kernels
between the last two k_merge_fused launches (the last rep of the RCCL world-1 root merge), with start
offsets and durations, plus the per-kernel totals over that window.  Keeps the multi-10-MB trace on the
box.  usage: python3 tools/merge_trace.py <kernel_trace.csv>"""
import json
import sys

import pandas as pd


def main():
    df = pd.read_csv(sys.argv[1], usecols=["Kernel_Name", "Start_Timestamp", "End_Timestamp"]).sort_values(
        "Start_Timestamp")
    idx = df.index[df.Kernel_Name.str.contains("k_merge_fused|k_merge_blocks")].tolist()
    a, b = df.loc[idx[-2]], df.loc[idx[-1]]
    d = df[(df.Start_Timestamp > a.End_Timestamp) & (df.Start_Timestamp <= b.Start_Timestamp)]
    s0 = d.Start_Timestamp.iloc[0]
    rows = [{"at_us": (r.Start_Timestamp - s0) / 1e3, "us": (r.End_Timestamp - r.Start_Timestamp) / 1e3,
             "kernel": r.Kernel_Name[:100]} for r in d.itertuples()]
    tot = d.assign(us=(d.End_Timestamp - d.Start_Timestamp) / 1e3).groupby(
        d.Kernel_Name.str[:80])["us"].agg(["sum", "count"]).sort_values("sum", ascending=False)
    print(json.dumps({"window_us": (b.Start_Timestamp - s0) / 1e3, "timeline": rows,
                      "totals": {k: {"us": float(v["sum"]), "n": int(v["count"])} for k, v in tot.iterrows()}},
                     indent=1))


if __name__ == "__main__":
    main()
