"""Summaries of a rocprofv3 --kernel-trace --hip-trace csv run small enough to copy back:
HIP API totals, and per-phase (kernel-name regex) kernel time vs wall span.
usage: python tools/api_summary.py DIR"""
import glob
import re
import sys

import pandas as pd

d = sys.argv[1]
api = pd.read_csv(glob.glob(f"{d}/*hip_api_stats.csv")[0])
print(api[["Name", "Calls", "TotalDurationNs", "AverageNs"]].head(25).to_string())
kt = pd.read_csv(glob.glob(f"{d}/*kernel_trace.csv")[0])
at = pd.read_csv(glob.glob(f"{d}/*hip_api_trace.csv")[0])
for tag, rx in [("meshfilter", r"mqr::mf::"), ("bvh", r"k_gather_tris|k_morton|k_radix_tree|k_leaves|k_node_depth|k_refit_level|k_level_bounds")]:
    k = kt[kt["Kernel_Name"].str.contains(rx, regex=True)]
    if k.empty:
        continue
    # last call window: group kernels by gaps > 20 ms
    k = k.sort_values("Start_Timestamp")
    starts = k["Start_Timestamp"].values
    brk = [0] + [i for i in range(1, len(starts)) if starts[i] - starts[i - 1] > 20e6]
    lo = brk[-1]
    w = k.iloc[lo:]
    t0, t1 = w["Start_Timestamp"].min(), w["End_Timestamp"].max()
    busy = (w["End_Timestamp"] - w["Start_Timestamp"]).sum()
    a = at[(at["Start_Timestamp"] >= t0 - 2e6) & (at["End_Timestamp"] <= t1 + 2e6)]
    g = a.assign(dur=a["End_Timestamp"] - a["Start_Timestamp"]).groupby("Function")["dur"].agg(["count", "sum"])
    g = g.sort_values("sum", ascending=False).head(12)
    print(f"== {tag}: window {(t1 - t0) / 1e6:.2f} ms, kernels busy {busy / 1e6:.2f} ms, {len(w)} kernels")
    print((g.assign(sum_ms=g["sum"] / 1e6).drop(columns="sum")).to_string())
    top = w.assign(dur=w["End_Timestamp"] - w["Start_Timestamp"]).groupby("Kernel_Name")["dur"].sum()
    print((top.sort_values(ascending=False).head(8) / 1e6).to_string())
