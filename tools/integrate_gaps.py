#!/usr/bin/env python3
"""Integrate-stream occupancy of the bench loop from a rocprofv3 --kernel-trace CSV: over the last
`--launches` integrate launches, their mean duration, the gaps between one launch's end and the next
one's start (the device's integrate stream idle), and how much of each launch another kernel (touch,
order, reset) ran beside.  With mqr_vbg_reset swapping table / pool sets, a step boundary no longer
drains the integrate stream, so this is the view that shows what is left between launches.
usage: python3 tools/integrate_gaps.py <kernel_trace.csv> [--launches 160] [--per-step 4]"""
import argparse
import json

import numpy as np
import pandas as pd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", type=int, default=160)
    ap.add_argument("--per-step", type=int, default=4)
    a = ap.parse_args()
    df = pd.read_csv(a.trace, usecols=["Kernel_Name", "Start_Timestamp", "End_Timestamp"]).sort_values("Start_Timestamp")
    is_int = df.Kernel_Name.str.contains("k_integrate_(?:wt|win|lean)")
    integ = df[is_int].tail(a.launches)
    other = df[~is_int]
    s = integ.Start_Timestamp.to_numpy(np.int64)
    e = integ.End_Timestamp.to_numpy(np.int64)
    dur = (e - s) / 1e3
    gaps = (s[1:] - e[:-1]) / 1e3
    os_, oe = other.Start_Timestamp.to_numpy(np.int64), other.End_Timestamp.to_numpy(np.int64)
    beside = []
    for a0, b0 in zip(s, e):
        m = (oe > a0) & (os_ < b0)
        beside.append(float(np.sum(np.minimum(oe[m], b0) - np.maximum(os_[m], a0))) / 1e3)
    span = (e[-1] - s[0]) / 1e3
    k = a.per_step
    gaps_by_pos = {f"gap_after_launch_{i}_of_{k}": float(np.median(gaps[i::k])) for i in range(min(k, len(gaps)))}
    print(json.dumps({
        "launches": int(len(s)),
        "integrate_mean_us": float(dur.mean()),
        "integrate_median_us": float(np.median(dur)),
        "gap_median_us": float(np.median(gaps)), "gap_mean_us": float(gaps.mean()), "gap_max_us": float(gaps.max()),
        "span_per_launch_us": span / (len(s) - 1) if len(s) > 1 else None,
        "span_per_step_us": span / (len(s) - 1) * k if len(s) > 1 else None,
        "integrate_busy_frac": float(dur[:-1].sum() / ((s[-1] - s[0]) / 1e3)) if len(s) > 1 else None,
        "other_kernels_beside_us_mean": float(np.mean(beside)),
        **gaps_by_pos,
        "note": "gap = next launch start - this launch end on the integrate stream; gap_after_launch_i: the median "
                "gap after the i-th launch of a step (launch 0 = a step's first; the index assumes the trace's "
                "last launches start at a step boundary, i.e. --launches a multiple of --per-step)",
    }, indent=1))


if __name__ == "__main__":
    main()
