#!/usr/bin/env python3
"""Step head of the bench from a rocprofv3 --kernel-trace CSV: per step (k_reset_table launch to the
next), when the first integrate launch starts, how long the first touch, k_lpt_order and k_gate run,
the step's wall time, and the kernel-idle gaps inside it.  Median over the last `--steps` steps.
usage: python3 tools/step_head.py <kernel_trace.csv> [--steps 40]"""
import json
import sys

import numpy as np
import pandas as pd


def main():
    path = sys.argv[1]
    n = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--steps" else 40
    df = pd.read_csv(path, usecols=["Kernel_Name", "Start_Timestamp", "End_Timestamp"]).sort_values("Start_Timestamp")
    starts = df[df["Kernel_Name"].str.contains("k_reset_table")]["Start_Timestamp"].tolist()
    rows = []
    for i in range(max(0, len(starts) - n - 1), len(starts) - 1):
        s, e = starts[i], starts[i + 1]
        d = df[(df.Start_Timestamp >= s) & (df.Start_Timestamp < e)]
        integ = d[d.Kernel_Name.str.contains("k_integrate_(?:wt|win|lean)")]
        touch = d[d.Kernel_Name.str.contains("k_touch")]
        lpt = d[d.Kernel_Name.str.contains("k_lpt_order")]
        gate = d[d.Kernel_Name.str.contains("k_gate")]
        if integ.empty or touch.empty:
            continue
        iv = sorted(zip(d.Start_Timestamp, d.End_Timestamp))
        busy, (cs, ce) = 0, iv[0]
        for a, b in iv[1:]:
            if a > ce:
                busy += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        busy += ce - cs
        rows.append({"step_us": (e - s) / 1e3, "first_integrate_at_us": (integ.Start_Timestamp.iloc[0] - s) / 1e3,
                     "first_touch_us": (touch.End_Timestamp.iloc[0] - touch.Start_Timestamp.iloc[0]) / 1e3,
                     "first_lpt_us": ((lpt.End_Timestamp.iloc[0] - lpt.Start_Timestamp.iloc[0]) / 1e3) if len(lpt) else None,
                     "gate_at_us": ((gate.Start_Timestamp.iloc[0] - s) / 1e3) if len(gate) else None,
                     "integrate_launches": int(len(integ)),
                     "integrate_mean_us": float((integ.End_Timestamp - integ.Start_Timestamp).mean() / 1e3),
                     "last_integrate_end_to_next_step_us": (e - integ.End_Timestamp.iloc[-1]) / 1e3,
                     "idle_us": (e - s - busy) / 1e3})
    med = {k: float(np.median([r[k] for r in rows if r[k] is not None])) for k in rows[0] if
           any(r[k] is not None for r in rows)}
    print(json.dumps({"steps": len(rows), "median": med}, indent=1))


if __name__ == "__main__":
    main()
