#!/usr/bin/env python3
"""Per-launch SQ counters of the integrate kernel from rocprofv3 --pmc csv passes (tools/pmc_sq.sh).
usage: sq_summary.py <dir with */*counter_collection.csv and workload.json> -> prints one JSON line."""
import glob
import json
import sys

import pandas as pd


def main(d):
    wl = json.load(open(f"{d}/workload.json"))
    rows = {}
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        df = pd.read_csv(path)
        df = df[df["Kernel_Name"].str.contains("k_integrate")]
        for c, g in df.groupby("Counter_Name"):
            rows[c] = float(g["Counter_Value"].mean())
            rows["launches"] = int(len(g))
    vf = wl["voxel_frames_per_launch"] if "voxel_frames_per_launch" in wl else None
    out = {"variant": wl.get("variant"), "counters_per_launch": rows, "workload": wl}
    if vf:
        out["valu_per_voxel_frame"] = rows.get("SQ_INSTS_VALU", 0) / vf * 64 / 64
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
