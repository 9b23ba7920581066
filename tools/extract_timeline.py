#!/usr/bin/env python3
"""Where the wall time of one extract_triangle_mesh goes (C2 volume, device-resident result).

Run:      rocprofv3 --kernel-trace -f csv -d gpurun_out/xt -o run -- python tools/extract_timeline.py --run
Analyse:  python tools/extract_timeline.py --analyze <kernel_trace.csv> gpurun_out/xt_walls.json
The run does `--reps` mqr_extract_mesh calls, each bracketed by host timestamps (CLOCK_MONOTONIC and
CLOCK_BOOTTIME; the analysis uses whichever clock rocprofv3's kernel stamps fall into); the analysis lists per call the host wall, the device span from
the first kernel's start to the last kernel's end, the kernel busy sum, the gaps between kernels and
the host time before the first kernel starts and after the last one ends (medians over the calls)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def run(a):
    import numpy as np
    import torch
    from bench import _DevPtr
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
    d = seq["depth_t"].contiguous()
    B, H, W = d.shape
    vbg = VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0)
    vbg.integrate_frames((_DevPtr(d.data_ptr()), B, H, W), seq["K"].astype(np.float64),
                         seq["T_wc"].astype(np.float64), depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    torch.cuda.synchronize()
    walls = []
    for r in range(a.reps + 2):
        g = ctypes.c_void_p()
        t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        _lib.call("mqr_extract_mesh", vbg.handle, 1.5, ctypes.byref(g))
        t1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC), time.clock_gettime_ns(time.CLOCK_BOOTTIME)
        _lib.call("mqr_geom_free", g)
        if r >= 2:  # the first two size the scratch and the speculative capacity
            walls.append((t0, t1))
        time.sleep(0.002)
    os.makedirs(os.path.dirname(a.walls), exist_ok=True)
    json.dump(walls, open(a.walls, "w"))


def analyze(trace, walls_path):
    import numpy as np
    import pandas as pd
    df = pd.read_csv(trace, usecols=["Kernel_Name", "Start_Timestamp", "End_Timestamp"]).sort_values("Start_Timestamp")
    walls = json.load(open(walls_path))
    # the clock (MONOTONIC or BOOTTIME) whose windows hold the kernels
    hits = [sum(((df.Start_Timestamp >= w[0][c]) & (df.End_Timestamp <= w[1][c])).sum() for w in walls) for c in (0, 1)]
    c = 0 if hits[0] >= hits[1] else 1
    rows = []
    for w in walls:
        t0, t1 = w[0][c], w[1][c]
        d = df[(df.Start_Timestamp >= t0) & (df.End_Timestamp <= t1)]
        if d.empty:
            continue
        ks = list(zip(d.Start_Timestamp, d.End_Timestamp, d.Kernel_Name))
        gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
        rows.append({"wall": t1 - t0, "span": ks[-1][1] - ks[0][0], "busy": sum(e - s for s, e, _ in ks),
                     "head": ks[0][0] - t0, "tail": t1 - ks[-1][1], "gaps": gaps,
                     "kernels": [(n.split("(")[0].split("::")[-1][:28], e - s) for s, e, n in ks]})
    med = lambda k: float(np.median([r[k] for r in rows])) / 1e3  # noqa: E731
    out = {"clock": ("CLOCK_MONOTONIC", "CLOCK_BOOTTIME")[c], "calls": len(rows), "wall_us": med("wall"), "device_span_us": med("span"), "kernel_busy_us": med("busy"),
           "host_head_us": med("head"), "host_tail_us": med("tail"),
           "gaps_us": [float(np.median([r["gaps"][i] for r in rows if len(r["gaps"]) > i])) / 1e3
                       for i in range(max(len(r["gaps"]) for r in rows))],
           "kernels_us": [(rows[0]["kernels"][i][0],
                           float(np.median([r["kernels"][i][1] for r in rows if len(r["kernels"]) > i])) / 1e3)
                          for i in range(len(rows[0]["kernels"]))]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--walls", default=os.path.join(ROOT, "gpurun_out", "xt_walls.json"))
    ap.add_argument("--analyze", nargs=2, metavar=("TRACE", "WALLS"))
    a = ap.parse_args()
    if a.analyze:
        analyze(*a.analyze)
    else:
        run(a)
