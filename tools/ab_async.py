#!/usr/bin/env python3
"""A/B of integrate variants in the bench's timed loop -- reset + integrate_frames over the 500-frame
C2 walk, K steps back to back bracketed by synchronize -- in alternating rounds of one process, with
every variant's volume compared to the first's bit for bit (blocks matched by key).  Default: the
asynchronous return of mqr_integrate_frames on device frames (variant 0: the call returns with its last
integrate queued) vs the synchronous one (variant bit 24: the streams drained before returning).
Prints one JSON object (median ms per step per variant).

python tools/ab_async.py --rounds 7 --steps 100 [--variants 0,0x1000000,0x400000,r0]   (r: resident frames)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--variants", default="0,0x1000000")
    a = ap.parse_args()
    import numpy as np
    import torch
    from bench import _DevPtr
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(a.frames), device="cuda:0")
    d = seq["depth_t"].contiguous()
    B, H, W = d.shape
    K, T = seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    torch.cuda.synchronize()
    names = {0: "async", 0x1000000: "sync"}
    # a variant prefixed "r" passes the frames as MQR_DEVICE_RESIDENT (integrate_frames(resident=True))
    modes = {(("resident" if v == "r0" else v) if v.startswith("r") else names.get(int(v, 0), v)):
             int(v.lstrip("r"), 0) for v in a.variants.split(",")}
    resident = {m: m.startswith("r") for m in modes}
    vols = {m: VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0) for m in modes}
    for m, v in modes.items():
        _lib.call("mqr_vbg_set_variant", vols[m].handle, v)
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    arg = (_DevPtr(d.data_ptr()), B, H, W)
    res = {m: [] for m in modes}
    for r in range(a.rounds + 1):
        for m in modes:
            vbg = vols[m]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                vbg.reset()
                vbg.integrate_frames(arg, K, T, resident=resident[m], **kw)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            if r:
                res[m].append(dt)
        print(f"round {r}: " + ", ".join(f"{m} {res[m][-1]:.4f}" for m in modes if res[m]), file=sys.stderr)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from gpu_helpers import compare_volumes
    first = vols[next(iter(modes))].export()
    same = True
    for m in list(modes)[1:]:
        try:
            same = same and compare_volumes(first, vols[m].export(), 0.0) == 0.0
        except AssertionError:
            same = False
    out = {"workload": f"C2 bench loop: reset + integrate_frames over {B} HBM-resident frames, {a.steps} steps per round",
           "variants": {m: hex(v) for m, v in modes.items()},
           "ms_per_step_median": {m: float(np.median(v)) for m, v in res.items()},
           "ms_per_step_all": res, "frames_per_s_median": {m: B / float(np.median(v)) * 1e3 for m, v in res.items()},
           "volumes_identical": bool(same)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
