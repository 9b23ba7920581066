#!/usr/bin/env python3
"""Wall-time breakdown of one bench step: vbg.reset() vs integrate_frames (device-resident frames)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from bench import _DevPtr
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
    d = seq["depth_t"].contiguous()
    B, H, W = d.shape
    K, T = seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    torch.cuda.synchronize()
    vbg = VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0)
    res = {"reset": [], "integrate": [], "integrate_profiled": []}
    for r in range(6):
        t0 = time.perf_counter()
        vbg.reset()
        t1 = time.perf_counter()
        prof = r % 2 == 1
        vbg.profile(prof, touch=True)
        vbg.integrate_frames((_DevPtr(d.data_ptr()), B, H, W), K, T, depth_scale=1.0, depth_max=4.0,
                             trunc_voxel_multiplier=10.0)
        t2 = time.perf_counter()
        vbg.profile(False)
        st = vbg.stats(reset=True)
        if r >= 2:
            res["reset"].append((t1 - t0) * 1e3)
            res["integrate_profiled" if prof else "integrate"].append((t2 - t1) * 1e3)
            if prof:
                res.setdefault("kernel_sum_ms", []).append(st["integrate_ms"])
                res.setdefault("touch_sum_ms", []).append(st["touch_ms"])
    print({k: [round(x, 3) for x in v] for k, v in res.items()})


if __name__ == "__main__":
    main()
