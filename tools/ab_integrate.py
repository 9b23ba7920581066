#!/usr/bin/env python3
"""Interleaved A/B of integrate-kernel variants on the bench workload (one process, same data).

python tools/ab_integrate.py --variants 0,5 --rounds 5
(variants 3 and 5 and bit 0x8000 need the A/B library: MQR_HIP_LIB=tools/_ab/libmqr_ab.so)
Prints per-variant median integrate-kernel ms per launch, touch ms, and step ms.
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
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--batch", type=int, default=0, help="frames per integrate_frames call (0 = all)")
    ap.add_argument("--no-profile", action="store_true", help="no per-launch timing events (step time only)")
    ap.add_argument("--separate", action="store_true", help="one volume per variant (variants that size the table)")
    ap.add_argument("--check", action="store_true", help="compare every variant's volume with the first's, bit for bit")
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
    variants = [int(x, 0) for x in a.variants.split(",")]
    shared = VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0)
    vols = {v: (VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0)
                if a.separate else shared) for v in variants}
    res = {v: {"int": [], "touch": [], "step": []} for v in variants}
    check = {}
    for r in range(a.rounds + 1):
        for v in variants:
            vbg = vols[v]
            _lib.call("mqr_vbg_set_variant", vbg.handle, v)
            vbg.reset()
            vbg.stats(reset=True)
            vbg.profile(not a.no_profile, touch=True)
            t0 = time.perf_counter()
            vbg.integrate_frames((_DevPtr(d.data_ptr()), B, H, W), K, T, depth_scale=1.0, depth_max=4.0,
                                 trunc_voxel_multiplier=10.0)
            dt = time.perf_counter() - t0
            vbg.profile(False)
            st = vbg.stats(reset=True)
            if r == 0:
                continue  # warm-up round
            res[v]["int"].append(st["integrate_ms"] / max(st["integrate_launches"], 1))
            res[v]["touch"].append(st["touch_ms"] / max(st["touch_launches"], 1))
            res[v]["step"].append(dt * 1e3)
            if a.check and r == a.rounds:
                keys, tsdf, wgt = vbg.export()
                order = np.lexsort(keys.T[::-1])
                check[v] = (keys[order], tsdf[order], wgt[order])
    out = {v: {k: float(np.median(x)) for k, x in r.items()} for v, r in res.items()}
    if a.check:
        k0, t0_, w0 = check[variants[0]]
        for v in variants[1:]:
            k1, t1, w1 = check[v]
            same = k0.shape == k1.shape and (k0 == k1).all() and (w0 == w1).all() and \
                (t0_.view(np.uint32) == t1.view(np.uint32)).all()
            out[v]["bit_identical_to_first"] = bool(same)
    print(json.dumps({"variants": out, "blocks": shared.size() if not a.separate else vols[variants[0]].size()}))


if __name__ == "__main__":
    main()
