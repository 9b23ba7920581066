#!/usr/bin/env python3
"""Interleaved A/B of extract_triangle_mesh configurations on the bench volume (C2, one process).

python tools/ab_extract.py --modes 3,7 --reps 15
mode = an extraction configuration under test (mqr_vbg_set_extract_mode, A/B library only; -1 = the
library default kExMode, extract.hip, the only mode of the product library): bit 0 per-cube triangle
counts from the count pass, bit 1 LDS row maps in the emission pass, bit 2 the scan's totals written
straight into pinned host memory instead of a D2H copy between the scan and the emission pass (all
three = 7, the default since round 5).  Round 4 also
measured, and removed: an emission over a compacted list of the blocks with output, the block's tsdf
staged in LDS for the interior vertex taps, XCD bands of the pool (profiles/r04_ab_extract.json),
the count pass emitting the vertices (0.264 vs 0.237 ms) and a vertex and a triangle workgroup per
block (0.187 vs 0.179 ms); round 3 measured a merged vertex / triangle item loop and 512-thread
emission blocks this way: no change (profiles/r03_ab_integrate_windows.json).
Prints per-mode median wall ms of mqr_extract_mesh (device-resident, the bench's extract_ms) and
whether positions / normals / triangles equal the first mode's bit for bit.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="-1")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--threshold", type=float, default=1.5)
    a = ap.parse_args()
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
    modes = [int(x) for x in a.modes.split(",")]
    ab = getattr(_lib.load(), "mqr_vbg_set_extract_mode", None) is not None
    times = {m: [] for m in modes}
    outs = {}
    for r in range(a.reps + 1):
        for m in modes:
            if ab:
                _lib.call("mqr_vbg_set_extract_mode", vbg.handle, m)
            elif m != -1:
                raise SystemExit("extraction modes other than -1 need the A/B library (MQR_HIP_LIB=tools/_ab/libmqr_ab.so)")
            g = ctypes.c_void_p()
            t0 = time.perf_counter()
            _lib.call("mqr_extract_mesh", vbg.handle, float(a.threshold), ctypes.byref(g))
            dt = (time.perf_counter() - t0) * 1e3
            if r > 0:
                times[m].append(dt)
            if r == a.reps:
                nv, nt = ctypes.c_int64(), ctypes.c_int64()
                _lib.call("mqr_geom_counts", g, ctypes.byref(nv), ctypes.byref(nt))
                p = np.empty((nv.value, 3), np.float32)
                n = np.empty((nv.value, 3), np.float32)
                t = np.empty((nt.value, 3), np.int32)
                _lib.call("mqr_geom_copy", g, p.ctypes.data_as(ctypes.c_void_p), n.ctypes.data_as(ctypes.c_void_p),
                          t.ctypes.data_as(ctypes.c_void_p), 0)
                outs[m] = (p, n, t)
            _lib.call("mqr_geom_free", g)
    res = {}
    p0, n0, t0_ = outs[modes[0]]
    for m in modes:
        p, n, t = outs[m]
        res[m] = {"ms": float(np.median(times[m])), "vertices": int(len(p)), "triangles": int(len(t)),
                  "bit_identical_to_first": bool(p.shape == p0.shape and t.shape == t0_.shape and
                                                 (p.view(np.uint32) == p0.view(np.uint32)).all() and
                                                 (n.view(np.uint32) == n0.view(np.uint32)).all() and
                                                 (t == t0_).all())}
    print(json.dumps({"modes": res, "blocks": vbg.size(), "threshold": a.threshold}))


if __name__ == "__main__":
    main()
