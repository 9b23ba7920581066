#!/usr/bin/env python3
"""Workload for the rocprofv3 --pmc traffic passes: the bench's integrate step (one 500-frame
pass, default kernel) followed by k_pack over every block (known bytes: U*R^3*8 read + written)
which calibrates FETCH_SIZE / WRITE_SIZE for 8-byte-per-lane accesses (MI355X_MICROARCH.md §HBM:
other widths are uncalibrated).  Writes gpurun_out/pmc/workload.json with the known byte counts."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def ctypes_int():
    import ctypes
    return ctypes.c_int(-1)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=-1, help="integrate kernel variant (-1 = library default)")
    ap.add_argument("--out", default="pmc")
    ap.add_argument("--extract", type=int, default=0, help="extract_triangle_mesh(1.5) calls after the pack")
    a = ap.parse_args()
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
    if a.variant >= 0:
        from mqr import _lib
        _lib.call("mqr_vbg_set_variant", vbg.handle, a.variant)
    vbg.profile(True)
    vbg.integrate_frames((_DevPtr(d.data_ptr()), B, H, W), K, T, depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    st = vbg.stats(reset=True)
    keys = torch.as_tensor(np.unique(vbg.export_keys(), axis=0), device="cuda:0").contiguous()
    U = keys.shape[0]
    out = torch.empty((U, 4096, 2), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    vbg.pack_weighted(keys.data_ptr(), U, out.data_ptr())
    torch.cuda.synchronize()
    if a.extract:
        from bench import extract_ms
        extract_ms(vbg, 1.5, a.extract)  # device-resident mqr_extract_mesh, result freed
    torch.cuda.synchronize()
    R3 = 4096
    info = {"integrate_launches": st["integrate_launches"], "union_blocks": st["union_blocks"],
            "frame_blocks": st["frame_blocks"], "frames": st["frames"], "H": H, "W": W,
            "alg_bytes_total": 16 * R3 * st["union_blocks"] + 4 * H * W * st["frames"] + 16 * st["frame_blocks"],
            "pack_blocks": U, "pack_read_bytes": U * R3 * 8, "pack_write_bytes": U * R3 * 8}
    info["variant"] = a.variant
    from mqr import _lib
    lv = ctypes_int()
    _lib.call("mqr_vbg_last_kernel", vbg.handle, lv)
    info["variant_ran"] = lv.value
    info["integrate_src"] = _lib.build_tag(0)  # the build this record measured (bench.py quotes matching ones)
    info["voxel_frames_per_launch"] = R3 * st["frame_blocks"] / max(st["integrate_launches"], 1)
    os.makedirs(os.path.join(ROOT, "gpurun_out", a.out), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", a.out, "workload.json"), "w") as f:
        json.dump(info, f)
    print(json.dumps(info))


if __name__ == "__main__":
    main()
