#!/usr/bin/env python3
"""Per-block triangle counts of the C2 mesh in the emission pass's order (triangles are emitted in
(block, cube, triangle) order, so runs of one block coordinate are the blocks, in pool order): how
the emission workgroups' triangle work is distributed and where the heavy blocks sit in the
dispatch order."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def runs(keys):
    import numpy as np
    if len(keys) == 0:
        return np.zeros(0, np.int64)
    change = np.nonzero(np.any(keys[1:] != keys[:-1], axis=1))[0] + 1
    edges = np.concatenate([[0], change, [len(keys)]])
    return np.diff(edges)


def main():
    import numpy as np
    import torch
    from bench import _DevPtr
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
    d = seq["depth_t"].contiguous()
    B, H, W = d.shape
    vbg = VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=40000, device=0)
    vbg.integrate_frames((_DevPtr(d.data_ptr()), B, H, W), seq["K"].astype(np.float64),
                         seq["T_wc"].astype(np.float64), depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    torch.cuda.synchronize()
    m = vbg.extract_triangle_mesh(weight_threshold=1.5)
    V = np.asarray(m.vertices, np.float64)
    T = np.asarray(m.triangles)
    bs = 0.005 * 16
    # a triangle belongs to the block of its cube: the floor of its centroid's block coordinate
    # (vertices are not attributed -- an edge vertex can sit on the far side of a block face)
    tblk = np.floor(V[T].mean(axis=1) / bs).astype(np.int64)
    nt = runs(tblk)
    a = np.sort(nt)[::-1]
    tot = a.sum()
    out = {"triangles": {"blocks": int(len(a)), "mean": float(a.mean()), "max": int(a[0]),
                         "q50": float(np.percentile(a, 50)), "q90": float(np.percentile(a, 90)),
                         "q99": float(np.percentile(a, 99)),
                         "share_in_blocks_over_256": float(a[a > 256].sum() / tot),
                         "share_in_blocks_over_512": float(a[a > 512].sum() / tot),
                         "blocks_over_512": int((a > 512).sum()), "blocks_over_1024": int((a > 1024).sum())}}
    # position of the heavy blocks in the dispatch (pool) order
    heavy = np.nonzero(nt > 512)[0]
    out["heavy_blocks_position_quantiles"] = ([float(x) for x in np.percentile(heavy / max(len(nt), 1), [0, 25, 50, 75, 100])]
                                              if len(heavy) else [])
    out["triangle_rounds_of_256"] = {"max": int(np.ceil(nt.max() / 256)), "mean": float(np.ceil(nt / 256).mean())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
