#!/usr/bin/env python3
"""Time the libmqr merge (mqr_merge_local: the mqr_reduce_rccl plan and merge kernels with local
copies in place of RCCL) for N frame-sharded volumes of the bench's weak-scaling walk on one GPU."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import numpy as np
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from bench import _DevPtr
    from mqr import synthetic
    from mqr.distributed import merge_local, merge_local_timing
    from mqr.vbg import VoxelBlockGrid
    poses = synthetic.room_loop_poses(a.frames * a.ranks)
    vols = []
    for r in range(a.ranks):
        seq = synthetic.make_sequence_fast("room", poses=poses[r * a.frames:(r + 1) * a.frames], seed=r, device="cuda:0")
        d = seq["depth_t"].contiguous()
        v = VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=16384, device=0)
        v.integrate_frames((_DevPtr(d.data_ptr()), *d.shape), seq["K"].astype(np.float64),
                           seq["T_wc"].astype(np.float64), depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        vols.append(v)
        del d, seq
    torch.cuda.synchronize()
    res = {"ranks": a.ranks, "blocks_per_rank": [v.size() for v in vols]}
    for mode in ("sharded", "root"):
        outs, ts = None, []
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            got = merge_local(vols, mode=mode, outs=outs)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            outs = [o for o, _ in got]
        per = merge_local_timing(a.ranks)
        res[mode] = {"ms": sorted(ts[1:])[len(ts[1:]) // 2] * 1e3, "owned": [n for _, n in got],
                     "per_destination_ms": per, "max_per_destination_ms": max(per)}
    # the RCCL path at world size 1 (plan, output volume, gather, merge kernels; no peers)
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("gloo", rank=0, world_size=1)
    from mqr.distributed import make_comm, merge_rccl
    comm = make_comm(0)
    for mode in ("sharded", "root"):
        out, ts = None, []
        for _ in range(a.reps + 1):
            t0 = time.perf_counter()
            out, owned = merge_rccl(vols[0], comm, mode=mode, out=out)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res["rccl_world1_" + mode] = {"ms": sorted(ts[1:])[len(ts[1:]) // 2] * 1e3, "owned": owned,
                                      "phases_ms": comm.timing()}
    comm.close()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
