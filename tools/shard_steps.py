#!/usr/bin/env python3
"""One rank's integrate of the C4 capture at world size W (bench.py's contiguous split), K passes of
reset + integrate_frames back to back, for a kernel trace (tools/step_head.py) of where a shard's step
goes.  Prints one JSON line: ms per pass and the per-launch integrate statistics of one profiled pass.

python tools/shard_steps.py --world 8 --rank 3 --steps 40
python tools/shard_steps.py --all --steps 40     (every rank of W = 2, 4, 8: per-rank ms per pass, one JSON line)
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
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--frames-per-side", type=int, default=1000)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--merge", action="store_true",
                    help="each pass also merges the shard through RCCL at world size 1 (root), alternating "
                         "rounds with a synchronize before the merge (no overlap with the integrate's last launch)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from mqr.distributed import shard_range
    from mqr.vbg import VoxelBlockGrid
    args = bench.parse([])
    full = bench.c4_capture(args, 0, a.frames_per_side)
    if a.all:
        kw = dict(depth_scale=1.0, depth_max=args.depth_max, trunc_voxel_multiplier=args.trunc)
        res = {}
        for world in (1, 2, 4, 8):
            per = []
            for r in range(world):
                lo, hi = shard_range(2 * a.frames_per_side, r, world)
                dd = full["depth_t"][lo:hi].contiguous()
                KK, TT = full["K"][lo:hi].astype(np.float64), full["T_wc"][lo:hi].astype(np.float64)
                v = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=16, block_count=args.block_count, device=0)
                ar = (bench._DevPtr(dd.data_ptr()), *dd.shape)
                for _ in range(3):
                    v.reset()
                    v.integrate_frames(ar, KK, TT, **kw)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    v.reset()
                    v.integrate_frames(ar, KK, TT, **kw)
                torch.cuda.synchronize()
                per.append((time.perf_counter() - t0) / a.steps * 1e3)
                del v, dd
            res[world] = {"ms_per_pass": per, "max_ms": max(per)}
            print(f"W={world}: max {max(per):.3f} ms per pass", file=sys.stderr, flush=True)
        print(json.dumps({"workload": "C4 capture, bench.py's contiguous split; per rank K passes of reset + "
                          "integrate_frames back to back (the bench's timed loop, asynchronous return)",
                          "steps": a.steps, "per_world": res}), flush=True)
        return
    if a.merge:
        import torch.distributed as dist
        from mqr.distributed import make_comm, merge_rccl
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29543")
        dist.init_process_group("gloo", rank=0, world_size=1)
        comm = make_comm(0)
        lo, hi = shard_range(2 * a.frames_per_side, a.rank, a.world)
        dd = full["depth_t"][lo:hi].contiguous()
        KK, TT = full["K"][lo:hi].astype(np.float64), full["T_wc"][lo:hi].astype(np.float64)
        v = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=16, block_count=args.block_count, device=0)
        kw = dict(depth_scale=1.0, depth_max=args.depth_max, trunc_voxel_multiplier=args.trunc)
        ar = (bench._DevPtr(dd.data_ptr()), *dd.shape)
        out = None
        res = {"overlap": [], "sync_first": []}
        for rnd in range(8):
            for mode in ("overlap", "sync_first"):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    v.reset()
                    v.integrate_frames(ar, KK, TT, **kw)
                    if mode == "sync_first":
                        torch.cuda.synchronize()
                    out, _ = merge_rccl(v, comm, mode="root", out=out)
                torch.cuda.synchronize()
                if rnd:
                    res[mode].append((time.perf_counter() - t0) / a.steps * 1e3)
        comm.close()
        dist.destroy_process_group()
        print(json.dumps({"workload": f"C4 shard {a.rank} of {a.world} ({hi - lo} frames): reset + integrate_frames + "
                          "merge_rccl (world size 1, root) per pass", "ms_per_pass_median":
                          {k: float(np.median(x)) for k, x in res.items()}, "ms_per_pass": res}), flush=True)
        return
    lo, hi = shard_range(2 * a.frames_per_side, a.rank, a.world)
    d = full["depth_t"][lo:hi].contiguous()
    K, T = full["K"][lo:hi].astype(np.float64), full["T_wc"][lo:hi].astype(np.float64)
    del full
    torch.cuda.synchronize()
    B, H, W = d.shape
    vbg = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=16, block_count=args.block_count, device=0)
    kw = dict(depth_scale=1.0, depth_max=args.depth_max, trunc_voxel_multiplier=args.trunc)
    arg = (bench._DevPtr(d.data_ptr()), B, H, W)
    for _ in range(3):
        vbg.reset()
        vbg.integrate_frames(arg, K, T, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        vbg.reset()
        vbg.integrate_frames(arg, K, T, **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    vbg.reset()
    vbg.stats(reset=True)
    vbg.profile(True, touch=True)
    vbg.integrate_frames(arg, K, T, **kw)
    vbg.profile(False)
    st = vbg.stats(reset=True)
    print(json.dumps({"world": a.world, "rank": a.rank, "frames": B, "range": [lo, hi], "ms_per_pass": ms,
                      "blocks": vbg.size(), "stats": st}), flush=True)


if __name__ == "__main__":
    main()
