#!/usr/bin/env python3
"""Benchmark of the TSDF fusion hot path (BASELINE.json config 1 at N=1).

A "step" = integrate the rank's whole 500-frame depth sequence (640x480, procedural room = a
512^3-voxel volume at 5 mm, R=16, depth_max 4 m, truncation 10 voxels) into an empty volume:
per 32-frame batch one touch launch (hash insert) + one integrate launch, inputs resident in HBM.
With N > 1 ranks every rank integrates its own 500 frames of an N*500-frame walk (weak scaling)
and the step ends with the single RCCL merge of the partial volumes into rank 0.

Prints ONE JSON line (rank 0): value = frames integrated per second over all ranks, the mesh
extraction time (weight_threshold 1.5, the pipeline's setting), the integrate kernel's roofline
(algorithmic bytes per launch / its average HIP-event duration) and the CPU-oracle baseline.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))

METRIC = "depth frames/sec integrated + mesh-extract ms, 512³ @ 5 mm; HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


class _DevPtr:
    def __init__(self, p):
        self.ptr = ctypes.c_void_p(p)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--voxel", type=float, default=0.005)
    ap.add_argument("--block-resolution", type=int, default=16)
    ap.add_argument("--block-count", type=int, default=40000)
    ap.add_argument("--depth-max", type=float, default=4.0)
    ap.add_argument("--trunc", type=float, default=10.0)
    ap.add_argument("--extract-threshold", type=float, default=1.5)
    ap.add_argument("--extract-reps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def extract_ms(vbg, thr, reps):
    from mqr import _lib
    times, counts = [], (0, 0)
    for _ in range(reps):
        g = ctypes.c_void_p()
        t0 = time.perf_counter()
        _lib.call("mqr_extract_mesh", vbg.handle, float(thr), ctypes.byref(g))
        times.append((time.perf_counter() - t0) * 1e3)
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("mqr_geom_counts", g, ctypes.byref(nv), ctypes.byref(nt))
        counts = (nv.value, nt.value)
        _lib.call("mqr_geom_free", g)
    times.sort()
    return times[len(times) // 2], counts


def pmc_traffic(H, W, frames):
    """HBM bytes per integrate launch from the committed rocprofv3 --pmc passes of this workload
    (tools/traffic_workload.py + tools/pmc_summary.py; FETCH_SIZE/WRITE_SIZE calibrated on k_pack)."""
    import glob
    recs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    for path in reversed(recs):
        try:
            rec = json.load(open(path))
            wl = rec["workload"]
            if (wl["H"], wl["W"], wl["frames"]) == (H, W, frames):
                return rec["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


def cpu_baseline(seq_host, K, T, args):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker / CPU restatement (port) -- timed here as the baseline only
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    oracle.set_threads(cores)
    ref = oracle.OracleVBG(args.voxel, args.block_resolution, args.block_count)
    t0 = time.perf_counter()
    n = 0
    while n < len(seq_host) and time.perf_counter() - t0 < args.cpu_seconds:
        ref.integrate_frame(seq_host[n], K[n], T[n], 1.0, args.depth_max, args.trunc)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"first {n} of the {len(seq_host)} frames, touch+integrate per frame (oracle/mqr_oracle.c, "
                      f"OpenMP over blocks), {dt:.1f} s"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import numpy as np
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from mqr import synthetic
    from mqr.distributed import merge_to_root
    from mqr.vbg import VoxelBlockGrid

    # this rank's frames of an N*frames closed walk through the room
    poses = synthetic.room_loop_poses(args.frames * world)[rank * args.frames:(rank + 1) * args.frames]
    seq = synthetic.make_sequence_fast("room", poses=poses, height=args.height, width=args.width, seed=rank,
                                       device=f"cuda:{local}")
    depth_t = seq["depth_t"].contiguous()
    B, H, W = depth_t.shape
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)
    dptr = (_DevPtr(depth_t.data_ptr()), B, H, W)
    torch.cuda.synchronize()

    vbg = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=args.block_resolution,
                         block_count=args.block_count, device=local)

    def step():
        vbg.reset()
        vbg.integrate_frames(dptr, K, T, depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc)
        if world > 1:
            merge_to_root(vbg)

    for _ in range(args.warmup):
        step()
    vbg.stats(reset=True)
    vbg.profile(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    vbg.profile(False)
    st = vbg.stats(reset=True)
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    blocks = vbg.size()
    ext_ms, (nv, nt) = (None, (0, 0))
    if rank == 0:
        ext_ms, (nv, nt) = extract_ms(vbg, args.extract_threshold, args.extract_reps)

    R3 = args.block_resolution ** 3
    alg_bytes = 16 * R3 * st["union_blocks"] + 4 * H * W * st["frames"] + 16 * st["frame_blocks"]
    launches = max(st["integrate_launches"], 1)
    avg_ms = st["integrate_ms"] / launches
    achieved = alg_bytes / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(depth_t.cpu().numpy(), K, T, args)

    traffic, traffic_src = pmc_traffic(H, W, B)

    if rank == 0:
        total_frames = B * world * args.steps
        out = {
            "metric": METRIC,
            "value": total_frames / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural room, GPU ray-cast, sigma=0.002z noise + 1% dropout)",
            "config": {"workload": "BASELINE config 1: 500-frame LEFT depth sequence per GPU, 640x480, hashed "
                                   "TSDF 5 mm voxels, 512^3 effective volume, R=16, depth_max 4 m, trunc 10",
                       "frames_per_gpu": B, "height": H, "width": W, "voxel_size": args.voxel,
                       "block_resolution": args.block_resolution, "depth_max": args.depth_max,
                       "trunc_voxel_multiplier": args.trunc, "frame_batch": 32,
                       "parallelism": f"frame-shard x{world}" + (" + RCCL reduce" if world > 1 else "")},
            "extract_ms": ext_ms,
            "extract": {"weight_threshold": args.extract_threshold, "vertices": nv, "triangles": nt,
                        "blocks": blocks, "note": "device-resident extract_triangle_mesh, median of reps"},
            "roofline": {"bound": "hbm", "kernel": "k_integrate", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes / launches, "avg_launch_ms": avg_ms,
                         "launches": st["integrate_launches"], "union_blocks_per_launch":
                             st["union_blocks"] / launches, "frame_blocks_per_frame":
                             st["frame_blocks"] / max(st["frames"], 1),
                         "touch_ms_per_launch": st["touch_ms"] / max(st["touch_launches"], 1)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
