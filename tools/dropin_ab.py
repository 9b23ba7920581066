#!/usr/bin/env python3
"""A/B of mqr.o3d_utils.CHUNK (frames per host -> device hand-off of the drop-in integrate()) on the
bench's on-disk C3 capture (bench.py dropin_e2e_leg: raw NDC files + descriptor CSV, confidence npz
written by estimate_depth_confidences), chunk sizes interleaved in one process, page cache warm.
Prints one JSON line: per chunk size the median integrate() seconds and frames/s, and whether every
chunk size left the same volume (keys and tsdf / weight bit for bit)."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="64,127")
    ap.add_argument("--firsts", default="", help="FIRST_CHUNK values to cross with the chunk sizes (default: the module's)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--profile", action="store_true", help="cProfile one integrate() per chunk size (main thread)")
    a = ap.parse_args()
    import numpy as np
    from mqr import o3d_utils, synthetic
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import CoordinateSystem, Side
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(a.frames), device="cuda:0")
    cap = {"raw": seq["raw_t"].cpu().numpy(), "unity": seq["unity"], "tangents": seq["tangents"],
           "near": seq["near"], "far": seq["far"], "width": seq["width"], "height": seq["height"]}
    tmp = tempfile.mkdtemp(prefix="mqr_chunk_ab_")
    try:
        synthetic.write_capture(tmp, cap)
        io = DepthDataIO(tmp)
        ds = io.load_depth_dataset(Side.LEFT)
        cfg = DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0, error_threshold=0.08,
                                              skip_if_output_dir_exists=False, device=0)
        estimate_depth_confidences(io, cfg, sides=[Side.LEFT])
        ds.transforms = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                                is_camera=True)
        kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2,
                  voxel_size=0.005, block_resolution=16, block_count=40000, depth_max=4.0,
                  trunc_voxel_multiplier=10.0, device=0)
        chunks = [int(c) for c in a.chunks.split(",")]
        if a.profile:
            import cProfile
            import io as _io
            import pstats
            o3d_utils.integrate(ds, io, Side.LEFT, **kw)  # warm-up
            for c in chunks:
                o3d_utils.CHUNK = c
                pr = cProfile.Profile()
                pr.enable()
                o3d_utils.integrate(ds, io, Side.LEFT, **kw)
                pr.disable()
                buf = _io.StringIO()
                pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(14)
                print(f"== CHUNK {c}\n" + buf.getvalue(), file=sys.stderr)
        firsts = [int(f) for f in a.firsts.split(",")] if a.firsts else [o3d_utils.FIRST_CHUNK]
        configs = [(c, f) for c in chunks for f in firsts]
        key = (lambda c, f: str(c)) if len(firsts) == 1 else (lambda c, f: f"{c}/first{f}")
        times = {key(c, f): [] for c, f in configs}
        splits = {}
        vols = {}
        for r in range(a.rounds + 1):
            for c, f in configs:
                o3d_utils.CHUNK = c
                o3d_utils.FIRST_CHUNK = f
                c = key(c, f)
                t0 = time.perf_counter()
                vbg = o3d_utils.integrate(ds, io, Side.LEFT, **kw)
                dt = time.perf_counter() - t0
                if r:
                    times[c].append(dt)
                    splits.setdefault(c, []).append(dict(o3d_utils.last_integrate_times.__dict__))
                if r == a.rounds:
                    k, t, w = vbg.export()
                    o = np.lexsort(k.T[::-1])
                    vols[c] = (k[o], t[o], w[o])
                del vbg
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    k0, t0_, w0 = vols[key(*configs[0])]
    out = {"frames": len(ds), "rounds": a.rounds, "chunks": {}}
    for c in (key(c, f) for c, f in configs):
        k1, t1, w1 = vols[c]
        same = k0.shape == k1.shape and (k0 == k1).all() and (w0 == w1).all() and (t0_.view(np.uint32) == t1.view(np.uint32)).all()
        med = float(np.median(times[c]))
        out["chunks"][c] = {"integrate_s": med, "integrate_frames_per_s": len(ds) / med, "all_s": times[c],
                            "volume_identical_to_first": bool(same), "splits_s": splits[c]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
