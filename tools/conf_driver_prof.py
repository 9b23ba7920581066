#!/usr/bin/env python3
"""cProfile of mqr.confidence.estimate_depth_confidences on the bench's 500-frame on-disk capture (the
dropin_e2e leg's first half): one warm-up call, then a profiled one into a fresh output directory.
Prints the time split (confidence.last_confidence_times) as one JSON line on stdout and the profile's
top entries (cumulative and own time) on stderr."""
import cProfile
import io
import json
import os
import pstats
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def main():
    from mqr import confidence, synthetic
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
    cap = {"raw": seq["raw_t"].cpu().numpy(), "unity": seq["unity"], "tangents": seq["tangents"],
           "near": seq["near"], "far": seq["far"], "width": seq["width"], "height": seq["height"]}
    tmp = tempfile.mkdtemp(prefix="mqr_conf_prof_")
    try:
        synthetic.write_capture(tmp, cap)
        io_ = DepthDataIO(tmp)
        io_.load_depth_dataset(Side.LEFT)
        cfg = DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0, error_threshold=0.08,
                                              skip_if_output_dir_exists=False, device=0)
        estimate_depth_confidences(io_, cfg, sides=[Side.LEFT])  # warm-up
        shutil.rmtree(os.path.join(tmp, "left_depth_confidence"), ignore_errors=True)
        import gc
        gc_ms = []
        gc_t = {}

        def on_gc(phase, info):  # the collector's own passes during the profiled call
            if phase == "start":
                gc_t["t"] = time.perf_counter()
            else:
                gc_ms.append((info["generation"], (time.perf_counter() - gc_t["t"]) * 1e3))
        gc.callbacks.append(on_gc)
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        estimate_depth_confidences(io_, cfg, sides=[Side.LEFT])
        pr.disable()
        wall = time.perf_counter() - t0
        gc.callbacks.remove(on_gc)
        for key in ("cumulative", "tottime"):
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats(key).print_stats(22)
            print(f"== {key}\n" + buf.getvalue(), file=sys.stderr)
        print(json.dumps({"wall_s": wall, "split_s": dict(confidence.last_confidence_times.__dict__),
                          "gc_passes_ms": gc_ms}), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
