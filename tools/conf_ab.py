#!/usr/bin/env python3
"""A/B of the drop-in estimate_depth_confidences' map download on the bench's 500-frame on-disk capture
(the dropin_e2e leg's first half): the maps as (valid, consistent) byte pairs expanded by the npz writer
(confidence.COUNT_PAIRS = True) against the maps themselves (False), interleaved in one process, page cache
warm, a fresh output directory per call, dirty pages written back (os.sync) before each call.  Prints one JSON line: per mode the median seconds, the splits
(confidence.last_confidence_times), and whether the written files are identical between the modes."""
import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def _digest(d):
    h = hashlib.sha256()
    for name in sorted(os.listdir(d)):
        h.update(name.encode())
        with open(os.path.join(d, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=500)
    a = ap.parse_args()
    from mqr import confidence, synthetic
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(a.frames), device="cuda:0")
    cap = {"raw": seq["raw_t"].cpu().numpy(), "unity": seq["unity"], "tangents": seq["tangents"],
           "near": seq["near"], "far": seq["far"], "width": seq["width"], "height": seq["height"]}
    tmp = tempfile.mkdtemp(prefix="mqr_conf_ab_")
    try:
        synthetic.write_capture(tmp, cap)
        io_ = DepthDataIO(tmp)
        io_.load_depth_dataset(Side.LEFT)
        cfg = DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0, error_threshold=0.08,
                                              skip_if_output_dir_exists=False, device=0)
        out = os.path.join(tmp, "left_depth_confidence")
        res = {"pairs": [], "maps": []}
        splits = {"pairs": [], "maps": []}
        digests = {}
        for rnd in range(a.rounds + 1):
            for mode in (("pairs", "maps") if rnd % 2 == 0 else ("maps", "pairs")):
                confidence.COUNT_PAIRS = mode == "pairs"
                shutil.rmtree(out, ignore_errors=True)
                os.sync()  # every call starts without dirty pages from the previous ones (writeback throttling)
                t0 = time.perf_counter()
                estimate_depth_confidences(io_, cfg, sides=[Side.LEFT])
                dt = time.perf_counter() - t0
                if rnd == 0:  # warm-up round; the files of each mode are compared once
                    digests[mode] = _digest(out)
                    continue
                res[mode].append(dt)
                splits[mode].append(dict(confidence.last_confidence_times.__dict__))
        med = {m: sorted(v)[len(v) // 2] for m, v in res.items()}
        print(json.dumps({"frames": a.frames, "rounds": a.rounds, "median_s": med, "all_s": res, "splits_s": splits,
                          "files_identical": digests["pairs"] == digests["maps"]}), flush=True)
    finally:
        confidence.COUNT_PAIRS = True
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
