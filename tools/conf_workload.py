#!/usr/bin/env python3
"""Workload for rocprofv3 passes over the confidence kernel: the bench's C3 confidence leg (every
one of the C2 sequence's 500 frames as a reference frame, r = 10, depth_max 4, error 0.08),
device-resident depth in and maps out, one warm-up call then `--reps` calls."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--stats", action="store_true", help="also one counted call: pairs per deciding stage")
    ap.add_argument("--diag", action="store_true", help="also the timing-only build without tap loads")
    ap.add_argument("--ab", default="", help="comma list of mqr_confidence_stats modes to time against the "
                    "default (4 = the branchy float32 stages), each with its digest")
    a = ap.parse_args()
    import numpy as np
    import torch
    from mqr import _lib, synthetic
    seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
    d = seq["depth_t"].contiguous()
    B, H, W = d.shape
    T_cw = np.ascontiguousarray(seq["T_cw"], dtype=np.float32).reshape(B, 16)
    T_ci = np.ascontiguousarray(np.linalg.inv(seq["T_cw"]), dtype=np.float32).reshape(B, 16)
    K32 = np.ascontiguousarray(seq["K"], dtype=np.float32).reshape(B, 9)
    conf = torch.empty((B, H, W), dtype=torch.float64, device="cuda:0")
    valid = torch.empty((B, H, W), dtype=torch.int32, device="cuda:0")
    import hashlib
    import json
    import time
    times = []
    if os.environ.get("MQR_CONF_MODE"):  # counter passes over an A/B mode (mqr_confidence_stats)
        _lib.call("mqr_confidence_stats", 0, int(os.environ["MQR_CONF_MODE"], 0), None)
    for i in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.call("mqr_confidence", 0, ctypes.c_void_p(d.data_ptr()), 1, B, H, W, _lib.ptr(K32, _lib._f32p),
                  _lib.ptr(T_cw, _lib._f32p), _lib.ptr(T_ci, _lib._f32p), None, 0, B, 10, 4.0, 0.08,
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
        torch.cuda.synchronize()
        if i:
            times.append((time.perf_counter() - t0) * 1e3)
    digest = hashlib.sha256(conf.cpu().numpy().tobytes() + valid.cpu().numpy().tobytes()).hexdigest()[:16]
    vmean, cmean = float(valid.float().mean()), float(conf.mean())
    stages = None
    if a.stats:
        last = np.zeros(4, np.int64)
        _lib.call("mqr_confidence_stats", 0, 1, None)
        _lib.call("mqr_confidence", 0, ctypes.c_void_p(d.data_ptr()), 1, B, H, W, _lib.ptr(K32, _lib._f32p),
                  _lib.ptr(T_cw, _lib._f32p), _lib.ptr(T_ci, _lib._f32p), None, 0, B, 10, 4.0, 0.08,
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
        _lib.call("mqr_confidence_stats", 0, 0, _lib.ptr(last, _lib._i64p))
        stages = dict(zip(("pairs", "float32_prefilter", "float64_filter", "float64_backprojection"), last.tolist()))
    diag_ms = None
    if a.diag:
        _lib.call("mqr_confidence_stats", 0, 2, None)
        dt = []
        for i in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.call("mqr_confidence", 0, ctypes.c_void_p(d.data_ptr()), 1, B, H, W, _lib.ptr(K32, _lib._f32p),
                      _lib.ptr(T_cw, _lib._f32p), _lib.ptr(T_ci, _lib._f32p), None, 0, B, 10, 4.0, 0.08,
                      ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
            torch.cuda.synchronize()
            dt.append((time.perf_counter() - t0) * 1e3)
        _lib.call("mqr_confidence_stats", 0, 0, None)
        diag_ms = sorted(dt[1:])[1]
    ab = {}
    for mode in [int(x, 0) for x in a.ab.split(",") if x]:
        _lib.call("mqr_confidence_stats", 0, mode, None)
        conf.zero_()
        dt = []
        for i in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _lib.call("mqr_confidence", 0, ctypes.c_void_p(d.data_ptr()), 1, B, H, W, _lib.ptr(K32, _lib._f32p),
                      _lib.ptr(T_cw, _lib._f32p), _lib.ptr(T_ci, _lib._f32p), None, 0, B, 10, 4.0, 0.08,
                      ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
            torch.cuda.synchronize()
            if i:
                dt.append((time.perf_counter() - t0) * 1e3)
        _lib.call("mqr_confidence_stats", 0, 0, None)
        dg = hashlib.sha256(conf.cpu().numpy().tobytes() + valid.cpu().numpy().tobytes()).hexdigest()[:16]
        ab[mode] = {"ms_median": sorted(dt)[len(dt) // 2], "digest": dg, "same": dg == digest}
    rec = {"confidence_src": _lib.build_tag(1), "digest": digest}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "conf_workload.json"), "w") as f:
        json.dump(rec, f)
    print(json.dumps({"confidence_src": rec["confidence_src"], "ms_median": sorted(times)[len(times) // 2], "reps": a.reps, "valid_mean": vmean, "conf_mean": cmean, "digest": digest,
                      "single": os.environ.get("MQR_CONF_SINGLE") is not None, "stages": stages,
                      "no_tap_loads_ms": diag_ms, "ab": ab or None}))


if __name__ == "__main__":
    main()
