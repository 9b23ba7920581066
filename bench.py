#!/usr/bin/env python3
"""Benchmark of the TSDF fusion hot path (SURVEY.md §8(d) workload C2 at N=1).

A "step" = integrate the rank's whole 500-frame depth sequence (640x480, procedural room = a
512^3-voxel volume at 5 mm, R=16, depth_max 4 m, truncation 10 voxels) into an empty volume:
per batch of up to 127 frames one touch launch (hash insert) + one integrate launch, inputs resident in HBM.
With N > 1 ranks the step is BASELINE's C4 (configs[3]): the fixed 2000-frame LEFT+RIGHT capture
split over the ranks by contiguous frame ranges (strong scaling), each rank integrating its range,
then the single RCCL exchange (mqr_reduce_rccl, sharded: owned slice + halo per rank); the line
carries merge_phases_ms, the shards' parity against the oracle's pass over the whole capture, and
a weak C2-per-rank sub-leg (`weak_c2`).  If RCCL cannot start on every rank the line fails (exit
1, value null) -- no fallback transport is timed.

Prints ONE JSON line (rank 0): value = frames integrated per second over all ranks, the mesh
extraction time (weight_threshold 1.5, the pipeline's setting), the integrate kernel's roofline
(algorithmic bytes per launch / its average HIP-event duration), the CPU-oracle baseline and the
parity of the last timed step's volume, mesh and point cloud against the oracle's (checked before
any other leg touches the volume).  The C4 (2000 frames L+R chained) and C5 (4000 frames @ 3 mm +
colour) legs carry parity blocks of their own, on the volumes they timed.
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=5)
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
    ap.add_argument("--cpu1-seconds", type=float, default=8.0, help="bounded 1-thread CPU sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--conf-range", type=int, default=10, help="C3 confidence window r")
    ap.add_argument("--conf-depth-max", type=float, default=4.0)
    ap.add_argument("--conf-error", type=float, default=0.08)
    ap.add_argument("--no-extras", action="store_true", help="skip confidence / copy-peak / host-input legs")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle comparison of the timed volume")
    ap.add_argument("--conf-cpu-seconds", type=float, default=20.0,
                    help="bounded CPU sample of the confidence oracle (its maps are also the parity check)")
    ap.add_argument("--e2e-frames", type=int, default=500, help="frames of the on-disk C3 capture (0: skip the leg)")
    ap.add_argument("--merge", default="sharded", choices=["sharded", "root"],
                    help="N>1 volume merge inside libmqr over RCCL (mqr_reduce_rccl): owned slice + halo per "
                         "rank, or the whole volume on rank 0")
    ap.add_argument("--strong", action="store_true",
                    help="C4: a fixed 2000-frame LEFT+RIGHT capture (1000 + 1000, stereo baseline 0.064 m) "
                         "split over the ranks (strong scaling); the default for --gpus N > 1")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: C2 weak scaling (500 frames per rank) as the headline instead of the C4 split")
    ap.add_argument("--weak-steps", type=int, default=50,
                    help="N > 1 (C4 headline): timed steps of the weak C2-per-rank sub-leg (0: skip)")
    ap.add_argument("--strong-frames", type=int, default=1000, help="frames per side in --strong mode")
    ap.add_argument("--no-c5", action="store_true", help="skip the 1-GPU C5 leg (4000 frames @ 3 mm + colour)")
    ap.add_argument("--no-resident", action="store_true",
                    help="pass the timed step's frames as MQR_DEVICE (the caller stream waits for each pass's last "
                         "integrate) instead of MQR_DEVICE_RESIDENT (A/B)")
    ap.add_argument("--no-c4", action="store_true", help="skip the 1-GPU C4 leg (1000 + 1000 frames chained)")
    ap.add_argument("--touch-steps", type=int, default=20, help="profiled steps for touch_ms_per_launch (0: skip)")
    ap.add_argument("--c5-only", action="store_true",
                    help="run only the C5 leg and print its record (rocprof of the peak-HBM run)")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="--gpus N > 1 without WORLD_SIZE: overall limit on the N self-launched ranks (s)")
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, child=None, timeout=3000.0, out=None, grace=10.0):
    """`bench.py --gpus N` (N > 1) started without WORLD_SIZE: start N fresh rank processes of this
    script on this node (RANK = LOCAL_RANK = i, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free
    MASTER_PORT), relay rank 0's stdout (its JSON line) and return the worst exit code.  The parent
    imports no torch and touches no GPU (it starts children, it never execs).  When a rank fails, or
    `timeout` passes, the others are terminated (SIGTERM to each rank's process group, SIGKILL after
    `grace` s).  `child` replaces `[python, bench.py]` (the launcher test's stub)."""
    import signal
    import subprocess
    import threading
    out = out or sys.stdout
    cmd = list(child) if child else [sys.executable, "-u", os.path.abspath(__file__)]
    port = str(_free_port())
    procs = []
    printed = threading.Event()

    def relay(stream):
        for line in stream:
            out.write(line)
            out.flush()
            if line.lstrip().startswith("{"):
                printed.set()

    def stop_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass

    prev = signal.getsignal(signal.SIGTERM)
    signal.signal(signal.SIGTERM, lambda *_: (stop_all(signal.SIGTERM), sys.exit(143)))
    relay_thread = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", NODE_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            procs.append(subprocess.Popen(cmd + list(argv), env=env, start_new_session=True,
                                          stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))
            if r == 0:
                relay_thread = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
                relay_thread.start()
        t_end = time.monotonic() + timeout
        failed = timed_out = False
        while any(p.poll() is None for p in procs):
            if not failed and any(p.poll() not in (None, 0) for p in procs):
                failed = True
                bad = [(i, p.returncode) for i, p in enumerate(procs) if p.returncode not in (None, 0)]
                print(f"[bench launcher] rank(s) failed {bad}: terminating the others", file=sys.stderr, flush=True)
                stop_all(signal.SIGTERM)
                t_end = min(t_end, time.monotonic() + grace)
            elif time.monotonic() > t_end:
                if not (failed or timed_out):
                    timed_out = True
                    print(f"[bench launcher] {timeout:.0f} s limit: terminating the ranks", file=sys.stderr,
                          flush=True)
                    stop_all(signal.SIGTERM)
                    t_end = time.monotonic() + grace
                else:
                    stop_all(signal.SIGKILL)
            time.sleep(0.05)
        if relay_thread is not None:
            relay_thread.join(5.0)
    finally:
        stop_all(signal.SIGKILL)
        signal.signal(signal.SIGTERM, prev)
    codes = [p.returncode for p in procs]
    worst = 0
    for c in codes:
        c = 128 - c if c < 0 else c  # killed by a signal: 128 + signal number
        worst = max(worst, c)
    if timed_out:
        worst = max(worst, 124)
    if worst and not printed.is_set():
        out.write(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": n,
                              "error": f"self-launched ranks exited {codes}" + (" (time limit)" if timed_out else "")})
                  + "\n")
        out.flush()
    return worst


def _vmstat():
    """Host page-fault / huge-page / compaction counters (/proc/vmstat) around the host copies."""
    keys = ("thp_fault_alloc", "thp_fault_fallback", "compact_stall", "compact_fail", "compact_success",
            "pgfault", "pgmajfault")
    try:
        with open("/proc/vmstat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f) if k in keys}
    except OSError:
        return {}


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


def extract_phases(vbg, thr, reps):
    """VoxelBlockGrid._geom's steps timed one by one (ms): the extraction (result in HBM), the three host
    destination allocations, mqr_geom_copy (device -> host, 3 arrays), mqr_geom_free, and the release of
    the host arrays (not part of an extraction: the unmap of ~1 GB)."""
    import numpy as np
    from mqr import _lib
    out = []
    for _ in range(reps):
        ph = {}
        g = ctypes.c_void_p()
        t0 = time.perf_counter()
        _lib.call("mqr_extract_mesh", vbg.handle, float(thr), ctypes.byref(g))
        t1 = time.perf_counter()
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("mqr_geom_counts", g, ctypes.byref(nv), ctypes.byref(nt))
        pos = np.empty((nv.value, 3), np.float32)
        nrm = np.empty((nv.value, 3), np.float32)
        tri = np.empty((nt.value, 3), np.int32)
        t2 = time.perf_counter()
        _lib.call("mqr_geom_copy", g, _lib.ptr(pos), _lib.ptr(nrm), _lib.ptr(tri), _lib.MQR_HOST)
        t3 = time.perf_counter()
        _lib.call("mqr_geom_free", g)
        t4 = time.perf_counter()
        nbytes = pos.nbytes + nrm.nbytes + tri.nbytes
        ph = {"extract": (t1 - t0) * 1e3, "alloc": (t2 - t1) * 1e3, "copy": (t3 - t2) * 1e3,
              "free": (t4 - t3) * 1e3, "copy_gbs": nbytes / (t3 - t2) / 1e9}
        t5 = time.perf_counter()
        del pos, nrm, tri
        ph["release"] = (time.perf_counter() - t5) * 1e3
        out.append(ph)
    return out


def copy_peak_gbs(device, nbytes=2 << 30, reps=5):
    """Achievable HBM rate on this box: device-to-device copy (read + write bytes) / time."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(reps):
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2 * nbytes / (best * 1e-3) / 1e9


def confidence_leg(depth_t, K, T_wc, args, device):
    """C3: depth-confidence maps of every frame of the sequence (window r), device-resident
    inputs/outputs, one warm-up call (per-device stream and parameter buffers), then the median of 5
    calls; algorithmic bytes per ref frame = 4HW(1 + n_nb) + 12HW."""
    import numpy as np
    import torch
    from mqr import _lib
    B, H, W = depth_t.shape
    T_cw = np.linalg.inv(T_wc).astype(np.float32)
    T_cw_inv = np.linalg.inv(T_cw).astype(np.float32)
    K32 = np.ascontiguousarray(K, dtype=np.float32).reshape(B, 9)
    conf = torch.empty((B, H, W), dtype=torch.float64, device=device)
    valid = torch.empty((B, H, W), dtype=torch.int32, device=device)
    times = []
    for rep in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.call("mqr_confidence", int(device.index or 0), ctypes.c_void_p(depth_t.data_ptr()), 1, B, H, W,
                  _lib.ptr(K32, _lib._f32p), _lib.ptr(np.ascontiguousarray(T_cw.reshape(B, 16)), _lib._f32p),
                  _lib.ptr(np.ascontiguousarray(T_cw_inv.reshape(B, 16)), _lib._f32p), None, 0, B,
                  int(args.conf_range), float(args.conf_depth_max), float(args.conf_error),
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
        torch.cuda.synchronize()
        if rep:
            times.append(time.perf_counter() - t0)
    times.sort()
    t = times[len(times) // 2]
    n_nb = sum(min(B, i + args.conf_range + 1) - max(0, i - args.conf_range) - 1 for i in range(B))
    alg = 4 * H * W * (B + n_nb) + 12 * H * W * B
    return {"ref_frames": B, "window_r": args.conf_range, "ms": t * 1e3, "ref_frames_per_s": B / t,
            "alg_gbs": alg / t / 1e9, "depth_max": args.conf_depth_max, "error_threshold": args.conf_error,
            "binding": conf_binding(),
            "note": "mqr_confidence over all frames, device-resident depth in/out, wall time of the call"}, (conf, valid)


def conf_binding():
    """k_confidence's binding resource from the committed counter passes (tools/pmc_conf.sh over
    tools/conf_workload.py -> profiles/*_pmc_confidence.json): VALU issue share of the launch's
    cycles (fp64 instructions weighted at half rate), texture-addresser busy share, occupancy."""
    import glob
    tag = build_tag(1)
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_confidence.json")))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        d = rec.get("derived")
        if not d or rec.get("confidence_src") != tag:  # only a record of this build's kernel
            continue
        valu, ta = d.get("valu_issue_frac_f64_at_half_rate"), d.get("ta_busy_frac")
        bound = ("VALU issue (fp64 at half rate)" if valu is not None and (ta is None or valu >= ta)
                 else "vector-memory gather path (TA)")
        return {"bound": bound, "source": os.path.relpath(path, ROOT), "valu_issue_frac_f64_weighted": valu,
                "valu_issue_frac_f32_rate": d.get("valu_issue_frac_f32_rate"), "ta_busy_frac": ta,
                "f64_share_of_valu": d.get("f64_share_of_valu"),
                "waves_per_simd": d.get("waves_per_simd"),
                "note": "fractions of the k_confidence launch's GPU cycles (GRBM_GUI_ACTIVE / 8 XCDs) in the "
                        "counter run of the C3 workload"}
    return None


def ingest_leg(B, H, W, device):
    """Row f4: device decode of B raw NDC frames + validity + confidence mask (every frame masked),
    all buffers in HBM; algorithmic bytes = HW * (4 raw + 8 conf + 4 count + 4 out) per frame."""
    import numpy as np
    import torch
    from mqr import _lib
    g = torch.Generator(device=device).manual_seed(0)
    raw = torch.rand((B, H, W), generator=g, device=device)
    conf = torch.rand((B, H, W), generator=g, device=device, dtype=torch.float64)
    vc = torch.randint(0, 8, (B, H, W), generator=g, device=device, dtype=torch.int32)
    out = torch.empty_like(raw)
    nears = np.full(B, 0.1)
    fars = np.full(B, np.inf)
    strong = np.full(B, 3, np.uint8)
    has = np.ones(B, np.uint8)
    ok = np.zeros(B, np.uint8)
    times = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.call("mqr_decode_depth", int(device.index or 0), ctypes.c_void_p(raw.data_ptr()), 1, B, H, W,
                  _lib.ptr(nears, _lib._f64p), _lib.ptr(fars, _lib._f64p), _lib.ptr(strong, _lib._u8p),
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(vc.data_ptr()), _lib.ptr(has, _lib._u8p), 1,
                  0.3, 2, ctypes.c_void_p(out.data_ptr()), 1, _lib.ptr(ok, _lib._u8p))
        times.append(time.perf_counter() - t0)
    t = sorted(times[1:])[1]
    return {"frames": B, "ms": t * 1e3, "frames_per_s": B / t, "alg_gbs": 20 * H * W * B / t / 1e9,
            "note": "mqr_decode_depth, device raw/conf/count in, depth out, wall time of the call"}


def c3_leg(seq, vbg, args, device, reps=3, parity=True):
    """C3 on the device, inputs resident in HBM: decode the raw NDC stack (mqr_decode_depth), the
    confidence of every frame (mqr_confidence, r = conf_range), decode again with the confidence
    mask (0.02 / 2, o3d_utils.py:141-142) and integrate the masked frames -- the pipeline's
    estimate_depth_confidences -> integrate(use_confidence_filtered_depth=True) order."""
    import numpy as np
    import torch
    from mqr import _lib
    raw = seq["raw_t"].contiguous()
    B, H, W = raw.shape
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)
    T_cw = np.ascontiguousarray(seq["T_cw"], dtype=np.float32).reshape(B, 16)
    T_ci = np.ascontiguousarray(np.linalg.inv(seq["T_cw"]), dtype=np.float32).reshape(B, 16)
    K32 = np.ascontiguousarray(seq["K"], dtype=np.float32).reshape(B, 9)
    depth = torch.empty_like(raw)
    masked = torch.empty_like(raw)
    conf = torch.empty((B, H, W), dtype=torch.float64, device=device)
    valid = torch.empty((B, H, W), dtype=torch.int32, device=device)
    nears = np.full(B, seq["near"], np.float64)
    fars = np.full(B, seq["far"], np.float64)
    strong = np.full(B, 3, np.uint8)  # DepthDataset.nears / fars are numpy float64 scalars
    has = np.ones(B, np.uint8)
    ok = np.zeros(B, np.uint8)
    dev = int(device.index or 0)

    class _P:
        ptr = ctypes.c_void_p(masked.data_ptr())

    def run():
        _lib.call("mqr_decode_depth", dev, ctypes.c_void_p(raw.data_ptr()), 1, B, H, W, _lib.ptr(nears, _lib._f64p),
                  _lib.ptr(fars, _lib._f64p), _lib.ptr(strong, _lib._u8p), None, None, None, 1, 0.0, 0,
                  ctypes.c_void_p(depth.data_ptr()), 1, _lib.ptr(ok, _lib._u8p))
        _lib.call("mqr_confidence", dev, ctypes.c_void_p(depth.data_ptr()), 1, B, H, W, _lib.ptr(K32, _lib._f32p),
                  _lib.ptr(T_cw, _lib._f32p), _lib.ptr(T_ci, _lib._f32p), _lib.ptr(ok, _lib._u8p), 0, B,
                  int(args.conf_range), float(args.conf_depth_max), float(args.conf_error),
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), 1)
        _lib.call("mqr_decode_depth", dev, ctypes.c_void_p(raw.data_ptr()), 1, B, H, W, _lib.ptr(nears, _lib._f64p),
                  _lib.ptr(fars, _lib._f64p), _lib.ptr(strong, _lib._u8p), ctypes.c_void_p(conf.data_ptr()),
                  ctypes.c_void_p(valid.data_ptr()), _lib.ptr(has, _lib._u8p), 1, 0.02, 2,
                  ctypes.c_void_p(masked.data_ptr()), 1, _lib.ptr(ok, _lib._u8p))
        vbg.reset()
        vbg.integrate_frames((_P, B, H, W), K, T, frame_ok=ok, depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc)

    run()
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[len(times) // 2]
    out = {"frames": B, "ms": t * 1e3, "frames_per_s": B / t, "masked_fraction": float((masked == 0).float().mean()),
           "blocks": vbg.size(), "window_r": args.conf_range,
           "note": "device-resident raw NDC in: decode + confidence (all frames) + masked decode + integrate, "
                   "wall time, median of 3"}
    if parity:
        # the last run's outputs: the mask (o3d_utils.py:141-142 restated in torch on the leg's own decoded
        # depth and maps, bit for bit on the integrated frames), the confidence maps of sampled reference
        # frames against the oracle, and the masked volume against the oracle's volume of the same frames
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        okb = torch.from_numpy(ok.astype(bool)).to(device)
        want = torch.where((conf < 0.02) | (valid < 2), torch.zeros_like(depth), depth)
        mask_equal = bool(torch.equal(masked[okb].view(torch.int32), want[okb].view(torch.int32)))
        dh = depth.cpu().numpy()
        sample = sorted({0, 1, B // 4, B // 2, 3 * B // 4, B - 2, B - 1})
        conf_ok = True
        for i in sample:
            oc, ov = oracle.confidence(dh, K32.reshape(B, 3, 3), T_cw.reshape(B, 4, 4), T_ci.reshape(B, 4, 4), i,
                                       int(args.conf_range), float(args.conf_depth_max), float(args.conf_error),
                                       frame_valid=ok)
            conf_ok = conf_ok and bool(np.array_equal(valid[i].cpu().numpy(), ov)) and bool(
                np.array_equal(conf[i].cpu().numpy().view(np.uint64), oc.view(np.uint64)))
        del dh
        sel = np.flatnonzero(ok)
        mh = masked.cpu().numpy()[sel]
        ref = oracle_volume(mh, K[sel], T[sel], args.voxel, args)
        del mh
        out["parity"] = parity_check(vbg, ref, args.extract_threshold, points_thr=3.0)
        out["parity"]["mask_equal"] = mask_equal
        out["parity"]["confidence_frames_checked"] = sample
        out["parity"]["confidence_equal"] = conf_ok
        out["parity"]["all_ok"] = bool(out["parity"]["all_ok"] and mask_equal and conf_ok)
        del ref
    return out


def dropin_e2e_leg(seq, frames, device, fragment_workers=4):
    """The reference's own loop on disk: a C3 capture (raw NDC files + descriptor CSV) in a temp dir,
    mqr.confidence.estimate_depth_confidences writing the per-frame npz, then
    mqr.o3d_utils.integrate(use_confidence_filtered_depth=True) reading raw + npz back
    (o3d_utils.py:153-238 -> device decode / mask / batched integrate).  Page cache warm."""
    import shutil
    import tempfile
    import numpy as np
    from mqr import synthetic
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import CoordinateSystem, Side
    from mqr.o3d_utils import integrate
    cap = {"raw": seq["raw_t"][:frames].cpu().numpy(), "unity": seq["unity"], "tangents": seq["tangents"],
           "near": seq["near"], "far": seq["far"], "width": seq["width"], "height": seq["height"]}
    tmp = tempfile.mkdtemp(prefix="mqr_e2e_")
    try:
        synthetic.write_capture(tmp, cap)
        io = DepthDataIO(tmp)
        ds = io.load_depth_dataset(Side.LEFT)
        n = len(ds)
        cfg = DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0, error_threshold=0.08,
                                              skip_if_output_dir_exists=False, device=int(device.index or 0))
        from mqr import confidence as _conf
        t0 = time.perf_counter()
        estimate_depth_confidences(io, cfg, sides=[Side.LEFT])
        t_conf = time.perf_counter() - t0
        conf_split = dict(_conf.last_confidence_times.__dict__)
        # reconstruct_scene.py:27-53: confidences first (UNITY poses converted inside), then the
        # integrator gets the dataset with OPEN3D camera poses
        ds.transforms = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                                is_camera=True)
        kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2,
                  voxel_size=0.005, block_resolution=16, block_count=40000, depth_max=4.0,
                  trunc_voxel_multiplier=10.0, device=int(device.index or 0))
        integrate(ds, io, Side.LEFT, **kw)  # warm-up (allocations, page cache)
        from mqr import o3d_utils
        runs, splits = [], []
        for _ in range(5):  # median of 5: a single host-bound run varies by +-20 %
            t0 = time.perf_counter()
            vbg = integrate(ds, io, Side.LEFT, **kw)
            runs.append(time.perf_counter() - t0)
            splits.append(dict(o3d_utils.last_integrate_times.__dict__))
            blocks = vbg.size()
            del vbg
        t_int = float(np.median(runs))
        frag = fragments_leg(io, ds, fragment_workers) if fragment_workers > 0 else None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {"frames": n, "confidence_s": t_conf, "confidence_split_s": conf_split, "confidence_frames_per_s": n / t_conf, "integrate_s": t_int,
            "integrate_runs_s": runs, "integrate_splits_s": splits, "integrate_frames_per_s": n / t_int, "frames_per_s": n / (t_conf + t_int), "blocks": blocks,
            "fragments": frag,
            "note": "on-disk capture (raw + descriptor CSV), estimate_depth_confidences (writes npz) then "
                    "o3d_utils.integrate with confidence masking (median of 5 runs); host file I/O + PCIe included"}


def fragments_leg(io, ds, workers, fragment_size=100):
    """The fragment path (refine_fragment_poses.py:14-58, 81-90) on the same on-disk capture: 100-frame
    fragments, each into a FRESH volume (pipeline_config.yml:50-58: 1 cm, R 16, block_count 50 000,
    depth_max 4, trunc 10, confidence mask 0.02 / 2), then extract_point_cloud(); on a spawn Pool of
    `workers` processes sharing the GPU (warmed up before the timed run) and in-process; every
    fragment's points checked against the oracle's volume of the same masked frames."""
    import multiprocessing
    import numpy as np
    from mqr.fragments import (FragmentPoseRefinementConfig, _warm, fragment_datasets,
                               integrate_fragment_point_clouds)
    from mqr.models import Side
    from mqr.o3d_utils import _masked_depth, compute_o3d_intrinsic_matrices
    frags = fragment_datasets(ds, fragment_size)
    cfg = FragmentPoseRefinementConfig(device="CUDA:0", confidence_threshold=0.02, valid_count_threshold=2,
                                       voxel_size=0.01, block_count=50_000, depth_max=4.0, trunc_voxel_multiplier=10.0,
                                       use_multi_threading=True)
    os.environ["OMP_NUM_THREADS"] = "1"
    ctx = multiprocessing.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(processes=workers) as pool:
        pool.map(_warm, range(workers))  # spawn, import, HIP context per worker
        t_spawn = time.perf_counter() - t0
        integrate_fragment_point_clouds(io, {Side.LEFT: frags}, cfg, pool=pool)  # warm-up (first allocations)
        t0 = time.perf_counter()
        pooled = integrate_fragment_point_clouds(io, {Side.LEFT: frags}, cfg, pool=pool)
        t_pool = time.perf_counter() - t0
    cfg.use_multi_threading = False
    t0 = time.perf_counter()
    integrate_fragment_point_clouds(io, {Side.LEFT: frags}, cfg)
    t_seq = time.perf_counter() - t0
    out = {"fragments": len(frags), "fragment_frames": fragment_size, "workers": workers,
           "pool_spawn_s": t_spawn, "pool_s": t_pool, "fragments_per_s": len(frags) / t_pool,
           "sequential_s": t_seq, "sequential_fragments_per_s": len(frags) / t_seq,
           "points": [int(len(r[1])) if r else 0 for r in pooled],
           "note": "integrate_fragment_point_cloud on a spawn Pool sharing one GPU (one HIP context per worker), "
                   "from disk (raw + npz reads, device decode / mask), fresh 50 000-block volume per fragment, "
                   "extract_point_cloud(3.0) copied to the host"}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    from gpu_helpers import position_hashes
    cores, _ = host_cores()
    oracle.set_threads(cores)
    ok = True
    kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2)
    for fd, r in zip(frags, pooled):
        ref = oracle.OracleVBG(0.01, 16, 4096)
        K = compute_o3d_intrinsic_matrices(fd).astype(np.float64)
        T = fd.transforms.extrinsics_wc.astype(np.float64)
        for i in range(len(fd)):
            d = _masked_depth(io, Side.LEFT, i, fd, **kw)
            if d is not None:
                ref.integrate_frame(d, K[i], T[i], 1.0, 4.0, 10.0)
        op, _ = ref.extract_points(3.0)
        ok = ok and r is not None and len(r[1]) == len(op) and bool(
            np.array_equal(np.sort(position_hashes(r[1])), np.sort(position_hashes(op))))
    out["parity"] = {"all_ok": ok, "comparison": "per fragment: point positions as exact multisets (64-bit "
                                                 "position hashes) vs the oracle at weight 3.0"}
    return out


def c5_leg(args, device, frames_per_side=2000, voxel=0.003, key_every=40, parity=True):
    """C5 on one GPU (BASELINE.json configs[4] minus the 8-GPU split): a 2000 + 2000
    frame LEFT+RIGHT walk through an 8 x 8 x 3 m hall, 3 mm voxels (R = 16), integrated in
    reconstruct_scene.py's order (all LEFT, then all RIGHT) into one volume grown from a small
    capacity (multi-GB pool growth), the mesh extracted at 1.5, and per-vertex colour projected from
    every key_every-th frame's 640x480 colour image with ray-cast colour-aligned depth."""
    import numpy as np
    import torch
    from mqr import synthetic
    from mqr.color import color_map
    from mqr.raycasting import RaycastingScene
    from mqr.vbg import VoxelBlockGrid
    dev = int(device.index or 0)
    left = synthetic.hall_loop_poses(frames_per_side)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    poses = left + right
    t0 = time.perf_counter()
    seq = synthetic.make_sequence_fast("hall", poses=poses, height=args.height, width=args.width, seed=5,
                                       device=f"cuda:{dev}")
    depth = seq["depth_t"].contiguous()
    gen_s = time.perf_counter() - t0
    B, H, W = depth.shape
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)

    class _P:
        ptr = ctypes.c_void_p(depth.data_ptr())

    # pass 1: a fresh volume whose pool grows from 16384 blocks (reallocation + copy of the grown pool
    # inside the timed call); passes 2-3: the same volume emptied (vbg.reset keeps the grown pool),
    # with the integrate launches timed by HIP events for the roofline
    vbg = VoxelBlockGrid(voxel_size=voxel, block_resolution=16, block_count=16384, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vbg.integrate_frames((_P, B, H, W), K, T, depth_scale=1.0, depth_max=args.depth_max,
                         trunc_voxel_multiplier=args.trunc)
    torch.cuda.synchronize()
    t_grow = time.perf_counter() - t0
    vbg.stats(reset=True)
    vbg.profile(True)
    times = []
    for _ in range(2):
        vbg.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vbg.integrate_frames((_P, B, H, W), K, T, depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    vbg.profile(False)
    st = vbg.stats(reset=True)
    t_int = min(times)
    blocks = vbg.size()
    pool_gb = vbg.capacity() * 16 ** 3 * 8 / 1e9
    R3 = 16 ** 3
    launches = max(st["integrate_launches"], 1)
    alg = (16 * R3 * st["union_blocks"] + 4 * H * W * st["frames"] + 16 * st["frame_blocks"]) / launches
    avg_ms = st["integrate_ms"] / launches
    int_roof = {"bound": "hbm", "kernel": last_kernel_name(vbg), "unit": "GB/s", "peak": HBM_PEAK_GBS,
                "alg_bytes_per_launch": alg, "avg_launch_ms": avg_ms, "launches": st["integrate_launches"],
                "achieved": alg / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None,
                "union_blocks_per_launch": st["union_blocks"] / launches,
                "frame_blocks_per_frame": st["frame_blocks"] / max(st["frames"], 1),
                "note": "16 R^3 U + 4 H W k + 16 sum B_f per launch (SURVEY §8(d)) / mean HIP-event launch time "
                        "over the 2 timed passes"}
    int_roof["frac"] = int_roof["achieved"] / HBM_PEAK_GBS if int_roof["achieved"] else None
    # extraction on the device (the mqr_geom result stays in HBM), then the same with the host copy
    ext_dev_ms, (dnv, dnt) = extract_ms(vbg, 1.5, 3)
    ext_alg = 8 * R3 * blocks + 4 * 27 * blocks + 24 * dnv + 12 * dnt
    ext_roof = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS, "alg_bytes": ext_alg,
                "achieved": ext_alg / (ext_dev_ms * 1e-3) / 1e9, "frac": ext_alg / (ext_dev_ms * 1e-3) / 1e9 /
                HBM_PEAK_GBS, "note": "8 R^3 N + 108 N + 24 V + 12 T over the device-only extraction (median of 3)"}
    host = depth.cpu().numpy() if parity else None
    del depth, seq
    torch.cuda.empty_cache()
    ext = []
    vm0 = _vmstat()
    mesh = None
    for _ in range(3):
        mesh = None  # release the previous result (a ~1 GB unmap) outside the timed call
        t0 = time.perf_counter()
        mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
        _ = (mesh.vertices, mesh.vertex_normals, mesh.triangles)  # the host copies (the mesh is left in HBM)
        ext.append(time.perf_counter() - t0)
    vm1 = _vmstat()
    ext_phases = extract_phases(vbg, 1.5, 3)
    mesh_bytes = mesh.vertices.nbytes + mesh.vertex_normals.nbytes + mesh.triangles.nbytes
    key = list(range(0, B, key_every))
    Ko = K[0]
    imgs = synthetic.render_color_torch("hall", Ko, [poses[i] for i in key], H, W, device=f"cuda:{dev}").cpu().numpy()
    scene = RaycastingScene(device=dev)
    scene.add_triangles(mesh.vertices, mesh.triangles)
    from mqr import _lib
    t0 = time.perf_counter()
    _lib.call("mqr_scene_build", scene._h)
    bvh_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    cad = scene.cast_pinhole(K[key], T[key], W, H)["t_hit"].numpy()
    cast_s = time.perf_counter() - t0
    col_runs = []
    for _ in range(2):  # best of 2, like the device-resident calls below
        col = cnt = None
        t0 = time.perf_counter()
        col, cnt = color_map(mesh.vertices, imgs, cad, K[key], T[key], device=dev)
        col_runs.append(time.perf_counter() - t0)
    col_s = min(col_runs)
    # the same cast and colouring with every input and output resident in HBM (the kernels' own time;
    # the host-array calls above include the PCIe copies of ~0.8 GB)
    from mqr import _lib as _l
    nk = len(key)
    d_t = torch.empty(nk * H * W, dtype=torch.float32, device=f"cuda:{dev}")
    d_v = torch.from_numpy(np.ascontiguousarray(mesh.vertices, np.float32)).to(f"cuda:{dev}")
    d_im = torch.from_numpy(np.ascontiguousarray(imgs, np.uint8)).to(f"cuda:{dev}")
    d_col = torch.empty((len(mesh.vertices), 3), dtype=torch.float32, device=f"cuda:{dev}")
    d_cnt = torch.empty(len(mesh.vertices), dtype=torch.int32, device=f"cuda:{dev}")
    Kk = np.ascontiguousarray(K[key], np.float64)
    Tk = np.ascontiguousarray(T[key], np.float64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _l.call("mqr_scene_cast_pinhole", scene._h, _l.ptr(Kk, _l._f64p), _l.ptr(Tk, _l._f64p), nk, H, W,
            ctypes.c_void_p(d_t.data_ptr()), None, None, None, None, _l.MQR_DEVICE)
    cast_dev_s = time.perf_counter() - t0
    col_dev = []
    for _ in range(2):
        t0 = time.perf_counter()
        _l.call("mqr_color_map", dev, ctypes.c_void_p(d_v.data_ptr()), len(mesh.vertices), _l.MQR_DEVICE,
                ctypes.c_void_p(d_im.data_ptr()), ctypes.c_void_p(d_t.data_ptr()), _l.MQR_DEVICE, nk, H, W,
                _l.ptr(Kk, _l._f64p), _l.ptr(Tk, _l._f64p), 2.5, 0.03, 10, 0.1, 3, 3.0, 3,
                ctypes.c_void_p(d_col.data_ptr()), ctypes.c_void_p(d_cnt.data_ptr()), _l.MQR_DEVICE)
        col_dev.append(time.perf_counter() - t0)
    device_equal = bool(np.array_equal(d_t.cpu().numpy().reshape(cad.shape), cad) and
                        np.array_equal(d_col.cpu().numpy(), col) and np.array_equal(d_cnt.cpu().numpy(), cnt))
    del d_t, d_v, d_im, d_col, d_cnt
    # the whole colour tail as the pipeline runs it (project_vertex_colors: BVH, colour-view casts, colours):
    # on the mesh the extraction left in HBM, and on host arrays of the same mesh (every array over PCIe)
    from mqr.color import project_vertex_colors
    mesh_dev = vbg.extract_triangle_mesh(weight_threshold=1.5)
    mesh_host = mesh_dev.cpu()
    pipe = {"device_resident": [], "host_arrays": []}
    for _ in range(2):
        for name, m in (("device_resident", mesh_dev), ("host_arrays", mesh_host)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pc, pn = project_vertex_colors(m, imgs, K[key], T[key], device=dev)
            pipe[name].append(time.perf_counter() - t0)
            pipe_equal = bool(np.array_equal(pc, col) and np.array_equal(pn, cnt))
            if not pipe_equal:
                break
    del mesh_dev, mesh_host
    seen = cnt > 0
    err = float(np.abs(col[seen] - synthetic.texture(mesh.vertices[seen])).mean()) if seen.any() else None
    err_fill = (float(np.abs(col[~seen] - synthetic.texture(mesh.vertices[~seen])).mean()) if (~seen).any()
                else None)
    out = {"frames": B, "voxel_size": voxel, "integrate_ms": t_int * 1e3, "frames_per_s": B / t_int,
           "integrate_ms_with_growth": t_grow * 1e3, "roofline": int_roof,
           "blocks": blocks, "pool_gb": pool_gb, "extract_device_ms": ext_dev_ms, "extract_roofline": ext_roof,
           "extract_ms": sorted(ext)[1] * 1e3, "extract_runs_ms": [x * 1e3 for x in ext],
           "extract_vmstat_delta": {k: vm1[k] - vm0[k] for k in vm0 if k in vm1}, "extract_phases_ms": ext_phases,
           "extract_host_copy_bytes": mesh_bytes,
           "vertices": int(len(mesh.vertices)), "triangles": int(len(mesh.triangles)),
           "keyframes": len(key), "bvh_build_ms": bvh_s * 1e3, "colour_depth_cast_ms": cast_s * 1e3,
           "colour_ms": col_s * 1e3, "colour_runs_ms": [x * 1e3 for x in col_runs],
           "colour_pipeline_ms": {k: min(v) * 1e3 for k, v in pipe.items()}, "colour_pipeline_equal": pipe_equal, "colour_depth_cast_device_ms": cast_dev_s * 1e3,
           "colour_device_ms": min(col_dev) * 1e3, "colour_device_path_equal": device_equal,
           "coloured_fraction": float(seen.mean()), "colour_mean_abs_err": err,
           "colour_mean_abs_err_knn_filled": err_fill,
           "generation_s": gen_s,
           "note": "integrate: device-resident depth, best of 2 passes into the emptied volume whose pool the "
                   "first pass grew (integrate_ms_with_growth: that first pass, grown from 16384 blocks); "
                   "extract_device_ms: result left in HBM; extract_ms: host copy included, median of 3; "
                   "colour: mqr_color_map (boundary "
                   "masks, float64 means, 3-NN fill of unseen vertices), host arrays in/out (PCIe included; best of 2), error vs "
                   "the analytic texture the colour frames were rendered with; *_device_ms: the same cast / colouring "
                   "with inputs and outputs in HBM (colour: best of 2), results equal to the host-array calls"}
    if parity:
        # the volume of the last timed pass, its mesh (the one coloured above) and point cloud, and the
        # per-vertex colours, against the oracle on the same 4000 frames (LEFT then RIGHT)
        del scene
        log("C5 parity: oracle volume of the same frames")
        t0 = time.perf_counter()
        ref = oracle_volume(host, K, T, voxel, args, block_count=16384)
        out["oracle_s"] = time.perf_counter() - t0
        del host
        out["parity"] = parity_check(vbg, ref, 1.5, mesh=mesh, points_thr=3.0)
        del ref
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        oc, on = oracle.color_map(mesh.vertices, imgs, cad, K[key], T[key])
        out["parity"]["colour_counts_equal"] = bool(np.array_equal(cnt, on))
        out["parity"]["colours_equal"] = bool(np.array_equal(col, oc))
        out["parity"]["all_ok"] = bool(out["parity"]["all_ok"] and out["parity"]["colour_counts_equal"]
                                       and out["parity"]["colours_equal"])
        scene = None
    del vbg, mesh, scene
    torch.cuda.empty_cache()
    return out


def c5_sharded_leg(args, rank, world, dev, merge_fn, dist, parity=True, frames_per_side=2000, voxel=0.003,
                   key_every=40):
    """C5 in its multi-GPU form (BASELINE.json configs[4]; reconstruct_scene.py:64-122, 181-225): the
    2000 + 2000 frame hall walk at 3 mm (c5_leg's capture, seeded once, so every rank count shards the
    same frames) split over the ranks by contiguous frame ranges; each rank integrates its range into
    its own volume (pool grown from 16384 blocks by a first, untimed pass), ONE exchange (merge_fn:
    mqr_reduce_rccl, or the gloo-staged twin in a rehearsal) leaves every rank its owned slice of the
    block union plus a one-block halo, every rank extracts its owned cubes' mesh at 1.5
    (mqr_extract_mesh_owned) and colours its shard mesh from every key_every-th frame.  Colour-aligned
    depth: each rank casts the keyframe views against its shard mesh and the per-pixel MIN over ranks
    (an all-reduce over the gloo control plane, host-staged) is the cast against the whole mesh -- the
    triangles partition the mesh, and the closest hit of a union is the least of its parts'.  The
    3-NN fill of unseen vertices draws on the shard's own sampled vertices (the one deviation from
    colouring the concatenated mesh in one call).

    Parity (rank 0 gathers the owned slices point to point): the merged owned slices against the
    oracle's sequential pass over all 4000 frames (keys and weights exact, tsdf within 1e-4), the
    shard meshes' triangle count against the oracle mesh's, and every rank's colours bit for bit
    against the oracle's colour_map on the same shard vertices and reduced depth."""
    import numpy as np
    import torch
    from mqr import synthetic
    from mqr.color import color_map
    from mqr.distributed import extract_mesh_owned, shard_range
    from mqr.raycasting import RaycastingScene
    from mqr.vbg import VoxelBlockGrid
    H, W = args.height, args.width
    left = synthetic.hall_loop_poses(frames_per_side)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    poses = left + right
    B = len(poses)
    t0 = time.perf_counter()
    seq = synthetic.make_sequence_fast("hall", poses=poses, height=H, width=W, seed=5, device=f"cuda:{dev}")
    gen_s = time.perf_counter() - t0
    K, T = seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    lo, hi = shard_range(B, rank, world)
    host = seq["depth_t"].cpu().numpy() if (parity and rank == 0) else None
    part = seq["depth_t"][lo:hi].contiguous().clone()
    del seq
    torch.cuda.empty_cache()

    class _P:
        ptr = ctypes.c_void_p(part.data_ptr())

    vbg = VoxelBlockGrid(voxel_size=voxel, block_resolution=16, block_count=16384, device=dev)
    kw = dict(depth_scale=1.0, depth_max=args.depth_max, trunc_voxel_multiplier=args.trunc)
    vbg.integrate_frames((_P, hi - lo, H, W), K[lo:hi], T[lo:hi], **kw)  # grows the pool (untimed)

    def wall_max(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        e = torch.tensor([time.perf_counter() - t], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return r, float(e.item()) * 1e3

    def integrate():
        vbg.reset()
        vbg.integrate_frames((_P, hi - lo, H, W), K[lo:hi], T[lo:hi], **kw)

    _, int_ms = wall_max(integrate)
    stats = {}
    (out, owned), merge_ms = wall_max(lambda: merge_fn(vbg, stats))
    del vbg
    mesh, ext_ms = wall_max(lambda: extract_mesh_owned(out, owned, 1.5))
    key = list(range(0, B, key_every))
    imgs = synthetic.render_color_torch("hall", K[0], [poses[i] for i in key], H, W, device=f"cuda:{dev}").cpu().numpy()

    def cast():
        if len(mesh.triangles) == 0:
            return np.full((len(key), H, W), np.inf, np.float32)
        scene = RaycastingScene(device=dev)
        scene.add_triangles(mesh.vertices, mesh.triangles)
        return np.ascontiguousarray(scene.cast_pinhole(K[key], T[key], W, H)["t_hit"].numpy(), np.float32)

    cad_local, cast_ms = wall_max(cast)

    def reduce_min():
        t = torch.from_numpy(cad_local)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return t.numpy()

    cad, reduce_ms = wall_max(reduce_min)
    def colour():
        if len(mesh.vertices) == 0:
            return np.zeros((0, 3), np.float32), np.zeros(0, np.int32)
        return color_map(mesh.vertices, imgs, cad, K[key], T[key], device=dev)

    (col, cnt), col_ms = wall_max(colour)
    st = torch.tensor([len(mesh.triangles), len(mesh.vertices), owned, stats.get("sent_bytes", 0),
                       stats.get("recv_bytes", 0)], dtype=torch.float64)
    allst = [torch.zeros_like(st) for _ in range(world)]
    dist.all_gather(allst, st)
    allst = torch.stack(allst)
    rec = {"frames": B, "voxel_size": voxel, "frames_per_gpu": [shard_range(B, r, world)[1] - shard_range(B, r, world)[0]
                                                               for r in range(world)],
           "integrate_ms_max": int_ms, "merge_ms_max": merge_ms, "frames_per_s": B / ((int_ms + merge_ms) * 1e-3),
           "extract_owned_ms_max": ext_ms, "colour_depth_cast_ms_max": cast_ms, "colour_depth_min_reduce_ms": reduce_ms,
           "colour_ms_max": col_ms, "triangles": int(allst[:, 0].sum()),
           "vertices_with_boundary_copies": int(allst[:, 1].sum()), "union_blocks": int(allst[:, 2].sum()),
           "merge_max_sent_bytes": float(allst[:, 3].max()), "merge_max_recv_bytes": float(allst[:, 4].max()),
           "keyframes": len(key), "generation_s": gen_s,
           "note": "frames_per_s = 4000 / (integrate + merge), each the max over ranks of a barrier-bracketed "
                   "wall time; extraction (host copy of the shard mesh included), colour-view casts, the "
                   "host-staged MIN all-reduce of the cast depth and the colouring timed after it"}
    if parity:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle
        from gpu_helpers import _key_order
        cores, _ = host_cores()
        # every rank's colours vs the oracle on the same inputs (ranks share the host cores)
        oracle.set_threads(max(1, cores // world))
        if len(mesh.vertices):
            oc, on = oracle.color_map(mesh.vertices, imgs, cad, K[key], T[key])
            col_ok = bool(np.array_equal(col, oc) and np.array_equal(cnt, on))
            del oc, on
        else:
            col_ok = True
        k_, t_, w_ = out.export()
        k_, t_, w_ = k_[:owned], t_[:owned], w_[:owned]
        R3 = 16 ** 3
        if rank == 0:
            log("C5 sharded parity: oracle pass over the whole capture")
            oracle.set_threads(cores)
            ref = oracle_volume(host, K, T, voxel, args, block_count=16384)
            del host
            ok_, ot, ow = ref.export()
            _, _, otri = ref.extract_mesh(1.5)
            n_otri = len(otri)
            del ref, otri
            oa = _key_order(ok_)
            ok_, ot, ow = ok_[oa], ot[oa].reshape(-1, R3), ow[oa].reshape(-1, R3)
            okp = (ok_[:, 0].astype(np.int64) + (1 << 20)) << 42 | (ok_[:, 1].astype(np.int64) + (1 << 20)) << 21 | \
                (ok_[:, 2].astype(np.int64) + (1 << 20))
            seen, weq, err, flips, flip_max = 0, True, 0.0, 0, 0.0
            parts = []  # every rank's owned slice: the merged volume, for the oracle's extraction of it
            for r in range(world):
                if r == 0:
                    rk, rt, rw = k_, t_.reshape(-1, R3), w_.reshape(-1, R3)
                else:
                    n = torch.zeros(1, dtype=torch.int64)
                    dist.recv(n, src=r)
                    n = int(n.item())
                    rk, rt, rw = torch.empty((n, 3), dtype=torch.int32), torch.empty((n, R3)), torch.empty((n, R3))
                    for x in (rk, rt, rw):
                        dist.recv(x, src=r)
                    rk, rt, rw = rk.numpy(), rt.numpy(), rw.numpy()
                rp = (rk[:, 0].astype(np.int64) + (1 << 20)) << 42 | (rk[:, 1].astype(np.int64) + (1 << 20)) << 21 | \
                    (rk[:, 2].astype(np.int64) + (1 << 20))
                j = np.searchsorted(okp, rp)
                found = (j < len(okp)) & (okp[np.minimum(j, len(okp) - 1)] == rp)
                if not found.all():
                    weq = False
                    break
                seen += len(rp)
                parts.append((rk, rt, rw))
                for c in range(0, len(j), 4096):
                    jj = j[c:c + 4096]
                    weq = weq and bool(np.array_equal(rw[c:c + 4096], ow[jj]))
                    m = rw[c:c + 4096] > 0
                    if m.any():
                        a, b = rt[c:c + 4096][m], ot[jj][m]
                        err = max(err, float(np.abs(a - b).max()))
                        # voxels whose tsdf sign differs (the marching-cubes classification): the merge's
                        # sum of partial averages rounds differently from the sequential running average
                        f = ((a < 0) != (b < 0)) | ((a > 0) != (b > 0))
                        if f.any():
                            flips += int(f.sum())
                            flip_max = max(flip_max, float(np.maximum(np.abs(a[f]), np.abs(b[f])).max()))
            keys_ok = weq and seen == len(okp)
            del ok_, ot, ow, okp
            # the oracle's marching cubes over the merged volume itself (the owned slices put together):
            # equal to the shard meshes' summed triangle count when the owned-cube extraction is exact, so
            # any difference from the oracle's own mesh lies in the merged tsdf, not in the extraction
            n_mtri = -1
            if parts:
                mv = oracle.OracleVBG(voxel, 16, sum(len(q[0]) for q in parts))
                mv.import_blocks(np.concatenate([q[0] for q in parts]), np.concatenate([q[1] for q in parts]),
                                 np.concatenate([q[2] for q in parts]))
                del parts
                n_mtri = len(mv.extract_mesh(1.5)[2])
                del mv
            res = torch.tensor([float(keys_ok), float(weq), err, float(n_otri), float(flips), flip_max,
                                float(n_mtri)], dtype=torch.float64)
        else:
            dist.send(torch.tensor([len(k_)], dtype=torch.int64), dst=0)
            for x in (k_, t_.reshape(-1, R3), w_.reshape(-1, R3)):
                dist.send(torch.from_numpy(np.ascontiguousarray(x)), dst=0)
            res = torch.zeros(7, dtype=torch.float64)
        del k_, t_, w_
        dist.broadcast(res, src=0)
        cok = torch.tensor([1 if col_ok else 0], dtype=torch.int32)
        dist.all_reduce(cok, op=dist.ReduceOp.MIN)
        tri_ok = int(res[3].item()) == rec["triangles"]
        flips, flip_max = int(res[4].item()), float(res[5].item())
        merged_exact = int(res[6].item()) == rec["triangles"]
        rec["parity"] = {"keys_equal": bool(res[0].item()), "weights_equal": bool(res[1].item()),
                         "max_dtsdf": float(res[2].item()), "tolerance": 1e-4,
                         "oracle_triangles": int(res[3].item()), "triangle_count_equal": tri_ok,
                         "triangle_count_diff": rec["triangles"] - int(res[3].item()),
                         "tsdf_sign_flips": flips, "max_abs_tsdf_at_sign_flips": flip_max,
                         "oracle_triangles_of_merged_volume": int(res[6].item()),
                         "merged_mesh_count_exact": merged_exact,
                         "colours_equal": bool(cok.item()),
                         "comparison": "owned slices of the merged shards vs the oracle's sequential pass over all "
                                       "4000 frames (keys / weights exact, tsdf within tolerance), shard triangle counts "
                                       "summed vs the oracle mesh at 1.5 (exact, or: exactly the oracle's extraction of "
                                       "the merged owned slices, and every voxel whose tsdf sign differs from the oracle's "
                                       "within the tolerance of 0), every rank's colours and counts bit for bit vs "
                                       "oracle.color_map on its shard vertices with the reduced colour-view depth"}
        # the triangle count is exact unless the merge's rounding moved a voxel's tsdf across 0 -- then
        # the shard meshes must be exactly the oracle's mesh of the merged volume, and every such voxel must
        # lie within the tolerance of 0 (its sign is not determined at 1e-4)
        rec["parity"]["triangle_count_explained"] = bool(merged_exact and (tri_ok or (flips > 0 and flip_max <= 1e-4)))
        rec["parity"]["all_ok"] = bool(rec["parity"]["keys_equal"] and rec["parity"]["weights_equal"]
                                       and rec["parity"]["max_dtsdf"] <= 1e-4 and rec["parity"]["triangle_count_explained"]
                                       and rec["parity"]["colours_equal"])
    del out, mesh, part
    torch.cuda.empty_cache()
    return rec


def c4_leg(args, device, frames_per_side=1000, reps=3, parity=True):
    """C4 on one GPU (BASELINE.json configs[3], the N = 1 point): 1000 LEFT + 1000 RIGHT frames of
    the room walk (0.064 m stereo baseline), 640x480, 5 mm, integrated as reconstruct_scene.py:64-81
    does -- one integrate call per side into ONE volume (vbg_opt threaded through).  Inputs
    resident in HBM; best of `reps` passes from an emptied volume; the last pass's volume, its mesh
    at 1.5 and its point cloud at 3.0 are checked against the oracle's volume of the same frames."""
    import numpy as np
    import torch
    from mqr.vbg import VoxelBlockGrid
    dev = int(device.index or 0)
    seq = c4_capture(args, dev, frames_per_side)
    depth = seq["depth_t"].contiguous()
    B, H, W = depth.shape
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)
    n = frames_per_side

    class _L:
        ptr = ctypes.c_void_p(depth.data_ptr())

    class _R:
        ptr = ctypes.c_void_p(depth[n:].data_ptr())

    vbg = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=args.block_resolution, block_count=args.block_count,
                         device=dev)
    times = []
    for _ in range(reps + 1):
        vbg.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vbg.integrate_frames((_L, n, H, W), K[:n], T[:n], depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc)
        vbg.integrate_frames((_R, B - n, H, W), K[n:], T[n:], depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = min(times[1:])
    mesh = vbg.extract_triangle_mesh(weight_threshold=args.extract_threshold)
    out = {"frames": B, "sides": [n, B - n], "ms": t * 1e3, "frames_per_s": B / t, "blocks": vbg.size(),
           "triangles": int(len(mesh.triangles)),
           "note": "2 integrate_frames calls (LEFT, RIGHT) into one volume, device-resident depth, best of "
                   f"{reps} passes after a warm-up pass"}
    if parity:
        host = depth.cpu().numpy()
        del depth, seq
        t0 = time.perf_counter()
        ref = oracle_volume(host, K, T, args.voxel, args)
        out["oracle_s"] = time.perf_counter() - t0
        out["parity"] = parity_check(vbg, ref, args.extract_threshold, mesh=mesh, points_thr=3.0)
        del ref
    del vbg, mesh
    torch.cuda.empty_cache()
    return out


def raycast_leg(vbg, K, T, H, W, thr, frames=64):
    """Row f1: colour-aligned depth by ray casting the extracted mesh (RaycastingScene.cast_rays
    stand-in): BVH build + `frames` pinhole casts at H x W from the sequence's poses."""
    import numpy as np
    from mqr.raycasting import RaycastingScene
    m = vbg.extract_triangle_mesh(weight_threshold=thr)
    scene = RaycastingScene(device=vbg.device_id)
    scene.add_triangles(m.vertices, m.triangles)
    from mqr import _lib
    t0 = time.perf_counter()
    _lib.call("mqr_scene_build", scene._h)
    first_build_ms = (time.perf_counter() - t0) * 1e3
    # a second scene of the same mesh: the build without the process's one-time costs (the sort kernels'
    # code objects loaded on their first launch, first allocations)
    scene2 = RaycastingScene(device=vbg.device_id)
    scene2.add_triangles(m.vertices, m.triangles)
    t0 = time.perf_counter()
    _lib.call("mqr_scene_build", scene2._h)
    build_ms = (time.perf_counter() - t0) * 1e3
    del scene2
    idx = np.linspace(0, len(K) - 1, frames).astype(int)
    scene.cast_pinhole(K[idx[:4]], T[idx[:4]], W, H)  # warm-up
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        out = scene.cast_pinhole(K[idx], T[idx], W, H)["t_hit"].numpy()
        times.append(time.perf_counter() - t0)
    t = sorted(times)[1]
    return {"triangles": int(m.triangles.shape[0]), "bvh_build_ms": build_ms, "bvh_first_build_ms": first_build_ms,
            "frames": frames,
            "frames_per_s": frames / t, "mrays_per_s": frames * H * W / t / 1e6,
            "hit_fraction": float(np.isfinite(out).mean()),
            "note": "mqr_scene_cast_pinhole, t_hit copied to host (PCIe included), median of 3; bvh_build_ms: a "
                    "second scene's build, bvh_first_build_ms: the process's first (one-time code-object loads)"}


def meshfilter_leg(vbg, thr, min_count=2000, reps=3):
    """Row f3: filter_mesh_components (o3d_utils.py:241-321) on the extracted mesh, device-resident
    input (the extraction's own buffers), result left on the device."""
    import ctypes
    import numpy as np
    from mqr import _lib
    m = vbg.extract_triangle_mesh(weight_threshold=thr)
    nv, nt = int(m.vertices.shape[0]), int(m.triangles.shape[0])
    import torch
    dev = torch.device("cuda", vbg.device_id)
    v = torch.from_numpy(np.ascontiguousarray(m.vertices)).to(dev)
    n = torch.from_numpy(np.ascontiguousarray(m.vertex_normals)).to(dev)
    t = torch.from_numpy(np.ascontiguousarray(m.triangles, dtype=np.int32)).to(dev)
    torch.cuda.synchronize()
    stats = np.zeros(8, np.int64)
    times = []
    for _ in range(reps + 1):
        g = ctypes.c_void_p()
        t0 = time.perf_counter()
        _lib.call("mqr_mesh_filter_components", vbg.device_id, ctypes.c_void_p(v.data_ptr()),
                  ctypes.c_void_p(n.data_ptr()), nv, ctypes.c_void_p(t.data_ptr()), nt, 1, min_count,
                  ctypes.byref(g), _lib.ptr(stats, _lib._i64p))
        times.append(time.perf_counter() - t0)
        _lib.call("mqr_geom_free", g)
    ms = sorted(times[1:])[len(times[1:]) // 2] * 1e3
    return {"triangles_in": nt, "vertices_in": nv, "clusters": int(stats[1]), "kept_clusters": int(stats[2]),
            "triangles_out": int(stats[6]), "min_triangle_count": min_count, "ms": ms,
            "mtris_per_s": nt / ms / 1e3,
            "note": "mqr_mesh_filter_components, device-resident mesh in/out, wall time of the call, median"}


def last_kernel_name(vbg):
    """The main kernel of the volume's last integrate launch (mqr_vbg_last_kernel_name)."""
    from mqr import _lib
    buf = ctypes.create_string_buffer(64)
    _lib.call("mqr_vbg_last_kernel_name", vbg.handle, buf, 64)
    return buf.value.decode()


def build_tag(which):
    from mqr import _lib
    try:
        return _lib.build_tag(which)
    except Exception:  # noqa: BLE001
        return None


def pmc_traffic(H, W, frames, variant_ran):
    """HBM bytes per integrate launch from the committed rocprofv3 --pmc passes of this workload
    (tools/traffic_workload.py + tools/pmc_summary.py; FETCH_SIZE/WRITE_SIZE calibrated on k_pack).
    Quoted only from a record of THIS build's integrate sources (mqr_build_tag) and kernel variant:
    a record of another kernel would describe a kernel that did not run (then None)."""
    import glob
    tag = build_tag(0)
    recs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    for path in reversed(recs):
        try:
            rec = json.load(open(path))
            wl = rec["workload"]
            if (wl["H"], wl["W"], wl["frames"]) == (H, W, frames) and rec.get("integrate_src") == tag and \
                    rec.get("variant_ran") == variant_ran:
                return rec["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, f"no counter record of this build (integrate_src {tag}, variant {variant_ran})"


def gather_ceiling(avg_launch_ms, gathers_per_launch, cus, pattern="brick_x2"):
    """The integrate launch against the measured depth-read ceiling (tools/gather_ceiling.hip ->
    profiles/*_gather_ceiling.jsonl): `pattern` is the kernel's lane map reading what the default
    kernel reads ("brick_x2": each lane the aligned 8-byte window of its pixel; "brick": dword
    gathers) from an L2-resident frame with no other work.  One read instruction per 64 voxel-frames."""
    import glob
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_gather_ceiling.jsonl")))):
        try:
            rows = [json.loads(x) for x in open(path) if x.strip()]
        except (OSError, ValueError):
            continue
        ceil = {r["pattern"]: r["ns_per_gather_instr_per_cu"] for r in rows}
        if pattern not in ceil or not avg_launch_ms or not gathers_per_launch:
            continue
        achieved = avg_launch_ms * 1e6 / (gathers_per_launch / cus)
        return {"unit": "ns per depth-read instruction per CU", "achieved": achieved, "ceiling": ceil[pattern],
                "frac": ceil[pattern] / achieved, "pattern": pattern, "gathers_per_launch": gathers_per_launch,
                "ceiling_dword_gathers": ceil.get("brick"), "ceiling_16B_windows": ceil.get("brick_x4"),
                "source": os.path.relpath(path, ROOT)}
    return None


def pmc_binding(avg_launch_ms, variant_ran):
    """The integrate kernel's binding resource from the committed rocprofv3 counter passes of the
    default kernel (tools/pmc_ab.sh -> profiles/*_pmc_integrate_counters.json, entry "v0:..."):
    busy fractions of the texture addresser (TA), L1 tag lookups per CU-cycle, VALU issue share.
    The counters are per launch of this same workload; the live launch time rescales the rate."""
    import glob
    tag = build_tag(0)
    for path in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_integrate_counters.json")))):
        try:
            rec = json.load(open(path))
        except (OSError, ValueError):
            continue
        for name, r in rec.items():
            d = r.get("derived")
            # only the default variant's counters of THIS build's integrate sources
            if not name.startswith("v0:") or not d or r.get("integrate_src") != tag or \
                    r.get("variant_ran") != variant_ran:
                continue
            live_cycles = avg_launch_ms * 1e-3 * d["clock_ghz"] * 1e9 if avg_launch_ms else None
            return {"bound": "vector-memory gather path (TA address / TCP tag lookups)",
                    "kernel": name[3:].strip(), "source": os.path.relpath(path, ROOT),
                    "ta_busy_frac": d["ta_busy_frac"], "tcp_lookups_per_cu_cycle": d["tcp_lookups_per_cu_cycle"],
                    "valu_issue_frac": d["valu_issue_frac"],
                    "tcp_lookups_per_launch": r.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
                    "tcp_lookups_per_cu_cycle_live": (r.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / 256 / live_cycles
                                                      if live_cycles else None),
                    "note": "fractions of the launch's GPU cycles (GRBM_GUI_ACTIVE) in the counter run; "
                            "diagnostic builds (tools/diag_integrate.sh): no gathers 0.20 ms, no update ~0.34 "
                            "of ~0.35 ms -- the gathers, not HBM or VALU, set the time (DESIGN.md §4)"}
    return None


def host_cores():
    """Threads this job can run at once: the affinity set, capped by a cgroup CPU quota if any."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use = min(aff, quota) if quota else aff
    return use, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "cpu_model": model}


def cpu_baseline(seq_host, K, T, args):
    """The oracle (oracle/mqr_oracle.c, OpenMP over blocks) over whole passes of the sequence, a
    fresh volume each like a bench step, for ~cpu_seconds.  Returns (record, last full volume)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker / CPU restatement (port) -- timed here as the baseline only
    cores, info = host_cores()
    oracle.set_threads(cores)
    t0 = time.perf_counter()
    n = passes = 0
    last = None
    while time.perf_counter() - t0 < args.cpu_seconds or last is None:
        ref = oracle.OracleVBG(args.voxel, args.block_resolution, args.block_count)
        for i in range(len(seq_host)):
            ref.integrate_frame(seq_host[i], K[i], T[i], 1.0, args.depth_max, args.trunc)
        n += len(seq_host)
        passes += 1
        last = ref
    dt = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "frames/s", "cores": cores, "kind": "port",
           "sample": f"{passes} pass(es) over the {len(seq_host)}-frame sequence ({n} frames), touch+integrate per "
                     f"frame (oracle/mqr_oracle.c, OpenMP over blocks, {cores} threads), {dt:.1f} s", **info}
    if args.cpu1_seconds > 0:
        oracle.set_threads(1)
        ref1 = oracle.OracleVBG(args.voxel, args.block_resolution, args.block_count)
        t0 = time.perf_counter()
        n1 = 0
        while n1 < len(seq_host) and time.perf_counter() - t0 < args.cpu1_seconds:
            ref1.integrate_frame(seq_host[n1], K[n1], T[n1], 1.0, args.depth_max, args.trunc)
            n1 += 1
        dt1 = time.perf_counter() - t0
        out["one_thread"] = {"value": n1 / dt1, "frames": n1, "seconds": dt1}
        oracle.set_threads(cores)
    return out, last


def parity_check(vbg, ref, thr, mesh=None, points_thr=None):
    """A GPU volume (and its mesh at `thr`, and optionally its point cloud at `points_thr`) vs the
    oracle's volume of the same frames: identical block keys and weights, |dtsdf| <= 1e-4 on w > 0,
    identical vertex-position and oriented-triangle multisets (tests/gpu_helpers.py)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from gpu_helpers import _key_order, mesh_signature, position_hashes
    gk, gt, gw = vbg.export()
    ok_, ot, ow = ref.export()
    out = {"blocks": int(len(gk))}
    ga, oa = _key_order(gk), _key_order(ok_)
    keys_equal = gk.shape == ok_.shape and bool(np.array_equal(gk[ga], ok_[oa]))
    out["keys_equal"] = keys_equal
    if keys_equal:
        weq, err = True, 0.0
        for c in range(0, len(ga), 4096):
            i, j = ga[c:c + 4096], oa[c:c + 4096]
            w1, w2 = gw[i], ow[j]
            weq = weq and bool(np.array_equal(w1, w2))
            m = w1 > 0
            if m.any():
                err = max(err, float(np.abs(gt[i][m] - ot[j][m]).max()))
        out["weights_equal"], out["max_dtsdf"] = weq, err
    del gt, gw, ot, ow
    if mesh is None:
        mesh = vbg.extract_triangle_mesh(weight_threshold=thr)
    ov, _, otri = ref.extract_mesh(thr)
    out["mesh_threshold"] = thr
    out["triangles"] = int(len(mesh.triangles))
    out["triangle_count_equal"] = len(mesh.triangles) == len(otri)
    out["vertex_count_equal"] = len(mesh.vertices) == len(ov)
    if out["triangle_count_equal"] and out["vertex_count_equal"]:
        gs, os_ = mesh_signature(mesh.vertices, mesh.triangles), mesh_signature(ov, otri)
        out["vertices_equal"] = bool(np.array_equal(gs[0], os_[0]))
        out["triangles_equal"] = bool(np.array_equal(gs[1], os_[1]))
    del ov, otri
    ok_pts = True
    if points_thr is not None:
        pcd = vbg.extract_point_cloud(weight_threshold=points_thr)
        op, on = ref.extract_points(points_thr)
        hg, ho = position_hashes(pcd.points), position_hashes(op)
        out["points"] = {"weight_threshold": points_thr, "count": int(len(op)),
                         "count_equal": len(op) == len(pcd.points)}
        if out["points"]["count_equal"]:
            og, oo = np.argsort(hg, kind="stable"), np.argsort(ho, kind="stable")
            out["points"]["positions_equal"] = bool(np.array_equal(hg[og], ho[oo]))
        ok_pts = bool(out["points"].get("positions_equal"))
    out["tolerance"] = 1e-4
    out["comparison"] = ("keys/weights exact, tsdf within tolerance, mesh and points as exact multisets of 64-bit "
                         "position hashes (order-independent)")
    out["all_ok"] = bool(out.get("keys_equal") and out.get("weights_equal") and out.get("max_dtsdf", 1) <= 1e-4
                         and out.get("triangles_equal") and out.get("vertices_equal") and ok_pts)
    return out


def oracle_volume(depth_host, K, T, args_voxel, args, block_count=4096):
    """The oracle's volume of the same frames, one by one (touch + integrate per frame)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker only
    cores, _ = host_cores()
    oracle.set_threads(cores)
    ref = oracle.OracleVBG(args_voxel, args.block_resolution, block_count)
    for i in range(len(depth_host)):
        ref.integrate_frame(depth_host[i], K[i], T[i], 1.0, args.depth_max, args.trunc)
    return ref


def confidence_cpu(depth_host, K, T_wc, args, budget_s, gpu_maps=None):
    """CPU baseline of the confidence leg: the oracle's build_confidence_map restatement (fp64,
    OpenMP over pixels) on as many reference frames as fit in ~budget_s.  Every oracle map computed
    is also compared bit for bit with the GPU leg's (conf, valid) of that frame (`parity`)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cores, _ = host_cores()
    oracle.set_threads(cores)
    T_cw = np.linalg.inv(T_wc).astype(np.float32)
    Ti = np.linalg.inv(T_cw).astype(np.float32)
    n = len(depth_host)
    t0 = time.perf_counter()
    done = 0
    cmp_s = 0.0
    veq = ceq = True
    bad = []
    for i in np.linspace(0, n - 1, n).astype(int)[np.random.default_rng(0).permutation(n)]:
        oc, ov = oracle.confidence(depth_host, K, T_cw, Ti, int(i), args.conf_range, args.conf_depth_max,
                                   args.conf_error)
        done += 1
        if gpu_maps is not None:  # the comparison is not part of the timed baseline
            tc = time.perf_counter()
            gv = gpu_maps[1][int(i)].cpu().numpy()
            gc = gpu_maps[0][int(i)].cpu().numpy()
            v_ok, c_ok = bool(np.array_equal(gv, ov)), bool(np.array_equal(gc.view(np.uint64), oc.view(np.uint64)))
            veq, ceq = veq and v_ok, ceq and c_ok
            if not (v_ok and c_ok) and len(bad) < 16:
                bad.append(int(i))
            cmp_s += time.perf_counter() - tc
        if time.perf_counter() - t0 - cmp_s > budget_s:
            break
    dt = time.perf_counter() - t0 - cmp_s
    out = {"value": done / dt, "unit": "ref frames/s", "cores": cores, "kind": "port",
           "sample": f"{done} random reference frames of the sequence (r = {args.conf_range}), oracle.confidence "
                     f"(oracle/mqr_oracle.c, OpenMP over pixels), {dt:.1f} s"}
    parity = None
    if gpu_maps is not None:
        parity = {"frames_compared": done, "frames_total": n, "valid_equal": veq, "conf_equal": ceq,
                  "mismatched_frames": bad, "all_ok": bool(veq and ceq and done > 0),
                  "comparison": "valid_count (int32) and confidence (float64 bit patterns) of every reference frame "
                                "the CPU baseline computed, against the GPU leg's maps of the same call"}
    return out, parity


def log(msg):
    """Progress on stderr (long legs must not look hung to a supervisor watching the output)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def c4_capture(args, dev, frames_per_side):
    """BASELINE.json configs[3]'s capture: frames_per_side LEFT + as many RIGHT frames of the room
    walk (0.064 m stereo baseline), 640x480, in reconstruct_scene.py:64-81's order (all LEFT, then
    all RIGHT).  Seeded once for the whole capture, so every rank count shards the same frames."""
    from mqr import synthetic
    left = synthetic.room_loop_poses(frames_per_side)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    return synthetic.make_sequence_fast("room", poses=left + right, height=args.height, width=args.width, seed=4,
                                        device=f"cuda:{dev}")


def sharded_parity(full_host, K, T, args, owned, meshes):
    """The C4 shards merged over RCCL against the oracle's single sequential pass over the whole
    capture (rank 0): the owned slices partition the oracle's block set, weights are identical, tsdf
    within 1e-4 (the merge sums partial running averages: fp32 rounding differs from the sequential
    update), and the shard meshes (owned cubes) have the oracle mesh's triangle count; whether the
    triangle position multisets are also identical is reported (a rounding difference can move a vertex)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from gpu_helpers import _key_order, mesh_signature
    ref = oracle_volume(full_host, K, T, args.voxel, args)
    ok_, ot, ow = ref.export()
    gk = np.concatenate([o[0] for o in owned])
    out = {"blocks": int(len(gk)), "oracle_blocks": int(len(ok_))}
    ga, oa = _key_order(gk), _key_order(ok_)
    out["keys_equal"] = gk.shape == ok_.shape and bool(np.array_equal(gk[ga], ok_[oa]))
    if out["keys_equal"]:
        gt = np.concatenate([o[1] for o in owned])
        gw = np.concatenate([o[2] for o in owned])
        weq, err = True, 0.0
        for c in range(0, len(ga), 4096):
            i, j = ga[c:c + 4096], oa[c:c + 4096]
            weq = weq and bool(np.array_equal(gw[i], ow[j]))
            m = gw[i] > 0
            if m.any():
                err = max(err, float(np.abs(gt[i][m] - ot[j][m]).max()))
        out["weights_equal"], out["max_dtsdf"] = weq, err
        del gt, gw
    ov, _, otri = ref.extract_mesh(args.extract_threshold)
    off, V, Tr = 0, [], []
    for v, t in meshes:
        V.append(v)
        Tr.append(t + off)
        off += len(v)
    V, Tr = np.concatenate(V), np.concatenate(Tr)
    out["mesh_threshold"] = args.extract_threshold
    out["triangles"] = int(len(Tr))
    out["triangle_count_equal"] = len(Tr) == len(otri)
    if out["triangle_count_equal"]:
        out["triangle_positions_equal"] = bool(np.array_equal(mesh_signature(V, Tr)[1], mesh_signature(ov, otri)[1]))
    out["tolerance"] = 1e-4
    out["comparison"] = ("owned slices of the RCCL-merged shards vs the oracle's sequential pass over all frames: "
                         "keys/weights exact, tsdf within tolerance, triangle count exact")
    out["all_ok"] = bool(out.get("keys_equal") and out.get("weights_equal") and out.get("max_dtsdf", 1) <= 1e-4
                         and out["triangle_count_equal"])
    return out


def _json_stdout():
    """The JSON line is the only thing this process writes to stdout.  Native libraries write to
    file descriptor 1 behind Python's back (gloo's "[Gloo] Rank 0 is connected to ..." lines, RCCL's
    and ROCm's messages); fd 1 is pointed at stderr and the line goes out through a private
    duplicate of the original stdout."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w", buffering=1)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # no launcher around us: start the N ranks here, before anything touches the GPU
            sys.exit(launch_ranks(args.gpus, sys.argv[1:], timeout=args.launch_timeout))
    out_json = _json_stdout()
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        if int(os.environ.get("RANK", 0)) == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": args.gpus,
                              "error": f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}"}),
                  file=out_json, flush=True)
        sys.exit(1)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import numpy as np
    import torch
    if os.environ.get("MQR_BENCH_WRAP_DEVICES"):  # rehearsal on fewer GPUs than ranks (gloo-staged merge)
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if args.c5_only:
        print(json.dumps({"c5": c5_leg(args, torch.device("cuda", local), parity=not (args.no_cpu or args.no_parity))}),
              file=out_json, flush=True)
        return
    dist = comm = None
    if world > 1:
        # control plane only (barriers, the RCCL id, max-over-ranks timing); volume data moves over
        # RCCL inside libmqr_hip.so (mqr_reduce_rccl)
        import datetime
        import torch.distributed as dist
        # a rank stuck in a collective (its peer died) fails after 10 minutes instead of gloo's 30
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=10))
    # N > 1 measures BASELINE's C4 (a fixed 2000-frame L+R capture split over the ranks) unless --weak
    strong = args.strong or (world > 1 and not args.weak)

    from mqr import synthetic
    from mqr.distributed import make_comm, merge_rccl, merge_staged, shard_range
    from mqr.vbg import VoxelBlockGrid

    full_host = K_full = T_full = None
    if strong:
        # C4: LEFT then RIGHT (reconstruct_scene.py:64-81 order), contiguous frame ranges per rank
        full = c4_capture(args, local, args.strong_frames)
        lo, hi = shard_range(2 * args.strong_frames, rank, world)
        if world == 1:
            seq = full
        else:
            seq = {k: (v[lo:hi] if k in ("depth_t", "raw_t", "K", "T_wc", "T_cw") else v) for k, v in full.items()
                   if k != "unity"}
            seq["depth_t"] = seq["depth_t"].clone()
            if rank == 0 and not (args.no_cpu or args.no_parity):
                full_host = full["depth_t"].cpu().numpy()
                K_full, T_full = full["K"].astype(np.float64), full["T_wc"].astype(np.float64)
            del full
            torch.cuda.empty_cache()
    else:
        # this rank's frames of an N*frames closed walk through the room (weak scaling)
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

    merge_times = []
    merge_phases = []
    shard = {"out": None, "owned": 0}
    transport = None
    staged = bool(os.environ.get("MQR_BENCH_WRAP_DEVICES")) and world > torch.cuda.device_count()
    if world > 1 and not staged:
        # RCCL inside libmqr.  If it cannot start on every rank (agreed over gloo) the line fails:
        # no value is printed for a run whose merge would not be the one measured.
        err = None
        try:
            comm = make_comm(local)
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            comm, err = None, f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if comm is None else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()):
            if comm is not None:
                comm.close()
            if rank == 0:
                print(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": world,
                                  "merge_transport": f"RCCL failed to start on at least one rank: {err or 'peer'}",
                                  "error": "no measurement: the RCCL merge could not run"}), file=out_json, flush=True)
            dist.destroy_process_group()
            sys.exit(1)
        transport = "rccl (mqr_reduce_rccl)"
    elif staged:
        transport = "gloo-staged (mqr_xchg_*, rehearsal with several ranks per GPU; not a scaling measurement)"
    if world > 1:
        log(f"rank {rank}: merge transport {transport}")
        shard["out"] = VoxelBlockGrid(voxel_size=args.voxel, block_resolution=args.block_resolution,
                                      block_count=args.block_count, device=local)

    def merge():
        # (integrate_frames returns with its last launch queued; the merge's all-gathers and plan overlap
        # it and only its send gather waits for it -- so this wall time includes that wait, and
        # merge_phases_ms is the merge's own device time)
        t = time.perf_counter()
        if comm is not None:
            shard["out"], shard["owned"] = merge_rccl(vbg, comm, mode=args.merge, out=shard["out"])
            merge_phases.append(comm.timing())
        else:
            shard["out"], shard["owned"] = merge_staged(vbg, mode=args.merge, out=shard["out"], stats=shard)
        torch.cuda.synchronize()
        merge_times.append(time.perf_counter() - t)
        if comm is not None:
            shard.update(comm.counts())

    # The frames are generated once and never written again: MQR_DEVICE_RESIDENT (include/mqr.h), so a pass's
    # first touch can run beside the previous pass's last integrate.  Every pass still resets the volume and
    # integrates all B frames; the timed region ends with a synchronize.
    resident = not args.no_resident

    def step():
        vbg.reset()
        vbg.integrate_frames(dptr, K, T, depth_scale=1.0, depth_max=args.depth_max,
                             trunc_voxel_multiplier=args.trunc, resident=resident)
        if world > 1:
            merge()

    log(f"rank {rank}: {B} frames {H}x{W} generated ({'C4 strong split' if strong else 'C2 per rank'}); "
        f"warm-up {args.warmup} steps")
    for _ in range(args.warmup):
        step()
    merge_times.clear()
    merge_phases.clear()
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
    log(f"rank {rank}: {args.steps} timed steps in {elapsed:.3f} s")
    vbg.profile(False)
    st = vbg.stats(reset=True)
    # the touch launches' times (HIP events on the touch stream) from a separate profiled pass of the
    # same step: recorded inside the timed steps they would add two event commands per batch
    tst = None
    if args.touch_steps > 0:
        vbg.profile(True, touch=True)
        for _ in range(args.touch_steps):
            vbg.reset()
            vbg.integrate_frames(dptr, K, T, depth_scale=1.0, depth_max=args.depth_max,
                                 trunc_voxel_multiplier=args.trunc)
        tst = vbg.stats(reset=True)
        vbg.profile(False)
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    merge_ms = (sum(merge_times) / len(merge_times) * 1e3) if merge_times else None
    merge_bytes = None
    if dist and "sent_bytes" in shard:
        # what each rank's exchange moved to / from its peers (self segment excluded), last timed step
        mb = torch.tensor([shard["sent_bytes"], shard["recv_bytes"], shard["sent_blocks"], shard["recv_blocks"]],
                          dtype=torch.float64)
        allmb = [torch.zeros_like(mb) for _ in range(world)]
        dist.all_gather(allmb, mb)
        allmb = torch.stack(allmb)
        merge_bytes = {"sent_bytes_per_rank": allmb[:, 0].tolist(), "recv_bytes_per_rank": allmb[:, 1].tolist(),
                       "max_sent_bytes": float(allmb[:, 0].max()), "max_recv_bytes": float(allmb[:, 1].max()),
                       "total_bytes": float(allmb[:, 0].sum()),
                       "bytes_per_block": shard.get("bytes_per_block", 8 * args.block_resolution ** 3),
                       "note": "whole blocks to each peer, the local self segment excluded: tsdf float32 with the "
                               "weights as uint16 (6 B per voxel) when every rank's weights fit, else float32 "
                               "(tsdf, weight) pairs (8 B per voxel)"}
    merge_phases_ms = ({k: sum(p[k] for p in merge_phases) / len(merge_phases) for k in merge_phases[0]}
                       if merge_phases else None)

    blocks = vbg.size()
    R3_ = args.block_resolution ** 3
    ext_ms, (nv, nt) = (None, (0, 0))
    sharded = sharded_par = weak_leg = c5_sharded = None
    if world > 1:
        # every rank extracts its owned cubes (mqr_extract_mesh_owned); the mesh is the concatenation
        from mqr.distributed import extract_mesh_owned
        dist.barrier()
        t = time.perf_counter()
        m = extract_mesh_owned(shard["out"], shard["owned"], args.extract_threshold)
        tx = time.perf_counter() - t
        stats = torch.tensor([tx, len(m.triangles), len(m.vertices), shard["owned"]], dtype=torch.float64)
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)
        allst = torch.stack(allst)
        sharded = {"mode": args.merge, "extract_ms_max": float(allst[:, 0].max()) * 1e3,
                   "triangles": int(allst[:, 1].sum()), "vertices_with_boundary_copies": int(allst[:, 2].sum()),
                   "union_blocks": int(allst[:, 3].sum()) if args.merge == "sharded" else int(allst[0, 3]),
                   "note": "per-rank owned-cube extraction of the merged shard (host copy of the shard mesh "
                           "included); triangles add up to the single-volume mesh"}
        blocks = sharded["union_blocks"]
        nv, nt = sharded["vertices_with_boundary_copies"], sharded["triangles"]
        if strong and args.merge == "sharded" and not (args.no_cpu or args.no_parity):
            # the last timed step's merged shards against the oracle's pass over the whole capture
            k_, t_, w_ = shard["out"].export()
            n_ = shard["owned"]
            gathered = [None] * world if rank == 0 else None
            dist.gather_object(((k_[:n_], t_[:n_], w_[:n_]), (m.vertices, m.triangles)), gathered, dst=0)
            del k_, t_, w_
            if rank == 0:
                log("C4 sharded parity: oracle pass over the whole capture")
                sharded_par = sharded_parity(full_host, K_full, T_full, args, [g[0] for g in gathered],
                                             [g[1] for g in gathered])
            del gathered
            dist.barrier()
        if strong and args.weak_steps > 0:
            # sub-leg: C2 weak scaling (500 frames per rank of an N*500-frame walk), same merge
            poses = synthetic.room_loop_poses(args.frames * world)[rank * args.frames:(rank + 1) * args.frames]
            wseq = synthetic.make_sequence_fast("room", poses=poses, height=args.height, width=args.width,
                                                seed=rank, device=f"cuda:{local}")
            wd = wseq["depth_t"].contiguous()
            wK, wT = wseq["K"].astype(np.float64), wseq["T_wc"].astype(np.float64)
            # no synchronize: libmqr orders its streams after torch's current stream (include/mqr.h)
            wptr = (_DevPtr(wd.data_ptr()), wd.shape[0], H, W)

            def wstep():
                vbg.reset()
                vbg.integrate_frames(wptr, wK, wT, depth_scale=1.0, depth_max=args.depth_max,
                                     trunc_voxel_multiplier=args.trunc)
                merge()

            for _ in range(args.warmup):
                wstep()
            merge_times.clear()
            dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.weak_steps):
                wstep()
            torch.cuda.synchronize()
            dist.barrier()
            we = torch.tensor([time.perf_counter() - t1], dtype=torch.float64)
            dist.all_reduce(we, op=dist.ReduceOp.MAX)
            we = float(we.item())
            weak_leg = {"workload": "C2 per rank (weak): 500 frames per GPU of an N*500-frame room walk + merge",
                        "frames_per_gpu": int(wd.shape[0]), "steps": args.weak_steps,
                        "value": wd.shape[0] * world * args.weak_steps / we, "unit": "frames/s",
                        "ms_per_step": we / args.weak_steps * 1e3,
                        "merge_ms": sum(merge_times) / len(merge_times) * 1e3, "union_blocks": shard["out"].size()
                        if args.merge == "root" else None}
            del wd, wseq
        if not args.no_c5:
            # C5's multi-GPU form: 4000 hall frames at 3 mm sharded, one exchange, owned-cube meshes, colour
            def c5_merge(v, st):
                if comm is not None:
                    o = merge_rccl(v, comm, mode="sharded")
                    st.update(comm.counts())
                    return o
                return merge_staged(v, mode="sharded", stats=st)

            log(f"rank {rank}: C5 sharded sub-leg")
            try:
                c5_sharded = c5_sharded_leg(args, rank, world, local, c5_merge, dist,
                                            parity=not (args.no_cpu or args.no_parity))
            except Exception as e:  # noqa: BLE001 -- reported in the line; the C4 headline stands
                log(f"rank {rank}: C5 sharded sub-leg failed: {type(e).__name__}: {e}")
                c5_sharded = {"error": f"rank {rank}: {type(e).__name__}: {e}"}
            torch.cuda.empty_cache()
    elif rank == 0:
        ext_ms, (nv, nt) = extract_ms(vbg, args.extract_threshold, args.extract_reps)

    R3 = args.block_resolution ** 3
    alg_bytes = 16 * R3 * st["union_blocks"] + 4 * H * W * st["frames"] + 16 * st["frame_blocks"]
    launches = max(st["integrate_launches"], 1)
    avg_ms = st["integrate_ms"] / launches
    achieved = alg_bytes / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    cpu = parity = None
    host_depth = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # CPU baseline and parity FIRST: the volume checked is the one the last timed step left
        host_depth = depth_t.cpu().numpy()
        log("CPU baseline (oracle)")
        cpu, ref_vol = cpu_baseline(host_depth, K, T, args)
        if not args.no_parity:
            log("parity check of the timed volume")
            parity = parity_check(vbg, ref_vol, args.extract_threshold, points_thr=3.0)
        del ref_vol
    elif world > 1:
        parity = sharded_par

    extras = {}
    conf_maps = None
    if rank == 0 and world == 1 and not args.no_extras:
        dev = torch.device("cuda", local)
        log("extra legs: copy peak, confidence, ingest, raycast, mesh filter, C3, drop-in")
        extras["hbm_copy_gbs"] = copy_peak_gbs(dev)
        extras["confidence"], conf_maps = confidence_leg(depth_t, K, T, args, dev)
        extras["ingest"] = ingest_leg(B, H, W, dev)
        extras["raycast"] = raycast_leg(vbg, K, T, H, W, args.extract_threshold)
        extras["meshfilter"] = meshfilter_leg(vbg, args.extract_threshold)
        extras["c3"] = c3_leg(seq, vbg, args, dev, parity=not (args.no_cpu or args.no_parity))
        if not strong and not args.no_c4:
            log("C4 leg (1000 + 1000 frames chained, parity)")
            extras["c4"] = c4_leg(args, dev, parity=not (args.no_cpu or args.no_parity))
        if not args.no_c5:
            log("C5 leg (4000 frames @ 3 mm, extract, colour, parity)")
            extras["c5"] = c5_leg(args, dev, parity=not (args.no_cpu or args.no_parity))
        log("C3 / C5 legs done; drop-in leg (on-disk capture)")
        if args.e2e_frames > 0:
            extras["dropin_e2e"] = dropin_e2e_leg(seq, min(args.e2e_frames, B), dev)
        # PCIe-inclusive: the same step from host (numpy) frames, H2D inside integrate_frames
        host = depth_t.cpu().numpy()
        best = None
        for _ in range(3):  # best of 3 (a single run varies with the host's copy path)
            vbg.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            vbg.integrate_frames(host, K, T, depth_scale=1.0, depth_max=args.depth_max,
                                 trunc_voxel_multiplier=args.trunc)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        extras["host_input_frames_per_s"] = B / best
    ext_alg = None
    if ext_ms:
        ext_alg = (8 * R3_ * blocks + 4 * 27 * blocks + 24 * nv + 12 * nt) / (ext_ms * 1e-3) / 1e9

    if host_depth is not None:
        if extras.get("confidence") is not None and args.conf_cpu_seconds > 0:
            log("confidence CPU baseline + parity of the GPU maps")
            extras["confidence"]["cpu_baseline"], extras["confidence"]["parity"] = confidence_cpu(
                host_depth, K, T, args, args.conf_cpu_seconds, conf_maps)
    conf_maps = None

    from mqr import _lib
    _vr = ctypes.c_int(-1)
    _lib.call("mqr_vbg_last_kernel", vbg.handle, ctypes.byref(_vr))
    variant_ran = _vr.value
    kernel_ran = last_kernel_name(vbg)
    traffic, traffic_src = pmc_traffic(H, W, B, variant_ran)

    if rank == 0:
        total_frames = (2 * args.strong_frames if strong else B * world) * args.steps
        c4_name = ("C4 (SURVEY.md §8(d); BASELINE.json configs[3]): 2000-frame LEFT+RIGHT capture (1000 + 1000) "
                   f"split over {world} GPU(s) by contiguous frame ranges, 640x480, 5 mm voxels, R=16, depth_max 4 m, "
                   "trunc 10" + (f", merged over {transport} ({args.merge})" if world > 1 else ""))
        out = {
            "metric": METRIC,
            "value": total_frames / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural room, GPU ray-cast, sigma=0.002z noise + 1% dropout)",
            "config": {"workload": c4_name if strong else
                                   ("C2 (SURVEY.md §8(d); BASELINE.json configs[1]): 500-frame LEFT depth sequence "
                                    "per GPU, 640x480, hashed TSDF 5 mm voxels, 512^3 effective volume, R=16, "
                                    "depth_max 4 m, trunc 10"),
                       "frames_per_gpu": B, "height": H, "width": W, "voxel_size": args.voxel,
                       "block_resolution": args.block_resolution, "depth_max": args.depth_max,
                       "trunc_voxel_multiplier": args.trunc, "frame_batch": 127,
                       "frames": "MQR_DEVICE" if args.no_resident else "MQR_DEVICE_RESIDENT (generated once, unchanged)",
                       "parallelism": f"frame-shard x{world}" + (f" + libmqr merge ({args.merge}, {transport})"
                                                                 if world > 1 else "")},
            "sharded_extract": sharded,
            "merge_ms": merge_ms,
            "merge_ms_note": ("wall time of the merge call per step; it overlaps the rank's last integrate launch "
                              "(all-gathers and plan) and waits for it before the send gather, so it includes that "
                              "wait; merge_phases_ms are the merge's own device phases") if world > 1 else None,
            "merge_phases_ms": merge_phases_ms,
            "merge_transport": transport,
            "merge_bytes_per_rank": merge_bytes,
            "weak_c2": weak_leg,
            "union_blocks": blocks if world > 1 else None,
            "extract_ms": ext_ms,
            "extract": {"weight_threshold": args.extract_threshold, "vertices": nv, "triangles": nt,
                        "blocks": blocks, "alg_gbs": ext_alg,
                        "note": "device-resident extract_triangle_mesh, median of reps; alg bytes = "
                                "8R^3 N + 108 N + 24 V + 12 T"},
            "confidence": extras.get("confidence"),
            "ingest": extras.get("ingest"),
            "raycast": extras.get("raycast"),
            "meshfilter": extras.get("meshfilter"),
            "host_input_frames_per_s": extras.get("host_input_frames_per_s"),
            "build": {"integrate_src": build_tag(0), "confidence_src": build_tag(1), "integrate_variant": variant_ran},
            "roofline_binding": dict(pmc_binding(avg_ms, variant_ran) or {}, gather_ceiling=gather_ceiling(
                avg_ms, st["frame_blocks"] * args.block_resolution ** 3 / 64 / launches,
                torch.cuda.get_device_properties(local).multi_processor_count)),
            "roofline": {"bound": "hbm", "kernel": kernel_ran, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "peak_measured_copy": extras.get("hbm_copy_gbs"),
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "alg_bytes_per_launch": alg_bytes / launches, "avg_launch_ms": avg_ms,
                         "launches": st["integrate_launches"], "union_blocks_per_launch":
                             st["union_blocks"] / launches, "frame_blocks_per_frame":
                             st["frame_blocks"] / max(st["frames"], 1),
                         "touch_ms_per_launch": (tst["touch_ms"] / tst["touch_launches"]) if tst and
                         tst["touch_launches"] else None,
                         "touch_launches_per_step": (tst["touch_launches"] / args.touch_steps) if tst else None,
                         "touch_note": f"k_touch launch time (HIP events on the touch stream) over {args.touch_steps} "
                                       "profiled steps after the timed ones; the first touch of a step runs alone, the "
                                       "others beside the previous batch's integrate"},
            "cpu_baseline": cpu,
            "parity": parity,
            "c3": extras.get("c3"),
            "c4": extras.get("c4"),
            "c5": extras.get("c5"),
            "c5_sharded": c5_sharded,
            "dropin_e2e": extras.get("dropin_e2e"),
        }
        print(json.dumps(out), file=out_json, flush=True)
    if comm is not None:
        comm.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
