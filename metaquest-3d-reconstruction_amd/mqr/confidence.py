"""Drop-in for the reference's multi-view depth-confidence estimator on the MI355X.

    estimate_depth_confidences(depth_data_io, config)   estimate_depth_confidences.py:120-153
    build_confidence_map(...)                           estimate_depth_confidences.py:15-79
    compute_pixel_error_map(...)                        compute_pixel_error_map.py:120-220

The reference runs one numpy task per reference frame on a process pool and re-reads every
neighbour frame from disk (~21x per frame).  Here each side's frames are decoded once, kept in
HBM, and one kernel launch computes a chunk of reference frames (thread per pixel, neighbour
loop in registers, float64 like numpy).  Outputs, file names and resume rules are the
reference's: ``<side>_depth_confidence/<timestamp>.npz`` with confidence_map f64 / valid_count i32,
existing per-frame files are kept, a side whose directory exists is skipped when
``skip_if_output_dir_exists``.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._io import io_pool
from ._lib import MQR_HOST, call, ptr
from .models import ConfidenceMap, CoordinateSystem, Side
from .o3d_utils import compute_o3d_intrinsic_matrices

REF_CHUNK = 64

# wall-clock split (seconds) of the last estimate_depth_confidences call on this thread: the resume scan,
# frame decoding (prefetch), the confidence calls (upload + kernel + download), waiting for npz writes
last_confidence_times = threading.local()


@dataclass
class DepthConfidenceEstimationConfig:
    """reconstruction_config.py:33-39 (defaults), config/pipeline_config.yml:30-35 (pipeline values)."""
    target_frame_range: int = 10
    depth_max: float = 3.0
    error_threshold: float = 0.05
    skip_if_output_dir_exists: bool = True
    use_dataset_cache: bool = True
    use_multi_threading: bool = True
    device: int = 0


def confidence_maps(depths, intrinsics, T_cw, T_cw_inv, ref_begin=0, ref_end=None, target_frame_range=10,
                    depth_max=3.0, error_threshold=0.05, frame_ok=None, device=0):
    """(conf (n,H,W) f64, valid (n,H,W) i32) for reference frames [ref_begin, ref_end)."""
    d = np.ascontiguousarray(depths, dtype=np.float32)
    N, H, W = d.shape
    ref_end = N if ref_end is None else ref_end
    K = np.ascontiguousarray(intrinsics, dtype=np.float32).reshape(N, 9)
    Tc = np.ascontiguousarray(T_cw, dtype=np.float32).reshape(N, 16)
    Ti = np.ascontiguousarray(T_cw_inv, dtype=np.float32).reshape(N, 16)
    ok = None if frame_ok is None else np.ascontiguousarray(frame_ok, dtype=np.uint8)
    nref = ref_end - ref_begin
    conf = np.empty((nref, H, W), np.float64)
    valid = np.empty((nref, H, W), np.int32)
    call("mqr_confidence", int(device), ptr(d), MQR_HOST, N, H, W, ptr(K, _lib._f32p), ptr(Tc, _lib._f32p),
         ptr(Ti, _lib._f32p), None if ok is None else ptr(ok, _lib._u8p), int(ref_begin), int(ref_end),
         int(target_frame_range), float(depth_max), float(error_threshold), ptr(conf), ptr(valid), MQR_HOST)
    return conf, valid


def compute_pixel_error_map(intrinsic_matrices, extrinsic_matrices, extrinsic_matrices_inv, ref_frame_idx,
                            ref_depth_map, target_frame_idx, target_depth_map, depth_max=3.0, device=0):
    ref = np.ascontiguousarray(ref_depth_map, dtype=np.float32)
    tgt = np.ascontiguousarray(target_depth_map, dtype=np.float32)
    H, W = ref.shape
    K = np.ascontiguousarray(intrinsic_matrices, dtype=np.float32)
    Tc = np.ascontiguousarray(extrinsic_matrices, dtype=np.float32)
    Ti = np.ascontiguousarray(extrinsic_matrices_inv, dtype=np.float32)
    out = np.empty((H, W), np.float32)
    f = _lib._f32p
    call("mqr_pixel_error_map", int(device), ptr(ref, f), ptr(tgt, f), H, W, ptr(K[ref_frame_idx], f),
         ptr(K[target_frame_idx], f), ptr(Tc[ref_frame_idx], f), ptr(Ti[target_frame_idx], f),
         ptr(Tc[target_frame_idx], f), float(depth_max), ptr(out, f))
    return out


def _canvas_stack(frames):
    """Stack a window of frames of possibly different sizes (None = failed load) on a zero canvas of
    the largest height and width.  Exact for the reference's arithmetic: bilinear_interpolate_depth
    bounds-checks against the target's own (h, w) (compute_pixel_error_map.py:4-60), and a tap in
    the zero padding fails the same tap test (`0 < depth`) that the reference's `u1 < w` / `v1 < h`
    check rejects; coordinates beyond 10 max(w, h) fail the bounds check either way."""
    shapes = [f.shape for f in frames if f is not None]
    H = max(h for h, _ in shapes)
    W = max(w for _, w in shapes)
    out = np.zeros((len(frames), H, W), np.float32)
    for i, f in enumerate(frames):
        if f is not None:
            out[i, :f.shape[0], :f.shape[1]] = f
    return out


def build_confidence_map(depth_data_io, dataset, intrinsic_matrices, extrinsic_matrices, extrinsic_matrices_inv,
                         side, ref_frame_idx, target_frame_range=10, depth_max=3.0,
                         error_threshold=0.05) -> Optional[ConfidenceMap]:
    ref = depth_data_io.load_depth_map_by_index(side=side, dataset=dataset, index=ref_frame_idx)
    if ref is None:
        return None
    lo = max(0, ref_frame_idx - target_frame_range)
    hi = min(len(dataset), ref_frame_idx + target_frame_range + 1)
    frames = [ref if i == ref_frame_idx else depth_data_io.load_depth_map_by_index(side=side, dataset=dataset,
                                                                                     index=i)
              for i in range(lo, hi)]
    ok = np.array([f is not None for f in frames])
    conf, valid = confidence_maps(_canvas_stack(frames), np.asarray(intrinsic_matrices)[lo:hi],
                                  np.asarray(extrinsic_matrices)[lo:hi], np.asarray(extrinsic_matrices_inv)[lo:hi],
                                  ref_frame_idx - lo, ref_frame_idx - lo + 1, target_frame_range, depth_max,
                                  error_threshold, ok)
    h, w = ref.shape
    return ConfidenceMap(confidence_map=np.ascontiguousarray(conf[0, :h, :w]),
                         valid_count=np.ascontiguousarray(valid[0, :h, :w]))


def _report(side, idx, timestamp, e):
    """estimate_depth_confidences.py:114-117: a failing reference frame is reported and skipped."""
    import traceback
    print(f"[Error] build_and_save_confidence_map failed for {side.name} frame {idx} (timestamp {timestamp}): {e}")
    traceback.print_exception(type(e), e, e.__traceback__)


# the native path downloads the maps as (valid, consistent) byte pairs (mqr_confidence_counts) when a window's
# neighbour count fits a byte; False: the maps themselves (A/B, tools/conf_ab.py)
COUNT_PAIRS = True

# decoded frames of a side kept in HBM by the native path (bytes); larger captures take the windowed path
RESIDENT_MAX_BYTES = 48 << 30
_READ_CHUNK = 127

# per thread: the native path's three host sets of count pairs (or of maps), kept across calls -- freeing
# the maps (~0.7 GB at 640 x 480) cost ~50 ms per call and re-faulting them slowed every download
# (tools/conf_driver_prof.py)
_TLS = threading.local()


def _map_sets(H, W, counts: bool):
    cache = getattr(_TLS, "map_sets", None)
    if cache is None:
        cache = _TLS.map_sets = {}
    sets = cache.get(counts)
    if sets is None or sets[0][0].shape[1:] != (H, W):
        if counts:
            sets = [(np.empty((REF_CHUNK, H, W), np.uint16),) for _ in range(3)]
        else:
            sets = [(np.empty((REF_CHUNK, H, W), np.float64), np.empty((REF_CHUNK, H, W), np.int32))
                    for _ in range(3)]
        cache[counts] = sets
    return sets


def _raw_stages(B, H, W):
    """The native path's two alternating raw read buffers, kept across calls like the map sets (freeing the
    ~0.3 GB of touched pages at the end of every call cost ~17 ms, tools/conf_driver_prof.py)."""
    st = getattr(_TLS, "raw_stages", None)
    if st is None or st[0].shape != (B, H, W):
        st = _TLS.raw_stages = [np.empty((B, H, W), np.float32) for _ in range(2)]
    return st


def release_host_maps():
    """Free this thread's cached host buffers of estimate_depth_confidences: the map sets (3 x REF_CHUNK frames of
    2 B per pixel, or 12 B when a window holds more than 255 neighbours) and the two raw read buffers
    (2 x 127 frames of 4 B per pixel)."""
    _TLS.map_sets = None
    _TLS.raw_stages = None


def _native_paths(depth_data_io, side, dataset):
    """(raw path fn, confidence path fn) when the side can run device-resident: frames read, decoded and
    saved by the standard code (this package's DepthDataIO with those methods not overridden, or the
    reference's DepthDataIO through its path config), one frame size, and the decoded frames within
    RESIDENT_MAX_BYTES; else None."""
    from .dataio import DepthDataIO
    from .o3d_utils import _frame_paths, _reference_methods_intact
    paths = _frame_paths(depth_data_io, side)
    if paths is None:
        return None
    methods = ("load_depth_map", "load_depth_map_by_index", "save_confidence_map", "is_depth_map_valid")
    if set(methods) & set(getattr(depth_data_io, "__dict__", {})):  # replaced on the instance
        return None
    if isinstance(depth_data_io, DepthDataIO):
        cls = type(depth_data_io)
        if any(getattr(cls, m) is not getattr(DepthDataIO, m) for m in methods):
            return None
    elif not _reference_methods_intact(depth_data_io, methods):  # a subclass of the reference's overrides one
        return None
    if len(dataset) == 0 or len(set(zip(np.asarray(dataset.widths).tolist(), np.asarray(dataset.heights).tolist()))) != 1:
        return None
    if 4 * len(dataset) * int(dataset.widths[0]) * int(dataset.heights[0]) > RESIDENT_MAX_BYTES:
        return None
    return paths


def _estimate_side_native(depth_data_io, config, side, dataset, todo, K, T_cw, T_inv, paths, times) -> bool:
    """One side, device-resident: the raw files read by native threads (mqr_read_frames), decoded on the
    GPU once into an HBM array of all frames (mqr_decode_depth: the reference's is_depth_map_valid and
    convert_depth_to_linear, bit for bit), the confidence kernel run on device windows of it as soon as a
    window is decoded, each run's maps downloaded and written by native threads (mqr_write_confidence_npz:
    np.savez's files) while the next frames are read and the next run computes.  Returns False when a raw
    file needs the Python reader: a file of the wrong size before anything is written; a read error later
    leaves the runs already written (windows read in full, so their files are what the standard path writes)
    -- the caller then takes the standard path for the side."""
    from concurrent.futures import ThreadPoolExecutor

    from ._io import io_threads
    from ._lib import DeviceBuffer, MQR_DEVICE
    from .ingest import decode_depth_frames
    raw_path, conf_path = paths
    n = len(dataset)
    H, W = int(dataset.heights[0]), int(dataset.widths[0])
    HW = H * W
    dev = int(getattr(config, "device", 0))
    r = int(config.target_frame_range)
    ts = dataset.timestamps
    t0 = time.perf_counter()
    raw_names = [os.fsencode(str(raw_path(t))) for t in ts]
    for name in raw_names:  # a raw file of the wrong size: the standard path reads (or rejects) it
        try:
            if os.stat(name).st_size != 4 * HW:
                return False
        except FileNotFoundError:
            pass  # missing: decoded invalid, as the reference skips it
    times["scan"] += time.perf_counter() - t0
    t0 = time.perf_counter()
    depth = DeviceBuffer(4 * n * HW, dev)
    times["alloc"] = times.get("alloc", 0.0) + time.perf_counter() - t0
    ok = np.zeros(n, bool)
    stages = _raw_stages(min(_READ_CHUNK, n), H, W)
    Kf = np.ascontiguousarray(K, dtype=np.float32).reshape(n, 9)
    Tc = np.ascontiguousarray(T_cw, dtype=np.float32).reshape(n, 16)
    Ti = np.ascontiguousarray(T_inv, dtype=np.float32).reshape(n, 16)
    ok8 = np.zeros(n, np.uint8)
    if todo:
        conf_path(ts[todo[0]]).parent.mkdir(parents=True, exist_ok=True)

    def read(c0, st):
        c1 = min(n, c0 + _READ_CHUNK)
        status = np.zeros(c1 - c0, np.uint8)
        names = (ctypes.c_char_p * (c1 - c0))(*raw_names[c0:c1])
        call("mqr_read_frames", c1 - c0, names, None, H, W, ptr(st), None, None, ptr(status), io_threads())
        return c0, c1, st, status

    def write(a, names, maps):
        status = np.zeros(len(names), np.int32)
        arr = (ctypes.c_char_p * len(names))(*names)
        if len(maps) == 1:  # count pairs, expanded to the maps by the writer threads
            call("mqr_write_confidence_npz_counts", len(names), arr, ptr(maps[0]), H, W, ptr(status), io_threads())
        else:
            call("mqr_write_confidence_npz", len(names), arr, ptr(maps[0]), ptr(maps[1]), H, W, ptr(status),
                 io_threads())
        return a, status

    pending = []
    # three host sets: the run computing and the at most two runs being written (settle(2)); reused, so
    # their pages are faulted in once.  Count pairs (mqr_confidence_counts: 2 B per pixel downloaded instead
    # of the maps' 12) whenever a window's neighbour count fits a byte.
    use_counts = COUNT_PAIRS and 2 * r <= 255
    outs = _map_sets(H, W, use_counts)
    runs = 0
    next_c0 = 0  # the first chunk of `todo` not computed yet

    def settle(keep):
        t_s = time.perf_counter()
        while len(pending) > keep:
            fw = pending.pop(0)
            try:
                a, status = fw.result()
            except Exception as e:  # noqa: BLE001 -- the whole run's writes failed
                a, status = None, e
            if isinstance(status, Exception):
                continue
            for j in np.nonzero(status)[0]:
                i = a + int(j)
                e = OSError(int(status[j]), os.strerror(int(status[j])), str(conf_path(ts[i])))
                _report(side, i, ts[i], e)
        times["write_wait"] += time.perf_counter() - t_s

    def compute_ready(limit):
        """The chunks of `todo` whose windows lie in the frames decoded so far ([0, limit))."""
        nonlocal next_c0, runs
        while next_c0 < len(todo) and (limit == n or todo[min(len(todo), next_c0 + REF_CHUNK) - 1] + r + 1 <= limit):
            c0 = next_c0
            next_c0 += REF_CHUNK
            chunk = [i for i in todo[c0:c0 + REF_CHUNK] if ok[i]]  # invalid refs: no output
            j = 0
            while j < len(chunk):  # runs spanning < REF_CHUNK indices, as the standard path groups them
                k = j + 1
                while k < len(chunk) and chunk[k] - chunk[j] < REF_CHUNK:
                    k += 1
                refs = chunk[j:k]
                j = k
                a, b = refs[0], refs[-1] + 1
                lo, hi = max(0, a - r), min(n, b + r)
                maps = tuple(x[:b - a] for x in outs[runs % 3])
                runs += 1
                t_c = time.perf_counter()
                args = (dev, ctypes.c_void_p(depth.ptr.value + 4 * lo * HW), MQR_DEVICE, hi - lo, H, W,
                        ptr(Kf[lo:hi], _lib._f32p), ptr(Tc[lo:hi], _lib._f32p), ptr(Ti[lo:hi], _lib._f32p),
                        ptr(ok8[lo:hi], _lib._u8p), a - lo, b - lo, r, float(config.depth_max),
                        float(config.error_threshold))
                try:
                    packed = ctypes.c_int(0)
                    if use_counts:
                        call("mqr_confidence_counts", *args, ptr(maps[0]), ctypes.byref(packed))
                    if not packed.value:  # the maps themselves
                        if use_counts:  # (a pixel with more than 255 valid neighbours: not reached for 2r <= 255)
                            maps = (np.empty((b - a, H, W), np.float64), np.empty((b - a, H, W), np.int32))
                        call("mqr_confidence", *args, ptr(maps[0]), ptr(maps[1]), MQR_HOST)
                except Exception as e:  # noqa: BLE001 -- every reference frame of the run failed
                    for i in refs:
                        _report(side, i, ts[i], e)
                    continue
                finally:
                    times["compute"] += time.perf_counter() - t_c
                want = set(refs)
                names = [os.fsencode(str(conf_path(ts[i]))) if i in want else None for i in range(a, b)]
                pending.append(writer.submit(write, a, names, maps))
                settle(2)  # at most two runs' maps held for writing

    with ThreadPoolExecutor(max_workers=1) as reader, ThreadPoolExecutor(max_workers=1) as writer:
        fut = reader.submit(read, 0, stages[0])
        turn = 0
        while fut is not None:
            t0 = time.perf_counter()
            c0, c1, st, status = fut.result()
            if (status & _lib.MQR_FRAME_RAW_OTHER).any():
                settle(0)
                depth.free()
                return False
            turn ^= 1
            fut = reader.submit(read, c1, stages[turn]) if c1 < n else None
            _, ok[c0:c1] = decode_depth_frames(st[:c1 - c0], [dataset.nears[i] for i in range(c0, c1)],
                                               [dataset.fars[i] for i in range(c0, c1)], device=dev,
                                               out_ptr=depth.ptr.value + 4 * c0 * HW)
            ok8[c0:c1] = ok[c0:c1]
            times["decode"] += time.perf_counter() - t0
            compute_ready(c1)
        settle(0)
    t0 = time.perf_counter()
    depth.free()
    times["free"] = times.get("free", 0.0) + time.perf_counter() - t0
    return True


def _todo(depth_data_io, side, dataset):
    """The frames without a loadable confidence map (load_confidence_map(...) is None, as the reference
    selects them).  With this package's DepthDataIO and its standard loader and paths, one listing of the
    confidence directory stands in for the per-frame existence checks: only frames whose file is present go
    through load_confidence_map (~10 us of path building and stat per frame otherwise)."""
    from .dataio import DepthDataIO, DepthPaths
    from .o3d_utils import _frame_paths
    ts = dataset.timestamps
    load = depth_data_io.load_confidence_map
    if (isinstance(depth_data_io, DepthDataIO) and type(depth_data_io.paths) is DepthPaths
            and _frame_paths(depth_data_io, side) is not None):
        try:
            present = set(os.listdir(depth_data_io.paths.confidence_dir(side)))
        except FileNotFoundError:
            present = set()
        except OSError:
            present = None
        if present is not None:
            return [i for i, t in enumerate(ts)
                    if f"{int(t)}.npz" not in present or load(side=side, timestamp=t) is None]
    return [i for i, t in enumerate(ts) if load(side=side, timestamp=t) is None]


def estimate_depth_confidences(depth_data_io, config: DepthConfidenceEstimationConfig, sides=None):
    """Per side: skip if the output directory exists (``skip_if_output_dir_exists``), keep existing
    per-frame files, compute the rest in chunks of REF_CHUNK reference frames.  Frames are decoded
    once each and held only while a chunk's window [first - r, last + r] needs them.  As in the
    reference (estimate_depth_confidences.py:98-117), an error while building or saving one
    reference frame's map is printed and that frame is skipped; the other frames go on."""
    times = {"scan": 0.0, "decode": 0.0, "compute": 0.0, "write_wait": 0.0, "total": 0.0}
    t_all = time.perf_counter()
    for side in (sides or list(Side)):
        if config.skip_if_output_dir_exists and depth_data_io.exists_depth_confidence_map_dir(side=side):
            print(f"[{side.name}] Skipping confidence map estimation: output directory already exists. "
                  "Set skip_if_output_dir_exists = False to force re-estimation.")
            continue
        t0 = time.perf_counter()
        dataset = depth_data_io.load_depth_dataset(side=side)
        n = len(dataset)
        if n == 0:
            continue
        K = compute_o3d_intrinsic_matrices(dataset)
        T_cw = dataset.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                            is_camera=True).extrinsics_cw
        T_inv = np.linalg.inv(T_cw)
        r = int(config.target_frame_range)
        times["prep"] = times.get("prep", 0.0) + time.perf_counter() - t0
        t0 = time.perf_counter()
        todo = _todo(depth_data_io, side, dataset)
        times["scan"] += time.perf_counter() - t0
        native = _native_paths(depth_data_io, side, dataset) if todo else None
        if native is not None and _estimate_side_native(depth_data_io, config, side, dataset, todo, K, T_cw, T_inv,
                                                        native, times):
            continue
        cache = {}  # index -> decoded frame (None: missing / invalid), frames of the current window only
        pool = io_pool()
        writes = []  # (frame index, npz write in flight on the I/O threads)

        def frame(i):
            if i not in cache:
                cache[i] = depth_data_io.load_depth_map_by_index(side=side, dataset=dataset, index=i)
            return cache[i]

        def prefetch(lo, hi):  # decode the frames of [lo, hi) not cached yet on the I/O threads
            need = [i for i in range(max(0, lo), min(n, hi)) if i not in cache]
            for i, d in zip(need, pool.map(lambda k: depth_data_io.load_depth_map_by_index(
                    side=side, dataset=dataset, index=k), need)):
                cache[i] = d

        def settle(keep):  # wait for all but the last `keep` writes, reporting failures per frame
            nonlocal writes
            t_s = time.perf_counter()
            cut = max(0, len(writes) - keep)
            for i, w in writes[:cut]:
                try:
                    w.result()
                except Exception as e:  # noqa: BLE001 -- the reference catches everything per frame
                    _report(side, i, dataset.timestamps[i], e)
            writes = writes[cut:]
            times["write_wait"] += time.perf_counter() - t_s

        for c0 in range(0, len(todo), REF_CHUNK):
            part = todo[c0:c0 + REF_CHUNK]
            t_p = time.perf_counter()
            prefetch(part[0] - r, part[-1] + r + 1)
            times["decode"] += time.perf_counter() - t_p
            chunk = [i for i in part if frame(i) is not None]  # invalid refs: no output
            for i in [k for k in cache if chunk and k < chunk[0] - r]:
                del cache[i]
            j = 0
            while j < len(chunk):  # runs spanning < REF_CHUNK indices (sparse resumes keep windows small)
                k = j + 1
                while k < len(chunk) and chunk[k] - chunk[j] < REF_CHUNK:
                    k += 1
                refs = chunk[j:k]
                j = k
                a, b = refs[0], refs[-1] + 1
                lo, hi = max(0, a - r), min(n, b + r)
                win = [frame(i) for i in range(lo, hi)]
                ok = np.array([f is not None for f in win])
                t_c = time.perf_counter()
                try:
                    conf, valid = confidence_maps(_canvas_stack(win), K[lo:hi], T_cw[lo:hi], T_inv[lo:hi], a - lo,
                                                  b - lo, r, config.depth_max, config.error_threshold, ok,
                                                  device=getattr(config, "device", 0))
                except Exception as e:  # noqa: BLE001 -- every reference frame of the run failed
                    for i in refs:
                        _report(side, i, dataset.timestamps[i], e)
                    continue
                finally:
                    times["compute"] += time.perf_counter() - t_c
                for i in refs:
                    h, w = frame(i).shape
                    cm = ConfidenceMap(np.ascontiguousarray(conf[i - a, :h, :w]),
                                       np.ascontiguousarray(valid[i - a, :h, :w]))
                    writes.append((i, pool.submit(depth_data_io.save_confidence_map, side=side,
                                                  timestamp=dataset.timestamps[i], confidence_map=cm)))
                if len(writes) > 2 * REF_CHUNK:  # bound the maps held for writing
                    settle(REF_CHUNK)
        settle(0)
    times["total"] = time.perf_counter() - t_all
    last_confidence_times.__dict__.update(times)
