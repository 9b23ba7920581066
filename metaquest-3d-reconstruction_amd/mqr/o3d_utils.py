"""Drop-in for the reference's ``processing/reconstruction/utils/o3d_utils.py`` fusion entry points.

    compute_o3d_intrinsic_matrices(dataset)          o3d_utils.py:14-19
    load_depth_map(...)                              o3d_utils.py:109-150
    integrate(dataset, depth_data_io, side, ...)     o3d_utils.py:153-238

``integrate`` keeps the reference signature, frame order, skip rules (missing / invalid frames
dropped, confidence masking with the same thresholds) and error behaviour (a frame touching no
block raises RuntimeError), but hands the frames to the MI355X in batches: host decode of the
next chunk overlaps the device work of the current one, and the device integrates each batch
with one touch launch + one integrate launch (bit-identical to per-frame calls).
The swap in the reference is one import line:
    from processing.reconstruction.utils.o3d_utils import integrate   ->   from mqr.o3d_utils import integrate
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Optional

import numpy as np

from ._io import io_pool, io_threads
from .ingest import count_threshold
from .geometry import Image
from .meshfilter import filter_mesh_components  # noqa: F401  (re-exported: o3d_utils.py:241-321)
from .raycasting import raycast_in_color_view  # noqa: F401  (re-exported: o3d_utils.py:324-341)
from .vbg import VoxelBlockGrid

# frames per host->device hand-off: a full device batch (kMaxBatch).  With the chunk read straight into
# reused host staging sets, 127-frame hand-offs take 0.362 s against 0.420 s for 64-frame ones on the
# bench's 500-frame on-disk capture, identical volumes (tools/dropin_ab.py,
# profiles/r05_ab_dropin_chunk_staged.json); before that staging, 127 was the slower size (0.629 vs
# 0.535 s, profiles/r05_ab_dropin_chunk.json)
CHUNK = 127
# frames of the first hand-off: nothing overlaps the first chunk's reads, so a short first chunk starts the
# device sooner (A/B: profiles/r05_ab_dropin_first_chunk.json)
FIRST_CHUNK = 32


class _HostStage:
    """Reusable host staging of one chunk of raw frames and their confidence masks, one byte per pixel:
    (confidence_map < threshold) | (valid_count < threshold), reduced as the maps are read (pageable, so no
    pinning cost; reused, so its pages are faulted in once instead of per chunk).  5 B per pixel go to
    the device instead of the 16 B of raw + confidence_map + valid_count."""

    def __init__(self, B, H, W, with_conf):
        self.key = (B, H, W, with_conf)
        self.raw = np.empty((B, H, W), np.float32)
        self.mask = np.empty((B, H, W), np.uint8) if with_conf else None


# per thread: the two alternating sets of the last shape used, kept across integrate() calls (the fragment
# path calls integrate() once per 100 frames)
_TLS = threading.local()


def _host_stage(turn, B, H, W, with_conf) -> _HostStage:
    stages = getattr(_TLS, "stages", None)
    if stages is None:
        stages = _TLS.stages = [None, None]
    st = stages[turn]
    if st is None or st.key != (B, H, W, with_conf):
        st = stages[turn] = _HostStage(B, H, W, with_conf)
    return st


def release_host_staging():
    """Free this thread's drop-in integrate() host staging (5 B per pixel per staged frame, two chunks)."""
    _TLS.stages = None


def compute_o3d_intrinsic_matrices(dataset) -> np.ndarray:
    """(N,3,3) float32 with the Quest->Open3D principal-point flip cx := W - cx."""
    widths = dataset.widths
    k = dataset.get_intrinsic_matrices()
    k[:, 0, 2] = widths - k[:, 0, 2]
    return k


def _masked_depth(depth_data_io, side, index, dataset, use_confidence_filtered_depth, confidence_threshold,
                  valid_count_threshold, warn=print) -> Optional[np.ndarray]:
    depth = depth_data_io.load_depth_map(side=side, timestamp=dataset.timestamps[index],
                                         width=dataset.widths[index], height=dataset.heights[index],
                                         near=dataset.nears[index], far=dataset.fars[index])
    if depth is None:
        return None
    if use_confidence_filtered_depth:
        cm = depth_data_io.load_confidence_map(side=side, timestamp=dataset.timestamps[index])
        if cm is None:
            warn(f"[Warning] Confidence map not found for timestamp {dataset.timestamps[index]}")
        else:
            depth[cm.confidence_map < confidence_threshold] = 0.0
            depth[cm.valid_count < valid_count_threshold] = 0.0
    return depth


def _raw_reader(depth_data_io, side):
    """fn(timestamp, width, height) -> raw float32 NDC buffer or None (missing file), from either
    this package's DepthDataIO or the reference's (via its depth_path_config); None if neither."""
    if hasattr(depth_data_io, "load_raw_depth"):
        return lambda ts, w, h: depth_data_io.load_raw_depth(side, ts, w, h)
    cfg = getattr(depth_data_io, "depth_path_config", None)
    if cfg is not None and hasattr(cfg, "get_depth_map_path"):
        def read(ts, w, h):
            path = cfg.get_depth_map_path(side=side, timestamp=ts)
            if not path.exists():
                return None
            return np.fromfile(path, dtype="<f4").reshape((int(h), int(w)))
        return read
    return None


def _reference_methods_intact(depth_data_io, methods) -> bool:
    """False when one of `methods` is replaced on the instance, or overridden by a subclass of the
    reference's DepthDataIO (scripts/dataio/depth_data_io.py; a class of that name in the MRO): then the
    native readers / writers must not stand in for it.  A duck type of the reference's shape (no such
    base) keeps its methods as the standard ones."""
    if set(methods) & set(getattr(depth_data_io, "__dict__", {})):
        return False
    mro = type(depth_data_io).__mro__
    base = next((c for c in mro if c.__name__ == "DepthDataIO"), None)
    if base is None:
        return True
    return not any(m in c.__dict__ for c in mro[:mro.index(base)] for m in methods)


def _frame_paths(depth_data_io, side):
    """(raw path fn, confidence npz path fn) of timestamp when the frames are read by the standard loaders
    -- this package's DepthDataIO (methods not overridden) or the reference's (its depth_path_config:
    get_depth_map_path / get_depth_confidence_map_path, depth_data_io.py:33-53, 91-104) -- so that the
    native reader (mqr_read_frames) reads exactly those files; None otherwise or with MQR_NATIVE_IO=0."""
    if os.environ.get("MQR_NATIVE_IO") == "0":
        return None
    from .dataio import DepthDataIO
    if isinstance(depth_data_io, DepthDataIO):
        cls = type(depth_data_io)
        if (cls.load_raw_depth is DepthDataIO.load_raw_depth and cls.load_confidence_map is DepthDataIO.load_confidence_map
                and not {"load_raw_depth", "load_confidence_map"} & set(vars(depth_data_io))):
            p = depth_data_io.paths
            return (lambda ts: p.depth_map_path(side, ts)), (lambda ts: p.confidence_path(side, ts))
        return None
    cfg = getattr(depth_data_io, "depth_path_config", None)
    if (not hasattr(depth_data_io, "load_raw_depth") and cfg is not None and hasattr(cfg, "get_depth_map_path")
            and hasattr(cfg, "get_depth_confidence_map_path")
            and _reference_methods_intact(depth_data_io, ("load_depth_map", "load_confidence_map"))):
        return ((lambda ts: cfg.get_depth_map_path(side=side, timestamp=ts)),
                (lambda ts: cfg.get_depth_confidence_map_path(side=side, timestamp=ts)))
    return None


class _Raised:
    """A frame whose read raised (in an I/O thread).  The reference's per-frame loop has integrated
    every frame before it and printed their messages when the exception leaves integrate()
    (o3d_utils.py:188-236): the chunk's frames before it are integrated, its messages printed, then
    the exception is re-raised on the calling thread; nothing of that frame or after it is read or
    printed (no further chunk is started)."""

    def __init__(self, index, exc):
        self.index, self.exc = index, exc


def load_depth_map(depth_data_io, side, index: int, dataset, device, use_confidence_filtered_depth: bool,
                   confidence_threshold: float, valid_count_threshold: int) -> Optional[Image]:
    d = _masked_depth(depth_data_io, side, index, dataset, use_confidence_filtered_depth, confidence_threshold,
                      valid_count_threshold)
    return None if d is None else Image(d, device=device)


# wall-clock split of the last integrate() call on this thread (seconds): volume creation, the main thread
# waiting for the I/O threads' chunks, and the device hand-off (decode + mask + batched integrate calls)
last_integrate_times = threading.local()


def integrate(dataset, depth_data_io, side, use_confidence_filtered_depth: bool, confidence_threshold: float,
              valid_count_threshold: int, voxel_size: float, block_resolution: int, block_count: int,
              depth_max: float, trunc_voxel_multiplier: float, device, show_progress: bool = False,
              desc: Optional[str] = None, vbg_opt: Optional[VoxelBlockGrid] = None) -> VoxelBlockGrid:
    from .dataio import DepthDataIO
    times = {"create": 0.0, "wait_io": 0.0, "device": 0.0, "chunks": 0}
    t_c = time.perf_counter()
    vbg = vbg_opt if vbg_opt is not None else VoxelBlockGrid(
        attr_names=("tsdf", "weight"), attr_dtypes=("float32", "float32"), attr_channels=((1), (1)),
        voxel_size=voxel_size, block_resolution=block_resolution, block_count=block_count, device=device)
    times["create"] = time.perf_counter() - t_c
    n = len(dataset.timestamps)
    extrinsic_wc = dataset.transforms.extrinsics_wc
    intrinsics = compute_o3d_intrinsic_matrices(dataset)
    read_raw = _raw_reader(depth_data_io, side)
    native = _frame_paths(depth_data_io, side) if read_raw is not None else None

    def chunk_end(lo):  # chunks: [0, FIRST_CHUNK), then CHUNK frames each
        return min(n, lo + (min(FIRST_CHUNK, CHUNK) if lo == 0 else CHUNK))

    def load_one(i):
        """(item or None, this frame's messages), or _Raised."""
        msgs = []
        try:
            if read_raw is None:
                d = _masked_depth(depth_data_io, side, i, dataset, use_confidence_filtered_depth,
                                  confidence_threshold, valid_count_threshold, warn=msgs.append)
                return (None if d is None else (i, d, None)), msgs
            raw = read_raw(dataset.timestamps[i], dataset.widths[i], dataset.heights[i])
            if raw is None:
                return None, msgs
            cm = None
            # the reference loads the confidence map only for a valid depth map (o3d_utils.py:109-142);
            # an invalid one is dropped by the device decode
            if use_confidence_filtered_depth and DepthDataIO.is_depth_map_valid(raw):
                cm = depth_data_io.load_confidence_map(side=side, timestamp=dataset.timestamps[i])
                if cm is None:
                    msgs.append(f"[Warning] Confidence map not found for timestamp {dataset.timestamps[i]}")
            return (i, raw, cm), msgs
        except Exception as e:  # noqa: BLE001 -- re-raised on the calling thread after the prefix
            return _Raised(i, e)

    def load_chunk(lo):
        """Host side of one chunk: file reads only (decode + mask run on the device), or the
        caller's own DataIO decode when it exposes no raw-buffer access; frames read by the I/O
        threads, results in frame order, cut at the first frame whose read raised."""
        hi = chunk_end(lo)
        items, msgs, err = [], [], None
        for r in io_pool().map(load_one, range(lo, hi)):
            if isinstance(r, _Raised):
                err = r
                break
            if r[0] is not None:
                items.append(r[0])
            msgs += r[1]
        return lo, hi, items, msgs, err

    def put_mask(st, j, cm):  # the reference's two masking comparisons (o3d_utils.py:131-142), as numpy makes them
        m = st.mask[j].view(np.bool_)
        np.less(cm.confidence_map, confidence_threshold, out=m)
        m |= cm.valid_count < valid_count_threshold

    def load_chunk_staged(lo, st):
        """load_chunk for a chunk of one frame size: the I/O threads read every frame straight into
        the reusable staging set `st` (raw buffer, and the confidence maps when masking) -- no
        per-chunk allocations, stacking or copies on the main thread.  A missing file leaves a zero
        raw buffer, which the device decode flags invalid (frame_ok 0: skipped, as the reference
        skips a missing frame)."""
        hi = chunk_end(lo)

        def one(j):  # 1: masked, 0: unmasked, -1: unmasked, confidence map not found (warned below)
            i = lo + j
            try:
                raw = read_raw(dataset.timestamps[i], dataset.widths[i], dataset.heights[i])
                if raw is None:
                    st.raw[j] = 0.0
                    return 0
                st.raw[j] = raw
                # the reference loads the confidence map only for a valid depth map (o3d_utils.py:109-142)
                if not use_confidence_filtered_depth or not DepthDataIO.is_depth_map_valid(raw):
                    return 0
                cm = depth_data_io.load_confidence_map(side=side, timestamp=dataset.timestamps[i])
                if cm is None:
                    return -1
                put_mask(st, j, cm)
                return 1
            except Exception as e:  # noqa: BLE001 -- re-raised on the calling thread after the prefix
                return _Raised(i, e)

        res = list(io_pool().map(one, range(hi - lo)))
        err = next((r for r in res if isinstance(r, _Raised)), None)
        if err is not None:  # the chunk ends before the frame that raised
            res = res[:err.index - lo]
        # in frame order, as the reference's loop prints them (on the calling thread, chunk by chunk)
        msgs = [f"[Warning] Confidence map not found for timestamp {dataset.timestamps[lo + j]}"
                for j, r in enumerate(res) if r < 0]
        return lo, lo + len(res), (st, np.array([r > 0 for r in res], bool)), msgs, err

    def load_chunk_native(lo, st):
        """load_chunk_staged through mqr_read_frames_masked: native threads pread the raw files into `st`
        and reduce the npz members to the mask bytes as they read them (on the I/O thread).  The frames
        the reader leaves to Python are finished by finish_native on the calling thread."""
        from . import _lib
        hi = chunk_end(lo)
        B = hi - lo
        H, W = st.raw.shape[1:]
        raw_path, conf_path = native
        ts = [dataset.timestamps[i] for i in range(lo, hi)]
        raws = (ctypes.c_char_p * B)(*[os.fsencode(str(raw_path(t))) for t in ts])
        confs = (ctypes.c_char_p * B)(*[os.fsencode(str(conf_path(t))) for t in ts]) if use_confidence_filtered_depth else None
        status = np.zeros(B, np.uint8)
        _lib.call("mqr_read_frames_masked", B, raws, confs, H, W, float(confidence_threshold),
                  count_threshold(valid_count_threshold), _lib.ptr(st.raw), _lib.ptr(st.mask) if confs else None,
                  _lib.ptr(status), io_threads())
        return lo, hi, ("native", st, status), [], None

    def finish_native(lo, hi, st, status):
        """The frames mqr_read_frames_masked left to Python (a raw file of the wrong size, a confidence
        npz it does not parse) through the standard loaders, in frame order, on the calling thread:
        confidence messages are printed only for frames whose depth map is valid -- the reference loads
        the confidence map only after is_depth_map_valid passed (o3d_utils.py:109-142) -- and a frame
        whose read raises ends the chunk there (returned as _Raised).  Returns (hi, has, err)."""
        from . import _lib
        B = hi - lo
        has = np.zeros(B, bool)
        for j in range(B):
            s = int(status[j])
            i = lo + j
            try:
                if s & _lib.MQR_FRAME_RAW_OTHER:
                    raw = read_raw(dataset.timestamps[i], dataset.widths[i], dataset.heights[i])  # raises as the reference
                    if raw is None:
                        continue
                    st.raw[j] = raw
                    s |= _lib.MQR_FRAME_RAW_OK
                if not (s & _lib.MQR_FRAME_RAW_OK) or not use_confidence_filtered_depth:
                    continue
                if s & _lib.MQR_FRAME_CONF_OK:
                    has[j] = True
                    continue
                if not DepthDataIO.is_depth_map_valid(st.raw[j]):
                    continue
                cm = (None if s & _lib.MQR_FRAME_CONF_MISSING else
                      depth_data_io.load_confidence_map(side=side, timestamp=dataset.timestamps[i]))
            except Exception as e:  # noqa: BLE001 -- re-raised by the caller after the prefix
                return i, has[:j], _Raised(i, e)
            if cm is None:
                print(f"[Warning] Confidence map not found for timestamp {dataset.timestamps[i]}")
                continue
            put_mask(st, j, cm)
            has[j] = True
        return hi, has, None

    stage = {}  # (H, W) -> DeviceBuffer of CHUNK decoded frames

    def device_buffer(H, W):
        from ._lib import DeviceBuffer
        buf = stage.get((H, W))
        if buf is None:
            buf = stage[(H, W)] = DeviceBuffer(4 * CHUNK * H * W, vbg.device_id)
        return buf

    def integrate_decoded(idx, buf, ok, H, W):
        if ok.any():
            K = intrinsics[idx].astype(np.float64)
            T = extrinsic_wc[idx].astype(np.float64)
            vbg.integrate_frames((buf, len(idx), H, W), K, T, frame_ok=ok.astype(np.uint8), depth_scale=1.0,
                                 depth_max=float(depth_max), trunc_voxel_multiplier=float(trunc_voxel_multiplier))

    def run(idx, frames, cms, H, W):
        K = intrinsics[idx].astype(np.float64)
        T = extrinsic_wc[idx].astype(np.float64)
        kw = dict(depth_scale=1.0, depth_max=float(depth_max), trunc_voxel_multiplier=float(trunc_voxel_multiplier))
        if read_raw is None:
            vbg.integrate_frames(np.stack(frames), K, T, **kw)
            return
        from .ingest import decode_depth_frames
        B = len(idx)
        buf = device_buffer(H, W)
        has = np.array([cm is not None for cm in cms], bool)
        conf = vc = None
        if has.any():
            conf = np.zeros((B, H, W), np.float64)
            vc = np.zeros((B, H, W), np.int32)
            for j, cm in enumerate(cms):
                if cm is not None:
                    conf[j] = cm.confidence_map
                    vc[j] = cm.valid_count
        _, ok = decode_depth_frames(np.stack(frames), [dataset.nears[i] for i in idx], [dataset.fars[i] for i in idx],
                                    conf=conf, valid_count=vc, has_mask=has,
                                    confidence_threshold=confidence_threshold,
                                    valid_count_threshold=valid_count_threshold, device=vbg.device_id,
                                    out_ptr=buf.ptr)
        integrate_decoded(idx, buf, ok, H, W)

    def run_staged(lo, hi, st, has):
        from .ingest import decode_depth_frames
        B = hi - lo
        H, W = st.raw.shape[1:]
        idx = np.arange(lo, hi)
        buf = device_buffer(H, W)
        any_mask = bool(has.any())
        _, ok = decode_depth_frames(st.raw[:B], [dataset.nears[i] for i in idx], [dataset.fars[i] for i in idx],
                                    mask=st.mask[:B] if any_mask else None,
                                    has_mask=has if any_mask else None, device=vbg.device_id, out_ptr=buf.ptr)
        integrate_decoded(idx, buf, ok, H, W)

    def uniform(lo):  # every frame of the chunk at lo has one size (the usual capture)
        hi = chunk_end(lo)
        return len({(int(dataset.heights[i]), int(dataset.widths[i])) for i in range(lo, hi)}) == 1

    def submit(pool, lo, turn):
        if read_raw is not None and uniform(lo):
            st = _host_stage(turn, min(CHUNK, n), int(dataset.heights[lo]), int(dataset.widths[lo]), use_confidence_filtered_depth)
            return pool.submit(load_chunk_native if native is not None else load_chunk_staged, lo, st)
        return pool.submit(load_chunk, lo)

    bar = None
    if show_progress:
        from tqdm import tqdm
        bar = tqdm(total=n, desc=desc, file=sys.stderr, dynamic_ncols=True, mininterval=0.1)
    with ThreadPoolExecutor(max_workers=1) as pool:
        # two staging sets alternate: the I/O threads fill chunk i + 1's while chunk i's is decoded
        turn = 0
        fut = submit(pool, 0, turn) if n else None
        while fut is not None:
            t0 = time.perf_counter()
            lo, hi, items, msgs, err = fut.result()
            t1 = time.perf_counter()
            times["wait_io"] += t1 - t0
            turn ^= 1
            # the next chunk's reads overlap this chunk's device work -- unless a read raised in this one
            end = chunk_end(lo)
            fut = submit(pool, end, turn) if end < n and err is None else None
            for m in msgs:  # this chunk's messages, in frame order, before its frames are integrated
                print(m)
            if isinstance(items, tuple) and items[0] == "native":
                hi, has, err = finish_native(lo, hi, items[1], items[2])
                if err is not None and fut is not None:  # never read past the frame that raised
                    fut.cancel()
                    fut = None
                items = (items[1], has)
            if isinstance(items, tuple):
                if hi > lo:
                    run_staged(lo, hi, *items)
            else:
                # consecutive runs of one frame size, in dataset order (the running average is order-dependent)
                j = 0
                while j < len(items):
                    k = j + 1
                    while k < len(items) and items[k][1].shape == items[j][1].shape:
                        k += 1
                    sel = items[j:k]
                    run(np.array([i for i, _, _ in sel]), [f for _, f, _ in sel], [c for _, _, c in sel],
                        *sel[0][1].shape)
                    j = k
            times["device"] += time.perf_counter() - t1
            times["chunks"] += 1
            if bar is not None:
                bar.update(hi - lo)
            if err is not None:
                if bar is not None:
                    bar.close()
                for b in stage.values():
                    b.free()
                raise err.exc
    if bar is not None:
        bar.close()
    for b in stage.values():
        b.free()
    last_integrate_times.__dict__.update(times)
    return vbg
