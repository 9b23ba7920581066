"""Device-side depth ingestion.

``decode_depth_frames`` turns a stack of raw Quest depth buffers (NDC in [0, 1], as stored in
``<side>_depth/<ts>.raw``) into metric depth on the GPU, together with the reference's
frame-validity verdict and the confidence mask -- the device twin of

    DepthDataIO.load_depth_map + is_depth_map_valid     scripts/dataio/depth_data_io.py:33-53, 80-85
    convert_depth_to_linear                             scripts/utils/depth_utils.py:21-46
    load_depth_map's confidence masking                 processing/reconstruction/utils/o3d_utils.py:131-142

numpy's promotion is part of the result: ``near`` / ``far`` given as numpy float64 scalars (what
the pipeline passes, ``DepthDataset.nears[i]``) make numpy >= 2 divide in float64, Python floats
keep the decode in float32.  The kernel reproduces both, per frame, from the operand types.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import MQR_DEVICE, MQR_HOST, call, ptr


def _strong(x) -> int:
    if isinstance(x, np.generic):
        if isinstance(x, np.float64):
            return 1
        raise TypeError(f"near/far of numpy type {type(x).__name__} are not supported (float64 or Python float)")
    return 0


def count_threshold(valid_count_threshold) -> int:
    """The int32 threshold t' with (count < t') == (count < valid_count_threshold) for every int32 count,
    as numpy compares an int32 map with a Python int or float threshold."""
    return int(min(max(math.ceil(valid_count_threshold), -(2 ** 31)), 2 ** 31 - 1))


def decode_depth_frames(raw, nears: Sequence, fars: Sequence, conf: Optional[np.ndarray] = None,
                        valid_count: Optional[np.ndarray] = None, has_mask: Optional[Sequence[bool]] = None,
                        confidence_threshold: float = 0.0, valid_count_threshold: int = 0, device: int = 0,
                        out_ptr: Optional[int] = None, mask: Optional[np.ndarray] = None):
    """raw: (N,H,W) float32 numpy array, or a tuple (device_ptr, N, H, W) of raw buffers in HBM.
    The confidence mask of the frames selected by `has_mask` comes either as the maps (`conf`,
    `valid_count` and the thresholds) or, already reduced, as `mask` ((N,H,W) uint8 host array, nonzero =
    depth 0; mqr_decode_depth_masked: 1 byte per pixel to stage instead of 12).

    Returns (depth, frame_ok): depth is a (N,H,W) float32 numpy array, or None when `out_ptr`
    (a device pointer with room for N*H*W floats) received it; frame_ok is (N,) bool."""
    if isinstance(raw, tuple):
        rptr, N, H, W = raw
        raw_arg, raw_loc = ctypes_ptr(rptr), MQR_DEVICE
    else:
        raw = np.ascontiguousarray(raw, dtype=np.float32)
        N, H, W = raw.shape
        raw_arg, raw_loc = ptr(raw), MQR_HOST
    nears = list(nears)
    fars = list(fars)
    if len(nears) != N or len(fars) != N:
        raise ValueError("one near / far per frame")
    strong = np.array([_strong(n) | (_strong(f) << 1) for n, f in zip(nears, fars)], np.uint8)
    n64 = np.array([float(x) for x in nears], np.float64)
    f64 = np.array([float(x) for x in fars], np.float64)
    mask_arg = None
    conf_arg = vc_arg = None
    ok = np.zeros(N, np.uint8)
    out = None
    if out_ptr is None:
        out = np.empty((N, H, W), np.float32)
        out_arg, out_loc = ptr(out), MQR_HOST
    else:
        out_arg, out_loc = ctypes_ptr(out_ptr), MQR_DEVICE
    if mask is not None:
        m8 = None
        if has_mask is not None and np.any(has_mask):
            mask_arg = ptr(np.ascontiguousarray(np.asarray(has_mask, dtype=np.uint8).reshape(N)), _lib._u8p)
            m8 = np.asarray(mask)
            if m8.dtype != np.uint8 or m8.shape != (N, H, W) or not m8.flags.c_contiguous:
                raise ValueError("mask must be a C-contiguous (N, H, W) uint8 array")
        call("mqr_decode_depth_masked", int(device), raw_arg, raw_loc, N, H, W, ptr(n64, _lib._f64p),
             ptr(f64, _lib._f64p), ptr(strong, _lib._u8p), None if m8 is None else ptr(m8), mask_arg, MQR_HOST,
             out_arg, out_loc, ptr(ok, _lib._u8p))
        return out, ok.astype(bool)
    if has_mask is not None and np.any(has_mask):
        mask = np.ascontiguousarray(np.asarray(has_mask, dtype=np.uint8).reshape(N))
        conf = np.ascontiguousarray(conf, dtype=np.float64).reshape(N, H, W)
        valid_count = np.ascontiguousarray(valid_count, dtype=np.int32).reshape(N, H, W)
        mask_arg, conf_arg, vc_arg = ptr(mask, _lib._u8p), ptr(conf), ptr(valid_count)
    call("mqr_decode_depth", int(device), raw_arg, raw_loc, N, H, W, ptr(n64, _lib._f64p), ptr(f64, _lib._f64p),
         ptr(strong, _lib._u8p), conf_arg, vc_arg, mask_arg, MQR_HOST, float(confidence_threshold),
         count_threshold(valid_count_threshold), out_arg, out_loc, ptr(ok, _lib._u8p))
    return out, ok.astype(bool)


def ctypes_ptr(p):
    """Device pointer from an int, a ctypes.c_void_p or an object with .ptr (DeviceBuffer)."""
    import ctypes
    if hasattr(p, "ptr"):
        p = p.ptr
    if isinstance(p, ctypes.c_void_p):
        return p
    return ctypes.c_void_p(int(p))
