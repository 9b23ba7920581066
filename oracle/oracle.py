"""ctypes wrapper for the CPU oracle (oracle/liborc.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module.  The product package (``mqr``) never imports it and never falls back to it.

The oracle restates the reference's hot path on the CPU (see mqr_oracle.c for the file:line
map): Open3D 0.19 VoxelBlockGrid touch / integrate / extract semantics (parity unpinned
against real Open3D, pinned by known-answer tests) and the numpy confidence estimator
(pinned by golden vectors generated from the reference, tests/golden/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborc.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "liborc.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_vbg_create.restype = ctypes.c_void_p
        L.orc_vbg_create.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_int64]
        L.orc_vbg_destroy.argtypes = [ctypes.c_void_p]
        L.orc_vbg_size.restype = ctypes.c_int64
        L.orc_vbg_size.argtypes = [ctypes.c_void_p]
        L.orc_set_threads.argtypes = [ctypes.c_int]
        L.orc_get_threads.restype = ctypes.c_int
        L.orc_touch.restype = ctypes.c_int
        L.orc_touch.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f64p, _f64p, ctypes.c_float, ctypes.c_int,
                                ctypes.c_float, ctypes.c_float, ctypes.c_float, _i32p, _i64p]
        L.orc_integrate.restype = ctypes.c_int
        L.orc_integrate.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int64, _f32p, ctypes.c_int, ctypes.c_int,
                                    _f64p, _f64p, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.orc_export.argtypes = [ctypes.c_void_p, _i32p, _f32p, _f32p]
        L.orc_import.restype = ctypes.c_int
        L.orc_import.argtypes = [ctypes.c_void_p, _i32p, _f32p, _f32p, ctypes.c_int64]
        L.orc_extract_points.restype = ctypes.c_int64
        L.orc_extract_points.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.POINTER(_f32p),
                                         ctypes.POINTER(_f32p)]
        L.orc_extract_mesh.restype = ctypes.c_int64
        L.orc_extract_mesh.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.POINTER(_f32p),
                                       ctypes.POINTER(_f32p), ctypes.POINTER(_i32p), _i64p]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_pixel_error_map.restype = ctypes.c_int
        L.orc_pixel_error_map.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p, _f32p,
                                          _f32p, ctypes.c_double, _f32p]
        L.orc_confidence.restype = ctypes.c_int
        L.orc_confidence.argtypes = [_f32p, _u8p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, _f64p, _i32p]
        L.orc_raycast.restype = ctypes.c_int
        L.orc_raycast.argtypes = [_f32p, ctypes.c_int64, _i32p, ctypes.c_int64, _f32p, ctypes.c_int64, _f32p, _i32p]
        L.orc_depth_boundary_mask.restype = ctypes.c_int
        L.orc_depth_boundary_mask.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                              ctypes.c_int, _f32p, _u8p]
        L.orc_color_map.restype = ctypes.c_int
        L.orc_color_map.argtypes = [_f32p, ctypes.c_int64, _u8p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    _f64p, _f64p, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_double, ctypes.c_int, _f32p, _i32p]
        L.orc_color_vertices.restype = ctypes.c_int
        L.orc_color_vertices.argtypes = [_f32p, ctypes.c_int64, _u8p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         _f64p, _f64p, ctypes.c_double, ctypes.c_double, ctypes.c_int, _f32p, _i32p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def set_threads(n: int) -> None:
    lib().orc_set_threads(int(n))


def get_threads() -> int:
    return int(lib().orc_get_threads())


def touch(depth, K, T, voxel_size, R, depth_scale, depth_max, trunc_mult):
    """Unique touched block keys (n,3) int32 (Appendix A.2), or raises like upstream."""
    depth = np.ascontiguousarray(depth, dtype=np.float32)
    H, W = depth.shape
    K = np.ascontiguousarray(K, dtype=np.float64)
    T = np.ascontiguousarray(T, dtype=np.float64)
    cap = 4 * (H // 4) * (W // 4)
    out = np.empty((max(cap, 1), 3), np.int32)
    n = ctypes.c_int64(0)
    rc = lib().orc_touch(_p(depth, _f32p), H, W, _p(K, _f64p), _p(T, _f64p), voxel_size, R, depth_scale,
                         depth_max, trunc_mult, _p(out, _i32p), ctypes.byref(n))
    if rc == 1:
        raise RuntimeError("No block is touched in TSDF volume, abort integration.")
    return out[: n.value].copy()


class OracleVBG:
    def __init__(self, voxel_size=0.01, block_resolution=16, block_count=1000):
        self.voxel_size = float(voxel_size)
        self.R = int(block_resolution)
        self._h = lib().orc_vbg_create(self.voxel_size, self.R, int(block_count))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_vbg_destroy(self._h)
            self._h = None

    def size(self):
        return int(lib().orc_vbg_size(self._h))

    def touch(self, depth, K, T, depth_scale=1.0, depth_max=3.0, trunc_mult=8.0):
        return touch(depth, K, T, self.voxel_size, self.R, depth_scale, depth_max, trunc_mult)

    def integrate(self, keys, depth, K, T, depth_scale=1.0, depth_max=3.0, trunc_mult=8.0):
        keys = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        depth = np.ascontiguousarray(depth, dtype=np.float32)
        H, W = depth.shape
        K = np.ascontiguousarray(K, dtype=np.float64)
        T = np.ascontiguousarray(T, dtype=np.float64)
        rc = lib().orc_integrate(self._h, _p(keys, _i32p), keys.shape[0], _p(depth, _f32p), H, W, _p(K, _f64p),
                                 _p(T, _f64p), depth_scale, depth_max, trunc_mult)
        if rc:
            raise RuntimeError("oracle integrate failed (%d)" % rc)

    def integrate_frame(self, depth, K, T, depth_scale=1.0, depth_max=3.0, trunc_mult=8.0):
        keys = self.touch(depth, K, T, depth_scale, depth_max, trunc_mult)
        self.integrate(keys, depth, K, T, depth_scale, depth_max, trunc_mult)
        return keys

    def export(self):
        """(keys (n,3) int32, tsdf (n,R,R,R) f32, weight (n,R,R,R) f32) in activation order."""
        n = self.size()
        R = self.R
        keys = np.empty((n, 3), np.int32)
        tsdf = np.empty((n, R, R, R), np.float32)
        wgt = np.empty((n, R, R, R), np.float32)
        lib().orc_export(self._h, _p(keys, _i32p), _p(tsdf, _f32p), _p(wgt, _f32p))
        return keys, tsdf, wgt

    def import_blocks(self, keys, tsdf, weight):
        keys = np.ascontiguousarray(keys, dtype=np.int32)
        tsdf = np.ascontiguousarray(tsdf, dtype=np.float32)
        weight = np.ascontiguousarray(weight, dtype=np.float32)
        rc = lib().orc_import(self._h, _p(keys, _i32p), _p(tsdf, _f32p), _p(weight, _f32p), keys.shape[0])
        if rc:
            raise RuntimeError("oracle import failed")

    def extract_points(self, weight_threshold=3.0):
        pp, nn = _f32p(), _f32p()
        n = lib().orc_extract_points(self._h, weight_threshold, ctypes.byref(pp), ctypes.byref(nn))
        pos = np.ctypeslib.as_array(pp, shape=(max(n, 1) * 3,))[: 3 * n].reshape(n, 3).copy()
        nrm = np.ctypeslib.as_array(nn, shape=(max(n, 1) * 3,))[: 3 * n].reshape(n, 3).copy()
        lib().orc_free(ctypes.cast(pp, ctypes.c_void_p))
        lib().orc_free(ctypes.cast(nn, ctypes.c_void_p))
        return pos, nrm

    def extract_mesh(self, weight_threshold=3.0):
        vp, np_, tp = _f32p(), _f32p(), _i32p()
        nt = ctypes.c_int64(0)
        nv = lib().orc_extract_mesh(self._h, weight_threshold, ctypes.byref(vp), ctypes.byref(np_),
                                    ctypes.byref(tp), ctypes.byref(nt))
        t = nt.value
        verts = np.ctypeslib.as_array(vp, shape=(max(nv, 1) * 3,))[: 3 * nv].reshape(nv, 3).copy()
        nrms = np.ctypeslib.as_array(np_, shape=(max(nv, 1) * 3,))[: 3 * nv].reshape(nv, 3).copy()
        tris = np.ctypeslib.as_array(tp, shape=(max(t, 1) * 3,))[: 3 * t].reshape(t, 3).copy()
        for q in (vp, np_, tp):
            lib().orc_free(ctypes.cast(q, ctypes.c_void_p))
        return verts, nrms, tris


def pixel_error_map(K, Tcw, Tcw_inv, ref, ref_depth, tgt, tgt_depth, depth_max=3.0):
    """compute_pixel_error_map (compute_pixel_error_map.py:120-220) for one frame pair."""
    ref_depth = np.ascontiguousarray(ref_depth, dtype=np.float32)
    tgt_depth = np.ascontiguousarray(tgt_depth, dtype=np.float32)
    H, W = ref_depth.shape
    K = np.ascontiguousarray(K, dtype=np.float32)
    Tcw = np.ascontiguousarray(Tcw, dtype=np.float32)
    Tcw_inv = np.ascontiguousarray(Tcw_inv, dtype=np.float32)
    out = np.empty((H, W), np.float32)
    lib().orc_pixel_error_map(_p(ref_depth, _f32p), _p(tgt_depth, _f32p), H, W, _p(K[ref], _f32p),
                              _p(K[tgt], _f32p), _p(Tcw[ref], _f32p), _p(Tcw_inv[tgt], _f32p), _p(Tcw[tgt], _f32p),
                              float(depth_max), _p(out, _f32p))
    return out


def confidence(depths, K, Tcw, Tcw_inv, ref, target_frame_range=10, depth_max=3.0, error_threshold=0.05,
               frame_valid=None):
    """build_confidence_map (estimate_depth_confidences.py:15-79) -> (confidence f64, valid_count i32)."""
    depths = np.ascontiguousarray(depths, dtype=np.float32)
    N, H, W = depths.shape
    K = np.ascontiguousarray(K, dtype=np.float32)
    Tcw = np.ascontiguousarray(Tcw, dtype=np.float32)
    Tcw_inv = np.ascontiguousarray(Tcw_inv, dtype=np.float32)
    fv = None if frame_valid is None else np.ascontiguousarray(frame_valid, dtype=np.uint8)
    conf = np.empty((H, W), np.float64)
    valid = np.empty((H, W), np.int32)
    lib().orc_confidence(_p(depths, _f32p), None if fv is None else _p(fv, _u8p), _p(K, _f32p), _p(Tcw, _f32p),
                         _p(Tcw_inv, _f32p), N, H, W, int(ref), int(target_frame_range), float(depth_max),
                         float(error_threshold), _p(conf, _f64p), _p(valid, _i32p))
    return conf, valid


def raycast(vertices, triangles, rays):
    """Closest-hit t (inf on miss) and primitive index (-1) per ray, brute force in float64."""
    V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    T = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 3)
    r = np.ascontiguousarray(rays, dtype=np.float32)
    shape = r.shape[:-1]
    r = r.reshape(-1, 6)
    t = np.empty(r.shape[0], np.float32)
    pr = np.empty(r.shape[0], np.int32)
    lib().orc_raycast(_p(V, _f32p), V.shape[0], _p(T, _i32p), T.shape[0], _p(r, _f32p), r.shape[0], _p(t, _f32p),
                      _p(pr, _i32p))
    return t.reshape(shape), pr.reshape(shape)


def color_vertices(vertices, images, depths, K, T_wc, max_depth=2.5, visibility_threshold=0.03, margin=10):
    """Per-vertex colour averaging over keyframes (colour-map pipeline input, row f1) ->
    (colours (V,3) float32, counts (V,) int32)."""
    V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    im = np.ascontiguousarray(images, dtype=np.uint8)
    N, H, W = im.shape[:3]
    d = np.ascontiguousarray(depths, dtype=np.float32).reshape(N, H, W)
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(N, 9)
    T = np.ascontiguousarray(T_wc, dtype=np.float64).reshape(N, 16)
    out = np.empty((len(V), 3), np.float32)
    cnt = np.empty(len(V), np.int32)
    lib().orc_color_vertices(_p(V, _f32p), len(V), _p(im, _u8p), _p(d, _f32p), N, H, W, _p(K, _f64p), _p(T, _f64p),
                             float(max_depth), float(visibility_threshold), int(margin), _p(out, _f32p),
                             _p(cnt, _i32p))
    return out, cnt


def depth_boundary_mask(t_hit, depth_trunc=3.0, disc_thr=0.1, half=3):
    """(truncated RGBD depth (H,W) f32, boundary mask (H,W) u8) of one colour-aligned depth map."""
    t = np.ascontiguousarray(t_hit, dtype=np.float32)
    H, W = t.shape
    d = np.empty((H, W), np.float32)
    m = np.empty((H, W), np.uint8)
    lib().orc_depth_boundary_mask(_p(t, _f32p), H, W, float(depth_trunc), float(disc_thr), int(half), _p(d, _f32p),
                                  _p(m, _u8p))
    return d, m


def color_map(vertices, images, t_hit, K, T_wc, max_depth=2.5, visibility_threshold=0.03, margin=10, disc_thr=0.1,
              half=3, depth_trunc=3.0, knn=3):
    """run_rigid_optimizer's vertex colours with the poses as given (see orc_color_map) ->
    (colours (V,3) float32, counts (V,) int32; 0 for vertices filled from their knn sampled ones)."""
    V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    im = np.ascontiguousarray(images, dtype=np.uint8)
    N, H, W = im.shape[:3]
    d = np.ascontiguousarray(t_hit, dtype=np.float32).reshape(N, H, W)
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(N, 9)
    T = np.ascontiguousarray(T_wc, dtype=np.float64).reshape(N, 16)
    out = np.empty((len(V), 3), np.float32)
    cnt = np.empty(len(V), np.int32)
    lib().orc_color_map(_p(V, _f32p), len(V), _p(im, _u8p), _p(d, _f32p), N, H, W, _p(K, _f64p), _p(T, _f64p),
                        float(max_depth), float(visibility_threshold), int(margin), float(disc_thr), int(half),
                        float(depth_trunc), int(knn), _p(out, _f32p), _p(cnt, _i32p))
    return out, cnt
