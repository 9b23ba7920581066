#!/usr/bin/env python3
"""Wall time of mqr_scene_build on fresh scenes (a grid mesh of ~2.1 M triangles, the C2 mesh's size) and
the kernels' share (run it under `rocprofv3 --kernel-trace --stats` for the per-kernel sums): is the build
bound by its kernels or by its per-build allocations?  One JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))


def grid_mesh(n):
    """A wavy n x n vertex grid, 2 (n - 1)^2 triangles."""
    y, x = np.meshgrid(np.arange(n, dtype=np.float32), np.arange(n, dtype=np.float32), indexing="ij")
    z = 0.05 * np.sin(x * 0.1) * np.cos(y * 0.07)
    v = np.stack([x * 0.004, y * 0.004, z], -1).reshape(-1, 3).astype(np.float32)
    i = np.arange(n * n, dtype=np.int32).reshape(n, n)
    a, b, c, d = i[:-1, :-1].ravel(), i[:-1, 1:].ravel(), i[1:, :-1].ravel(), i[1:, 1:].ravel()
    t = np.concatenate([np.stack([a, b, c], -1), np.stack([b, d, c], -1)]).astype(np.int32)
    return v, t


def main():
    from mqr import _lib
    L = _lib.load()
    v, t = grid_mesh(1025)
    walls = []
    for _ in range(6):
        s = ctypes.c_void_p()
        _lib.call("mqr_scene_create", 0, ctypes.byref(s))
        gid = ctypes.c_uint32()
        _lib.call("mqr_scene_add_triangles", s, _lib.ptr(v), v.shape[0], _lib.ptr(t), t.shape[0], _lib.MQR_HOST,
                  ctypes.byref(gid))
        t0 = time.perf_counter()
        _lib.call("mqr_scene_build", s)
        walls.append((time.perf_counter() - t0) * 1e3)
        L.mqr_scene_destroy(s)
    # pinhole casts of the last scene shape: 64 VGA frames looking down at the grid, t_hit to the host
    s = ctypes.c_void_p()
    _lib.call("mqr_scene_create", 0, ctypes.byref(s))
    gid = ctypes.c_uint32()
    _lib.call("mqr_scene_add_triangles", s, _lib.ptr(v), v.shape[0], _lib.ptr(t), t.shape[0], _lib.MQR_HOST,
              ctypes.byref(gid))
    F, H, W = 64, 480, 640
    K = np.tile(np.array([[500.0, 0, 320], [0, 500.0, 240], [0, 0, 1]]), (F, 1, 1))
    T = np.tile(np.eye(4), (F, 1, 1))
    T[:, 0, 3] = np.linspace(1.0, 3.0, F)
    T[:, 1, 3] = 2.0
    T[:, 2, 3] = 2.0
    T[:, 1, 1] = T[:, 2, 2] = -1.0  # looking down -z
    Kc, Tc = np.ascontiguousarray(K), np.ascontiguousarray(T)
    th = np.empty((F, H, W), np.float32)
    casts = []
    for _ in range(7):
        t0 = time.perf_counter()
        _lib.call("mqr_scene_cast_pinhole", s, _lib.ptr(Kc, _lib._f64p), _lib.ptr(Tc, _lib._f64p), F, H, W,
                  _lib.ptr(th), None, None, None, None, _lib.MQR_HOST)
        casts.append((time.perf_counter() - t0) * 1e3)
    L.mqr_scene_destroy(s)
    print(json.dumps({"lib": os.environ.get("MQR_HIP_LIB", "default"), "triangles": int(t.shape[0]),
                      "build_ms": walls, "cast64_ms": casts, "hit_fraction": float(np.isfinite(th).mean())}), flush=True)


if __name__ == "__main__":
    main()
