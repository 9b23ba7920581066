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
    print(json.dumps({"triangles": int(t.shape[0]), "build_ms": walls}), flush=True)


if __name__ == "__main__":
    main()
