"""Triangle-mesh ray casting on the GPU.

Stands in for ``o3d.t.geometry.RaycastingScene`` as the reference uses it for colour-aligned
depth (reconstruct_scene.py:197-201; o3d_utils.py:324-341; optimize_color_pose.py:24-47):

    scene = RaycastingScene(device=...)
    scene.add_triangles(mesh)                       # or (vertex_positions, triangle_indices)
    rays = RaycastingScene.create_rays_pinhole(K, T_wc, width_px, height_px)
    depth = scene.cast_rays(rays)['t_hit'].cpu().numpy()

The BVH is built on the device (libmqr_hip.so, csrc/raycast.hip) at the first query after the
geometry changed.  ``cast_pinhole`` is the fused path (rays generated on the device, identical
to create_rays_pinhole + cast_rays).  t_hit is inf where a ray hits nothing; ids are
0xFFFFFFFF (``INVALID_ID``) there.  A mesh already in HBM (this package's extraction or mesh filter)
is added in place, and the cast results stay in HBM as Open3D's do on a CUDA device (copied to the
host on the first ``.numpy()``), so ``color_map`` can take them without a round trip.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib
from ._lib import MQR_HOST, call, ptr
from .geometry import DeviceArray, Tensor, device_ptr

INVALID_ID = 0xFFFFFFFF


def _mesh_arrays(mesh_or_vertices, triangles=None):
    if triangles is not None:
        v, t = mesh_or_vertices, triangles
    elif hasattr(mesh_or_vertices, "vertex") and hasattr(mesh_or_vertices, "triangle"):   # tensor mesh
        v, t = mesh_or_vertices.vertex.positions, mesh_or_vertices.triangle.indices
    else:                                                                                # legacy mesh
        v, t = mesh_or_vertices.vertices, mesh_or_vertices.triangles
    v = v.numpy() if hasattr(v, "numpy") else np.asarray(v)
    t = t.numpy() if hasattr(t, "numpy") else np.asarray(t)
    return (np.ascontiguousarray(v, dtype=np.float32).reshape(-1, 3),
            np.ascontiguousarray(t, dtype=np.int32).reshape(-1, 3))


def _device_mesh(mesh_or_vertices, triangles, device_id):
    """((vertex ptr, nv), (triangle ptr, nt)) when positions (float32 (n,3)) and indices (int32 (m,3)) are
    Tensors in HBM on `device_id`, else None."""
    if triangles is not None:
        v, t = mesh_or_vertices, triangles
    elif hasattr(mesh_or_vertices, "vertex") and hasattr(mesh_or_vertices, "triangle"):
        v, t = mesh_or_vertices.vertex.positions, mesh_or_vertices.triangle.indices
    else:
        return None
    pv, pt = device_ptr(v, device_id), device_ptr(t, device_id)
    if pv is None or pt is None or v.dtype != np.float32 or t.dtype != np.int32 or v.shape[-1:] != (3,) \
            or t.shape[-1:] != (3,):
        return None
    return (pv[0], int(np.prod(v.shape[:-1]))), (pt[0], int(np.prod(t.shape[:-1])))


def _pinhole_params(K, T):
    """float32(R^T K^-1) and float32(-R^T t), as Open3D's CreateRaysPinhole forms them."""
    K = np.asarray(K, np.float64).reshape(3, 3)
    T = np.asarray(T, np.float64).reshape(4, 4)
    if K[0, 1] == 0 and K[1, 0] == 0 and K[2, 0] == 0 and K[2, 1] == 0 and K[2, 2] == 1:
        inv = np.array([[1.0 / K[0, 0], 0.0, -K[0, 2] / K[0, 0]],
                        [0.0, 1.0 / K[1, 1], -K[1, 2] / K[1, 1]],
                        [0.0, 0.0, 1.0]])
    else:
        inv = np.linalg.inv(K)
    RT = T[:3, :3].T
    m = np.empty((3, 3))
    for r in range(3):
        for k in range(3):
            m[r, k] = (RT[r, 0] * inv[0, k] + RT[r, 1] * inv[1, k]) + RT[r, 2] * inv[2, k]
    c = -((RT[:, 0] * T[0, 3] + RT[:, 1] * T[1, 3]) + RT[:, 2] * T[2, 3])
    return m.astype(np.float32), c.astype(np.float32)


class RaycastingScene:
    def __init__(self, nthreads: int = 0, device=None):
        from .vbg import parse_device
        self.device_id = parse_device(device)
        h = ctypes.c_void_p()
        call("mqr_scene_create", self.device_id, ctypes.byref(h))
        self._h = h
        self._ngeom = 0

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and self._h.value:
                call("mqr_scene_destroy", self._h)
                self._h = None
        except Exception:
            pass

    def add_triangles(self, vertex_positions, triangle_indices=None) -> int:
        gid = ctypes.c_uint32()
        dev = _device_mesh(vertex_positions, triangle_indices, self.device_id)
        if dev is not None:  # the mesh is in HBM on this scene's device: no host round trip
            (pv, nv), (pt, nt) = dev
            call("mqr_scene_add_triangles", self._h, ctypes.c_void_p(pv), nv, ctypes.c_void_p(pt), nt, _lib.MQR_DEVICE,
                 ctypes.byref(gid))
            self._ngeom += 1
            return int(gid.value)
        v, t = _mesh_arrays(vertex_positions, triangle_indices)
        call("mqr_scene_add_triangles", self._h, ptr(v), v.shape[0], ptr(t), t.shape[0], MQR_HOST,
             ctypes.byref(gid))
        self._ngeom += 1
        return int(gid.value)

    def triangle_count(self) -> int:
        n = ctypes.c_int64()
        call("mqr_scene_triangle_count", self._h, ctypes.byref(n))
        return int(n.value)

    @staticmethod
    def create_rays_pinhole(intrinsic_matrix, extrinsic_matrix, width_px: int, height_px: int) -> Tensor:
        """(H, W, 6) float32 rays: origin = camera centre, direction = R^T K^-1 (x+0.5, y+0.5, 1)."""
        K = intrinsic_matrix.numpy() if hasattr(intrinsic_matrix, "numpy") else intrinsic_matrix
        T = extrinsic_matrix.numpy() if hasattr(extrinsic_matrix, "numpy") else extrinsic_matrix
        m, c = _pinhole_params(K, T)
        px = np.arange(width_px, dtype=np.float32) + np.float32(0.5)
        py = np.arange(height_px, dtype=np.float32) + np.float32(0.5)
        px, py = np.meshgrid(px, py)
        rays = np.empty((height_px, width_px, 6), np.float32)
        rays[..., :3] = c
        for r in range(3):
            rays[..., 3 + r] = (m[r, 0] * px + m[r, 1] * py) + m[r, 2]
        return Tensor(rays)

    def _outputs(self, n, full):
        """Device buffers for the cast's results: (t_hit, geometry ids, primitive ids, uvs, normals)."""
        from ._lib import DeviceBuffer
        specs = [(np.float32, ())] + ([(np.uint32, ()), (np.uint32, ()), (np.float32, (2,)), (np.float32, (3,))]
                                      if full else [])
        out = [(DeviceBuffer(max(4, n * np.dtype(dt).itemsize * int(np.prod(k, dtype=np.int64))), self.device_id),
                dt, k) for dt, k in specs]
        return out + [None] * (5 - len(out))

    @staticmethod
    def _p(o):
        return None if o is None else o[0].ptr

    def _tensors(self, outs, shape, full):
        """The results as Tensors over their device buffers (host copies on first access)."""
        names = ["t_hit"] + (["geometry_ids", "primitive_ids", "primitive_uvs", "primitive_normals"] if full else [])
        return {nm: Tensor(DeviceArray(buf, buf.ptr.value, shape + k, dt, self.device_id))
                for nm, (buf, dt, k) in zip(names, outs)}

    def cast_rays(self, rays, nthreads: int = 0, full: bool = True) -> dict:
        r = rays.numpy() if hasattr(rays, "numpy") else np.asarray(rays)
        shape = r.shape[:-1]
        r = np.ascontiguousarray(r, dtype=np.float32).reshape(-1, 6)
        n = r.shape[0]
        outs = self._outputs(n, full)
        t, g, p, uv, nr = outs
        call("mqr_scene_cast_rays", self._h, ptr(r), n, MQR_HOST, self._p(t), self._p(g), self._p(p), self._p(uv),
             self._p(nr), _lib.MQR_DEVICE)
        return self._tensors([o for o in outs if o is not None], tuple(shape), full)

    def cast_pinhole(self, intrinsics, extrinsics, width_px: int, height_px: int, full: bool = False) -> dict:
        """Fused create_rays_pinhole + cast_rays for one camera (K (3,3), T_wc (4,4)) or a stack
        (n,3,3) / (n,4,4) of same-size cameras; outputs shaped (n, H, W[, k]) or (H, W[, k])."""
        K = np.ascontiguousarray(intrinsics, dtype=np.float64)
        T = np.ascontiguousarray(extrinsics, dtype=np.float64)
        single = K.ndim == 2
        K = K.reshape(-1, 3, 3)
        T = T.reshape(-1, 4, 4)
        nf = K.shape[0]
        n = nf * height_px * width_px
        outs = self._outputs(n, full)
        t, g, p, uv, nr = outs
        call("mqr_scene_cast_pinhole", self._h, ptr(K, _lib._f64p), ptr(T, _lib._f64p), nf, int(height_px),
             int(width_px), self._p(t), self._p(g), self._p(p), self._p(uv), self._p(nr), _lib.MQR_DEVICE)
        shape = (height_px, width_px) if single else (nf, height_px, width_px)
        return self._tensors([o for o in outs if o is not None], shape, full)


def raycast_in_color_view(scene: RaycastingScene, dataset, batch: int = 16):
    """Generator of colour-aligned depth maps, one (H, W) float32 per dataset frame in order
    (reference o3d_utils.py:324-341); consecutive same-size frames are cast together."""
    from .o3d_utils import compute_o3d_intrinsic_matrices
    K = compute_o3d_intrinsic_matrices(dataset).astype(np.float32).astype(np.float64)
    T = dataset.transforms.extrinsics_wc.astype(np.float32).astype(np.float64)
    n = len(dataset)
    i = 0
    while i < n:
        w, h = int(dataset.widths[i]), int(dataset.heights[i])
        j = i + 1
        while j < n and j - i < batch and int(dataset.widths[j]) == w and int(dataset.heights[j]) == h:
            j += 1
        depth = scene.cast_pinhole(K[i:j], T[i:j], w, h)["t_hit"].numpy()
        for k in range(j - i):
            yield depth[k]
        i = j
