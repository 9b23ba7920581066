"""Result containers returned by the fusion path (duck-type what the reference's callers use).

The reference consumes Open3D tensor geometry:
  * ``vbg.extract_point_cloud().to_legacy()`` (reconstruct_scene.py:90) and
    ``pcd.point.positions.shape[0]`` (refine_fragment_poses.py:39-42);
  * ``mesh.to_legacy()``, ``mesh.cpu()``, ``mesh.device``, ``mesh.to(device)``
    (reconstruct_scene.py:105-122, 186-198; o3d_utils.py:258, 304-307).
These classes expose the same attribute paths over numpy arrays; ``to_legacy()`` returns a real
Open3D legacy object when ``open3d`` is importable and otherwise returns ``self`` (which offers
``points`` / ``vertices`` / ``triangles`` / ``*_normals`` arrays and a binary PLY writer).
"""
from __future__ import annotations

import numpy as np


class Tensor:
    """Minimal host tensor facade (``.numpy()``, ``.shape``, ``.dtype``, indexing)."""

    def __init__(self, array: np.ndarray):
        self._a = np.asarray(array)

    def numpy(self) -> np.ndarray:
        return self._a

    @property
    def shape(self):
        return self._a.shape

    @property
    def dtype(self):
        return self._a.dtype

    def __len__(self):
        return len(self._a)

    def __getitem__(self, i):
        return self._a[i]

    def __array__(self, dtype=None, copy=None):
        return self._a if dtype is None else self._a.astype(dtype)

    def cpu(self):
        return self

    def __repr__(self):
        return f"mqr.Tensor(shape={self._a.shape}, dtype={self._a.dtype})"


class Image:
    """Depth image wrapper (stands in for o3d.t.geometry.Image over a float32 H x W array)."""

    def __init__(self, tensor=None, device=None):
        a = tensor.numpy() if hasattr(tensor, "numpy") else np.asarray(tensor)
        self._a = np.ascontiguousarray(a, dtype=np.float32)
        if self._a.ndim == 3 and self._a.shape[2] == 1:
            self._a = self._a[:, :, 0]
        self.device = device

    def as_tensor(self):
        return Tensor(self._a)

    def numpy(self):
        return self._a

    @property
    def rows(self):
        return self._a.shape[0]

    @property
    def columns(self):
        return self._a.shape[1]


class _AttrMap(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def _try_open3d():
    try:
        import open3d  # noqa: F401
        return open3d
    except Exception:
        return None


def _write_ply(path, verts, normals=None, tris=None):
    verts = np.asarray(verts, np.float32)
    n = len(verts)
    props = ["property float x", "property float y", "property float z"]
    cols = [verts]
    if normals is not None and len(normals) == n:
        props += ["property float nx", "property float ny", "property float nz"]
        cols.append(np.asarray(normals, np.float32))
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {n}"] + props
    if tris is not None:
        header += [f"element face {len(tris)}", "property list uchar int vertex_indices"]
    header.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode())
        f.write(np.ascontiguousarray(np.concatenate(cols, axis=1), dtype="<f4").tobytes())
        if tris is not None:
            t = np.asarray(tris, np.int32)
            rec = np.empty(len(t), dtype=[("c", "u1"), ("i", "<i4", (3,))])
            rec["c"] = 3
            rec["i"] = t
            f.write(rec.tobytes())


class PointCloud:
    def __init__(self, positions: np.ndarray, normals: np.ndarray, device=None):
        self.point = _AttrMap(positions=Tensor(positions), normals=Tensor(normals))
        self.device = device

    @property
    def points(self):
        return self.point.positions.numpy()

    @property
    def normals(self):
        return self.point.normals.numpy()

    def cpu(self):
        return self

    def to(self, device):
        self.device = device
        return self

    def to_legacy(self):
        o3d = _try_open3d()
        if o3d is None:
            return self
        pcd = o3d.geometry.PointCloud()
        pcd.points = o3d.utility.Vector3dVector(self.points.astype(np.float64))
        pcd.normals = o3d.utility.Vector3dVector(self.normals.astype(np.float64))
        return pcd

    def write_ply(self, path):
        _write_ply(path, self.points, self.normals)


class TriangleMesh:
    def __init__(self, vertices: np.ndarray, normals: np.ndarray, triangles: np.ndarray, device=None):
        self.vertex = _AttrMap(positions=Tensor(vertices), normals=Tensor(normals))
        self.triangle = _AttrMap(indices=Tensor(triangles))
        self.device = device

    @property
    def vertices(self):
        return self.vertex.positions.numpy()

    @property
    def vertex_normals(self):
        return self.vertex.normals.numpy()

    @property
    def triangles(self):
        return self.triangle.indices.numpy()

    def cpu(self):
        return self

    def to(self, device):
        self.device = device
        return self

    def to_legacy(self):
        o3d = _try_open3d()
        if o3d is None:
            return self
        m = o3d.geometry.TriangleMesh()
        m.vertices = o3d.utility.Vector3dVector(self.vertices.astype(np.float64))
        m.vertex_normals = o3d.utility.Vector3dVector(self.vertex_normals.astype(np.float64))
        m.triangles = o3d.utility.Vector3iVector(self.triangles.astype(np.int32))
        return m

    def write_ply(self, path):
        _write_ply(path, self.vertices, self.vertex_normals, self.triangles)
