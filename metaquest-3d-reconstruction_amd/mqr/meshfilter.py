"""filter_mesh_components on the GPU.

Same signature, messages and result as the reference's
``processing/reconstruction/utils/o3d_utils.py:241-321``: drop edge-connected triangle clusters
smaller than ``min_triangle_count`` (keep the largest if none qualifies), then the Open3D legacy
clean-up sequence (unreferenced vertices, degenerate / duplicated triangles, duplicated vertices,
non-manifold edges).  All of it runs in libmqr_hip.so (csrc/meshfilter.hip); non-manifold edges
are visited in ascending vertex-pair order where Open3D uses its hash-map order.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MQR_HOST, call, ptr
from .geometry import Tensor, TriangleMesh


def _device_inputs(mesh, device):
    """(pos, nrm or None, nv, tri, nt) device pointers when the tensor mesh lives in HBM on `device`."""
    from .geometry import device_ptr
    if not (hasattr(mesh, "vertex") and hasattr(mesh, "triangle")):
        return None
    v, t = mesh.vertex.positions, mesh.triangle.indices
    n = mesh.vertex.get("normals")
    pv, pt = device_ptr(v, device), device_ptr(t, device)
    if pv is None or pt is None or v.dtype != np.float32 or t.dtype != np.int32:
        return None
    pn = device_ptr(n, device) if n is not None and n.shape == v.shape and n.dtype == np.float32 else None
    return pv[0], None if pn is None else pn[0], v.shape[0], pt[0], t.shape[0]


def _arrays(mesh):
    if hasattr(mesh, "vertex") and hasattr(mesh, "triangle"):
        v = mesh.vertex.positions
        n = getattr(mesh.vertex, "normals", None)
        t = mesh.triangle.indices
    else:
        v, t = mesh.vertices, mesh.triangles
        n = getattr(mesh, "vertex_normals", None)
    v = np.ascontiguousarray(v.numpy() if hasattr(v, "numpy") else v, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(t.numpy() if hasattr(t, "numpy") else t, dtype=np.int32).reshape(-1, 3)
    if n is not None:
        n = np.ascontiguousarray(n.numpy() if hasattr(n, "numpy") else n, dtype=np.float32).reshape(-1, 3)
        if n.shape[0] != v.shape[0]:
            n = None
    return v, n, t


def filter_mesh_components_gpu(vertices, normals, triangles, min_triangle_count: int = 2000, device: int = 0):
    """Arrays in, (vertices, normals, triangles, stats dict) out."""
    v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(triangles, dtype=np.int32).reshape(-1, 3)
    n = None if normals is None else np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
    g = ctypes.c_void_p()
    stats = np.zeros(8, np.int64)
    call("mqr_mesh_filter_components", int(device), ptr(v), None if n is None else ptr(n), v.shape[0], ptr(t),
         t.shape[0], MQR_HOST, int(min_triangle_count), ctypes.byref(g), ptr(stats, _lib._i64p))
    try:
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        call("mqr_geom_counts", g, ctypes.byref(nv), ctypes.byref(nt))
        pos = np.empty((nv.value, 3), np.float32)
        nrm = np.empty((nv.value, 3), np.float32)
        tri = np.empty((nt.value, 3), np.int32)
        call("mqr_geom_copy", g, ptr(pos), ptr(nrm), ptr(tri) if nt.value else None, MQR_HOST)
    finally:
        call("mqr_geom_free", g)
    keys = ("input_triangles", "clusters", "kept_clusters", "small_cluster_triangles", "largest_cluster",
            "non_manifold_removed", "triangles", "vertices")
    return pos, (nrm if n is not None else None), tri, dict(zip(keys, (int(x) for x in stats)))


def _filter_device(mesh, dev_id, ins, min_triangle_count):
    """The tensor mesh in HBM, filtered in place of a host round trip; the result stays in HBM."""
    from .geometry import DeviceGeom
    pv, pn, nv, pt, nt = ins
    g = ctypes.c_void_p()
    stats = np.zeros(8, np.int64)
    call("mqr_mesh_filter_components", int(dev_id), ctypes.c_void_p(pv), None if pn is None else ctypes.c_void_p(pn), nv,
         ctypes.c_void_p(pt), nt, _lib.MQR_DEVICE, int(min_triangle_count), ctypes.byref(g), ptr(stats, _lib._i64p))
    geom = DeviceGeom(g, dev_id)
    keys = ("input_triangles", "clusters", "kept_clusters", "small_cluster_triangles", "largest_cluster",
            "non_manifold_removed", "triangles", "vertices")
    p, n, t = geom.tensors()
    if pn is None:
        n = Tensor(np.zeros((geom.nv, 3), np.float32))
    return p, n, t, dict(zip(keys, (int(x) for x in stats)))


def filter_mesh_components(mesh, min_triangle_count: int = 2000):
    """Drop-in for the reference's filter_mesh_components (o3d_utils.py:241-321).  A mesh in HBM (this
    package's extraction) is filtered there and the result stays there, as the reference's tensor mesh
    does on its CUDA device."""
    from .vbg import parse_device
    dev = getattr(mesh, "device", None)
    dev_id = parse_device(dev)
    ins = _device_inputs(mesh, dev_id)
    if ins is not None:
        if ins[4] == 0:
            print("[Warning] Mesh filtering: Input mesh has no triangles, returning as-is")
            return mesh
        pos, nrm, tri, st = _filter_device(mesh, dev_id, ins, min_triangle_count)
        return _report_filter(TriangleMesh(pos, nrm, tri, device=dev), st, min_triangle_count)
    v, n, t = _arrays(mesh)
    if t.shape[0] == 0:
        print("[Warning] Mesh filtering: Input mesh has no triangles, returning as-is")
        return mesh
    pos, nrm, tri, st = filter_mesh_components_gpu(v, n, t, min_triangle_count, dev_id)
    return _report_filter(TriangleMesh(pos, nrm if nrm is not None else np.zeros_like(pos), tri, device=dev), st,
                          min_triangle_count)


def _report_filter(out, st, min_triangle_count):
    """The reference's messages (o3d_utils.py:288-319) from the filter's statistics."""
    kept, comps = st["kept_clusters"], st["clusters"]
    if st["largest_cluster"] < min_triangle_count:  # no cluster qualified: the largest was kept
        print(f"[Warning] Mesh filtering: No components have >= {min_triangle_count} triangles. "
              f"Largest component has {st['largest_cluster']} triangles.")
        print("[Warning] Mesh filtering: Returning largest component only.")
    removed = comps - kept
    if removed > 0:
        print(f"[Info] Mesh filtering: Found {comps} connected component(s)")
        print(f"[Info] Mesh filtering: Removed {removed} small component(s) with < {min_triangle_count} triangles")
        print(f"[Info] Mesh filtering: Removed {st['small_cluster_triangles']} triangles from small components")
        print(f"[Info] Mesh filtering: Kept {kept} component(s) with >= {min_triangle_count} triangles")
        print(f"[Info] Mesh filtering: Final mesh has {st['triangles']} triangles (was {st['input_triangles']})")
    else:
        print(f"[Info] Mesh filtering: All {comps} component(s) have >= {min_triangle_count} triangles, "
              f"no filtering needed")
    return out
