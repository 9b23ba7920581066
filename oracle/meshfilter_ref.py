"""CPU restatement of filter_mesh_components (reference o3d_utils.py:241-321).  TEST
INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

The reference calls Open3D legacy TriangleMesh methods (Open3D 0.19, not installed here), so
this follows their published algorithms (upstream cpp/open3d/geometry/TriangleMesh.cpp):
ClusterConnectedTriangles (edge adjacency, BFS in triangle order), RemoveTrianglesByMask,
RemoveUnreferencedVertices, RemoveDegenerateTriangles, RemoveDuplicatedTriangles (rotation
canonical key, first kept), RemoveDuplicatedVertices (exact coordinates, first kept),
RemoveNonManifoldEdges (drop smallest-area triangles of edges with > 2, zero-area triangles
dropped; edges visited in ascending (v_min, v_max) order -- Open3D's unordered_map order is not
reproducible).  Parity against Open3D itself: unpinned.
"""
from __future__ import annotations

import numpy as np


def _edges(tri):
    a = tri[:, [0, 1, 2]].reshape(-1)
    b = tri[:, [1, 2, 0]].reshape(-1)
    lo, hi = np.minimum(a, b).astype(np.int64), np.maximum(a, b).astype(np.int64)
    return lo << 32 | hi


def cluster_connected_triangles(tri):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    n = tri.shape[0]
    keys = _edges(tri)
    slot = np.argsort(keys, kind="stable")
    k = keys[slot]
    same = np.nonzero(k[1:] == k[:-1])[0]
    a, b = slot[same] // 3, slot[same + 1] // 3
    g = coo_matrix((np.ones(len(a)), (a, b)), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    first = np.full(lab.max() + 1, n, np.int64)
    np.minimum.at(first, lab, np.arange(n))
    order = np.argsort(first, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    clusters = rank[lab]
    counts = np.bincount(clusters)
    return clusters, counts


def _remove_unreferenced(v, nrm, tri):
    used = np.zeros(len(v), bool)
    used[tri.reshape(-1)] = True
    new = np.cumsum(used) - 1
    return v[used], (None if nrm is None else nrm[used]), new[tri].astype(np.int32)


def _canon(tri):
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    out = np.empty_like(tri)
    m1 = (a <= b) & (a <= c)
    m2 = (a <= b) & ~(a <= c)
    m3 = ~(a <= b) & (b <= c)
    m4 = ~(a <= b) & ~(b <= c)
    out[m1] = tri[m1][:, [0, 1, 2]]
    out[m2] = tri[m2][:, [2, 0, 1]]
    out[m3] = tri[m3][:, [1, 2, 0]]
    out[m4] = tri[m4][:, [2, 0, 1]]
    return out


def _first_occurrence(keys):
    _, idx = np.unique(keys, axis=0, return_index=True)
    keep = np.zeros(len(keys), bool)
    keep[idx] = True
    return keep


def _area(v, tri):
    p = v.astype(np.float64)
    p0, p1, p2 = p[tri[:, 0]], p[tri[:, 1]], p[tri[:, 2]]
    x, y = p0 - p1, p0 - p2
    c = np.cross(x, y)
    return 0.5 * np.sqrt((c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) + c[:, 2] * c[:, 2])


def filter_mesh_components(v, nrm, tri, min_triangle_count=2000):
    v = np.asarray(v, np.float32)
    tri = np.asarray(tri, np.int32)
    clusters, counts = cluster_connected_triangles(tri)
    valid = np.nonzero(counts >= min_triangle_count)[0]
    if len(valid) == 0:
        valid = np.array([np.argmax(counts)])
    mask = np.isin(clusters, valid)
    stats = {"clusters": len(counts), "kept_clusters": len(valid), "small_cluster_triangles": int((~mask).sum()),
             "largest_cluster": int(counts.max())}
    if (~mask).any():
        tri = tri[mask]
        v, nrm, tri = _remove_unreferenced(v, nrm, tri)
    tri = tri[(tri[:, 0] != tri[:, 1]) & (tri[:, 1] != tri[:, 2]) & (tri[:, 2] != tri[:, 0])]
    if len(tri) > 1:
        tri = tri[_first_occurrence(_canon(tri))]
    # duplicated vertices: +0 == -0, NaN never equal
    if len(v) > 1:
        vk = v.copy()
        vk[vk == 0] = 0.0
        bits = vk.view(np.uint32).astype(np.int64)
        nan = np.isnan(v).any(axis=1)
        keys = np.concatenate([bits, np.where(nan, np.arange(len(v)), -1)[:, None]], axis=1)
        _, first_idx, inv = np.unique(keys, axis=0, return_index=True, return_inverse=True)
        rep = first_idx[inv.reshape(-1)]
        keepv = rep == np.arange(len(v))
        newidx = np.cumsum(keepv) - 1
        tri = newidx[rep][tri].astype(np.int32)
        v = v[keepv]
        nrm = None if nrm is None else nrm[keepv]
    # non-manifold edges
    n_before = len(tri)
    while True:
        area = _area(v, tri)
        keys = _edges(tri)
        order = np.argsort(keys, kind="stable")
        ks = keys[order]
        starts = np.r_[0, np.nonzero(ks[1:] != ks[:-1])[0] + 1]
        ends = np.r_[starts[1:], len(ks)]
        manifold = True
        for s, e in zip(starts, ends):
            if e - s <= 2:
                continue
            manifold = False
            tris = order[s:e] // 3
            to_delete = int((area[tris] > 0).sum()) - 2
            while to_delete > 0:
                best, ba = -1, np.inf
                for t in tris:
                    if area[t] > 0 and area[t] < ba:
                        best, ba = t, area[t]
                area[best] = -1
                to_delete -= 1
        tri = tri[area > 0]
        if manifold:
            break
    stats["non_manifold_removed"] = n_before - len(tri)
    stats["triangles"] = len(tri)
    stats["vertices"] = len(v)
    return v, nrm, tri, stats
