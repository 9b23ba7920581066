"""Known-answer tests for the filter_mesh_components restatement (oracle/meshfilter_ref.py),
hand-derived from the Open3D legacy algorithms the reference calls (o3d_utils.py:241-321)."""
import numpy as np

import meshfilter_ref as mf

V = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [2, 1, 0], [2, 2, 0], [1, 2, 0],
              [5, 5, 5], [6, 5, 5], [5, 6, 5], [0, 0, 0]], np.float32)
T = np.array([[0, 1, 2], [0, 2, 3], [2, 4, 5], [2, 5, 6], [7, 8, 9], [0, 2, 3], [1, 2, 0], [10, 1, 2]], np.int32)


def test_clusters_are_edge_connected_in_triangle_order():
    c, n = mf.cluster_connected_triangles(T)
    # squares sharing only vertex 2 are separate clusters; duplicates join through their edges
    assert c.tolist() == [0, 0, 1, 1, 2, 0, 0, 0]
    assert n.tolist() == [5, 2, 1]


def test_filter_known_answer():
    v, n, t, st = mf.filter_mesh_components(V, None, T, 2)
    # tri 4 dropped (cluster of 1) -> vertices 7-9 unreferenced and removed, 10 -> 7;
    # duplicates [0,2,3] and [1,2,0] (rotation of [0,1,2]) dropped; vertex 7 == vertex 0 merged,
    # making edge (0,2) carry 3 triangles of equal area -> the first one is dropped
    assert t.tolist() == [[0, 2, 3], [2, 4, 5], [2, 5, 6], [0, 1, 2]]
    assert len(v) == 7 and np.array_equal(v, V[:7])
    assert st["clusters"] == 3 and st["kept_clusters"] == 2 and st["small_cluster_triangles"] == 1
    assert st["non_manifold_removed"] == 1


def test_largest_kept_when_none_qualifies():
    v, n, t, st = mf.filter_mesh_components(V, None, T, 100)
    assert st["kept_clusters"] == 1 and st["largest_cluster"] == 5
    assert len(t) == 2  # cluster 0 after duplicate and non-manifold clean-up


def test_zero_area_and_signed_zero():
    v = np.array([[0, 0, 0], [1, 0, 0], [2, 0, 0], [0, 1, 0], [-0.0, 0, 0]], np.float32)
    t = np.array([[0, 1, 2], [0, 1, 3], [4, 3, 1]], np.int32)  # collinear, normal, same as #2 via -0
    v2, _, t2, st = mf.filter_mesh_components(v, None, t, 1)
    assert t2.tolist() == [[0, 1, 3], [0, 3, 1]]   # zero-area dropped, -0 merged into +0 (duplicate
    assert len(v2) == 4                            # triangles are checked before the vertex merge)
