"""Comparison helpers shared by the parity tests (order-independent volume / mesh comparison)."""
import numpy as np


def canon_blocks(keys, tsdf, weight):
    o = np.lexsort(keys.T[::-1])
    return keys[o], tsdf[o], weight[o]


def compare_volumes(a, b, tol=1e-4):
    """a, b: (keys, tsdf, weight).  Returns max |dtsdf| over w>0; asserts identical keys/weights."""
    ka, ta, wa = canon_blocks(*a)
    kb, tb, wb = canon_blocks(*b)
    assert ka.shape == kb.shape, (ka.shape, kb.shape)
    assert np.array_equal(ka, kb), "block key sets differ"
    assert np.array_equal(wa, wb), f"weights differ at {int((wa != wb).sum())} voxels"
    m = wa > 0
    err = float(np.abs(ta[m] - tb[m]).max()) if m.any() else 0.0
    assert err <= tol, f"tsdf max |diff| {err} > {tol}"
    return err


def canon_vertices(v):
    o = np.lexsort(v.T[::-1])
    rank = np.empty(len(v), np.int64)
    rank[o] = np.arange(len(v))
    return v[o], rank


def canon_triangles(v, tri):
    """Triangles as vertex-position triples, rotated to start at the lexicographically smallest
    vertex (orientation kept), rows sorted.  Position-based, so coincident vertices (ratio 0 on two
    edges of one voxel) compare equal whichever of them a triangle references."""
    P = v[tri]  # (T,3,3)
    key = np.lexsort(P.transpose(2, 0, 1)[::-1].reshape(3, -1)).reshape(-1)
    rank = np.empty(len(key), np.int64)
    rank[key] = np.arange(len(key))
    rank = rank.reshape(P.shape[0], 3)
    r = np.argmin(rank, axis=1)
    idx = (np.arange(3)[None, :] + r[:, None]) % 3
    P = np.take_along_axis(P, idx[:, :, None], axis=1).reshape(len(P), 9)
    return P[np.lexsort(P.T[::-1])]


def compare_meshes(gv, gt, ov, ot, pos_tol=0.0):
    assert gv.shape == ov.shape, (gv.shape, ov.shape)
    assert gt.shape == ot.shape, (gt.shape, ot.shape)
    sgv, _ = canon_vertices(gv)
    sov, _ = canon_vertices(ov)
    dv = float(np.abs(sgv - sov).max()) if len(gv) else 0.0
    assert dv <= pos_tol, f"vertex positions differ by {dv}"
    if len(gt):
        assert gt.min() >= 0 and gt.max() < len(gv), "triangle index out of range"
        assert np.array_equal(canon_triangles(gv, gt), canon_triangles(ov, ot)), "triangle sets differ"
    return dv


def compare_points_normals(gp, gn, op, on, tol=1e-6):
    """Order-independent comparison of (position, normal) rows."""
    assert gp.shape == op.shape, (gp.shape, op.shape)
    a = np.concatenate([gp, gn], axis=1)
    b = np.concatenate([op, on], axis=1)
    a = a[np.lexsort(a.T[::-1])]
    b = b[np.lexsort(b.T[::-1])]
    assert np.array_equal(a[:, :3], b[:, :3]), "positions differ"
    err = float(np.abs(a[:, 3:] - b[:, 3:]).max()) if len(a) else 0.0
    assert err <= tol, f"normals differ by {err}"
    return err
