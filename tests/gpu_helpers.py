"""Comparison helpers shared by the parity tests and bench.py's parity legs (order-independent
volume / mesh / point comparison).  Test infrastructure: the product never imports this.

Two mesh comparisons, both independent of vertex numbering and triangle order:

* ``compare_meshes`` (small meshes): sorted vertex positions and canonically rotated triangles as
  position triples, compared exactly.
* ``mesh_signature`` / ``compare_meshes_fast`` (config-size meshes, tens of millions of
  triangles): every vertex position -> a 64-bit hash of its float bit patterns; every triangle ->
  the minimum over its three cyclic rotations of a non-commutative hash of its vertices' hashes
  (orientation kept, rotation-invariant, coincident vertices compare equal); the two sorted hash
  arrays are compared exactly.  Equal arrays mean equal multisets of vertex positions and oriented
  triangles up to 64-bit hash collisions.
"""
import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(x):
    """splitmix64 finaliser on a uint64 array (wrapping arithmetic)."""
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        return x ^ (x >> np.uint64(31))


def canon_blocks(keys, tsdf, weight):
    o = np.lexsort(keys.T[::-1])
    return keys[o], tsdf[o], weight[o]


def _key_order(keys):
    k = keys.astype(np.int64) + (1 << 20)
    return np.argsort((k[:, 0] << 42) | (k[:, 1] << 21) | k[:, 2], kind="stable")


def compare_volumes(a, b, tol=1e-4, chunk=4096):
    """a, b: (keys, tsdf, weight).  Returns max |dtsdf| over w>0; asserts identical keys/weights.
    Blocks are matched by key and compared chunk by chunk (no full reordered copies)."""
    ka, ta, wa = a
    kb, tb, wb = b
    assert ka.shape == kb.shape, (ka.shape, kb.shape)
    oa, ob = _key_order(ka), _key_order(kb)
    assert np.array_equal(ka[oa], kb[ob]), "block key sets differ"
    err = 0.0
    for s in range(0, len(oa), chunk):
        ia, ib = oa[s:s + chunk], ob[s:s + chunk]
        wa_, wb_ = wa[ia], wb[ib]
        if not np.array_equal(wa_, wb_):
            raise AssertionError(f"weights differ at {int((wa_ != wb_).sum())} voxels (chunk at block {s})")
        m = wa_ > 0
        if m.any():
            err = max(err, float(np.abs(ta[ia][m] - tb[ib][m]).max()))
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


def position_hashes(p):
    """64-bit hash of each row of float32 positions (N,3) from its bit patterns."""
    b = np.ascontiguousarray(p, dtype=np.float32).view(np.uint32).astype(np.uint64)
    with np.errstate(over="ignore"):
        return _mix(_mix(_mix(b[:, 0]) ^ b[:, 1]) + b[:, 2])


def mesh_signature(v, tri):
    """(sorted vertex-position hashes, sorted triangle hashes); see the module docstring."""
    hv = position_hashes(v)
    tri = np.asarray(tri)
    if len(tri):
        assert tri.min() >= 0 and tri.max() < len(v), "triangle index out of range"
    h = hv[tri] if len(tri) else np.zeros((0, 3), np.uint64)
    with np.errstate(over="ignore"):
        rots = [_mix(_mix(_mix(h[:, r]) + h[:, (r + 1) % 3]) ^ h[:, (r + 2) % 3]) for r in range(3)]
    ht = np.minimum(np.minimum(rots[0], rots[1]), rots[2])
    hv.sort()
    ht.sort()
    return hv, ht


def compare_meshes_fast(gv, gt, ov, ot):
    """Exact multiset comparison of vertex positions and oriented triangles via mesh_signature."""
    assert gv.shape == ov.shape, (gv.shape, ov.shape)
    assert gt.shape == ot.shape, (gt.shape, ot.shape)
    ga, gb = mesh_signature(gv, gt)
    oa, ob = mesh_signature(ov, ot)
    assert np.array_equal(ga, oa), "vertex position multisets differ"
    assert np.array_equal(gb, ob), "triangle multisets differ"
    return True


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


def compare_points_fast(gp, gn, op, on, tol=1e-6):
    """Config-size point clouds: positions compared as exact multisets (sorted hashes); normals
    matched through the position order (points at one position are a multiset too: their normals
    are compared after sorting within equal positions) within tol."""
    assert gp.shape == op.shape, (gp.shape, op.shape)
    hg, ho = position_hashes(gp), position_hashes(op)
    og = np.lexsort((gn[:, 2], gn[:, 1], gn[:, 0], hg))
    oo = np.lexsort((on[:, 2], on[:, 1], on[:, 0], ho))
    assert np.array_equal(hg[og], ho[oo]), "point position multisets differ"
    assert np.array_equal(gp[og], op[oo]), "point positions differ"
    err = float(np.abs(gn[og] - on[oo]).max()) if len(gp) else 0.0
    assert err <= tol, f"normals differ by {err}"
    return err
