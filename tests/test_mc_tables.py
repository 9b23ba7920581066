"""Marching-cubes table consistency (the tables are shared data; see tools/mc_tables.py)."""
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import mc_tables as mc  # noqa: E402

FACES = [frozenset(i for i, s in enumerate(mc.VTX_SHIFTS) if s[a] == v) for a in range(3) for v in (0, 1)]


def _edge_faces(e):
    a, b = mc.EDGE_CORNERS[e]
    return [f for f in FACES if a in f and b in f]


def test_edge_table_is_sign_change_table():
    assert mc.EDGE_TABLE[:4] == [0x000, 0x109, 0x203, 0x30a]  # Bourke's first entries
    assert all(mc.EDGE_TABLE[c] == mc.EDGE_TABLE[255 - c] for c in range(256))


def test_edge_shifts_match_corners():
    for e, (a, b) in enumerate(mc.EDGE_CORNERS):
        sa, sb = np.array(mc.VTX_SHIFTS[a]), np.array(mc.VTX_SHIFTS[b])
        d = np.abs(sb - sa)
        assert d.sum() == 1
        axis = int(np.argmax(d))
        assert mc.EDGE_SHIFTS[e][3] == axis
        assert tuple(np.minimum(sa, sb)) == tuple(mc.EDGE_SHIFTS[e][:3])


def test_every_case_is_a_consistent_surface_patch():
    """Per case: the polygon uses exactly the crossing edges; every interior segment is shared by two
    triangles with opposite orientation; boundary segments lie on cube faces and pair up each face's
    crossing points."""
    for c in range(256):
        rows = mc.TRI_ROWS[c]
        want = {i for i in range(12) if mc.EDGE_TABLE[c] >> i & 1}
        assert set(rows) == want, c
        segs = Counter()
        for t in range(0, len(rows), 3):
            tri = rows[t:t + 3]
            for k in range(3):
                segs[(tri[k], tri[(k + 1) % 3])] += 1
        und = Counter()
        for (a, b), n in segs.items():
            und[frozenset((a, b))] += n
        for s, n in und.items():
            a, b = tuple(s)
            assert n in (1, 2), c
            if n == 2:
                assert segs[(a, b)] == 1 and segs[(b, a)] == 1, c
            else:
                assert set(_edge_faces(a)) & set(_edge_faces(b)), c
        for f in FACES:
            pts = [e for e in want if f in _edge_faces(e)]
            bsegs = [tuple(s) for s, n in und.items() if n == 1 and all(f in _edge_faces(x) for x in s)]
            cnt = Counter(x for s in bsegs for x in s)
            assert all(cnt[p] == 1 for p in pts) and 2 * len(bsegs) == len(pts), c


def test_tri_count_and_header_in_sync():
    assert mc.TRI_COUNT[0] == 0 and mc.TRI_COUNT[255] == 0 and max(mc.TRI_COUNT) == 5
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "mqr_mc_tables.h")).read()
    for r in mc.TRI_TABLE[:8]:
        assert "{" + ", ".join(str(v) for v in r) + "}" in hdr
