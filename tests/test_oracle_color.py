"""Known answers of the colour-map restatement in the CPU oracle (oracle.depth_boundary_mask,
oracle.color_map): the upstream-recalled depth truncation and Sobel / dilation boundary mask, and
the k-nearest-neighbour fill against a brute-force search with the same (squared distance, vertex
index) order.  Parity against Open3D itself is unpinned (not installed); these pin the rules."""
import numpy as np

import oracle


def test_boundary_mask_on_a_depth_step():
    t = np.full((40, 60), 1.0, np.float32)
    t[:, 30:] = 1.5
    t[0:4, 0:4] = np.inf
    t[20, 5] = 3.0
    d, m = oracle.depth_boundary_mask(t)
    # truncation: >= 3 m and misses become 0
    assert d[0, 0] == 0.0 and d[20, 5] == 0.0 and d[10, 10] == 1.0 and d[10, 40] == 1.5
    # |Sobel| = 4 * 0.5 > 0.1 on columns 29 and 30, dilated by 3 px: columns 26..33
    assert list(np.nonzero(m[10])[0]) == list(range(26, 34))
    assert m[0:8, 0:8].any() and m.dtype == np.uint8 and set(np.unique(m)) <= {0, 255}
    # a step below the threshold: |Sobel| = 4 * 0.02 = 0.08 <= 0.1
    t2 = np.full((20, 20), 1.0, np.float32)
    t2[:, 10:] = 1.02
    assert not oracle.depth_boundary_mask(t2)[1].any()


def test_knn_fill_equals_brute_force():
    rng = np.random.default_rng(1)
    V = (rng.random((3000, 3)) * 2).astype(np.float32)
    V[:1000, 2] = 1.0  # a plane in front of the camera: sampled
    V[:1000, :2] = (rng.random((1000, 2)) * 0.6 - 0.3).astype(np.float32)
    V[1500] = V[1600] = V[5]  # exact distance ties between sampled candidates
    H = W = 64
    K = np.array([[[40.0, 0, 32], [0, 40.0, 32], [0, 0, 1]]])
    T = np.eye(4)[None]
    t = np.full((1, H, W), 1.0, np.float32)
    im = rng.integers(0, 255, (1, H, W, 3)).astype(np.uint8)
    c, n = oracle.color_map(V, im, t, K, T)
    seen, unseen = np.nonzero(n > 0)[0], np.nonzero(n == 0)[0]
    assert len(seen) >= 900 and len(unseen) >= 1500
    P = V.astype(np.float64)
    for q in unseen[::5]:
        d2 = ((P[seen] - P[q]) ** 2).sum(1)
        o = np.lexsort((seen, d2))[:3]
        want = c[seen[o]].astype(np.float64).mean(0)
        assert np.abs(want - c[q]).max() <= 1e-6, q


def test_knn_fill_equals_brute_force_on_a_surface():
    """Surface-like points (a noisy sphere shell, many near-equal distances): the k-d tree's pruning
    planes must be the values recorded at build time."""
    rng = np.random.default_rng(7)
    n = 20000
    d = rng.normal(size=(n, 3))
    V = (d / np.linalg.norm(d, axis=1, keepdims=True) * 0.5 + np.array([0, 0, 2.0])).astype(np.float32)
    V = np.round(V / 0.002) * 0.002  # lattice-like coordinates: exact ties
    V = V.astype(np.float32)
    H = W = 96
    K = np.array([[[60.0, 0, 48], [0, 60.0, 48], [0, 0, 1]]])
    T = np.eye(4)[None]
    t = np.full((1, H, W), np.inf, np.float32)
    front = V[:, 2] < 2.0
    u = np.round(V[front, 0] * 60 / V[front, 2] + 48).astype(int)
    v = np.round(V[front, 1] * 60 / V[front, 2] + 48).astype(int)
    t[0, v.clip(0, H - 1), u.clip(0, W - 1)] = V[front, 2]
    im = rng.integers(0, 255, (1, H, W, 3)).astype(np.uint8)
    c, cnt = oracle.color_map(V, im, t, K, T, disc_thr=1e9)
    seen, unseen = np.nonzero(cnt > 0)[0], np.nonzero(cnt == 0)[0]
    assert len(seen) > 200 and len(unseen) > 1000
    P = V.astype(np.float64)
    for q in unseen[::37]:
        d2 = ((P[seen] - P[q]) ** 2).sum(1)
        o = np.lexsort((seen, d2))[:3]
        want = c[seen[o]].astype(np.float64).mean(0)
        assert np.abs(want - c[q]).max() <= 1e-6, q
