"""GPU parity of the confidence estimator against golden vectors produced by the reference itself."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden(golden_dir):
    import os
    from mqr import _lib
    _lib.load()
    return np.load(os.path.join(golden_dir, "confidence_golden.npz"))


@pytest.mark.parametrize("name", ["sphere", "room"])
@pytest.mark.parametrize("tag,params", [("a", (3, 3.0, 0.05)), ("b", (10, 4.0, 0.08))])
def test_confidence_matches_reference_golden(golden, name, tag, params):
    from mqr.confidence import confidence_maps
    r, dmax, thr = params
    d = golden[f"{name}_depth"]
    conf, valid = confidence_maps(d, golden[f"{name}_K"], golden[f"{name}_T_cw"], golden[f"{name}_T_cw_inv"], 0,
                                  d.shape[0], r, dmax, thr)
    assert np.array_equal(valid, golden[f"{name}_valid_{tag}"])
    assert np.array_equal(conf, golden[f"{name}_conf_{tag}"])


@pytest.mark.parametrize("name", ["sphere", "room"])
def test_pixel_error_map_matches_reference_golden(golden, name):
    from mqr.confidence import compute_pixel_error_map
    d = golden[f"{name}_depth"]
    for (a, b), e in zip(golden[f"{name}_pairs"], golden[f"{name}_err"]):
        g = compute_pixel_error_map(golden[f"{name}_K"], golden[f"{name}_T_cw"], golden[f"{name}_T_cw_inv"], a, d[a],
                                    b, d[b], depth_max=3.0)
        assert np.array_equal(np.isnan(g), np.isnan(e))
        m = ~np.isnan(e)
        assert np.array_equal(g[m], e[m])


def test_confidence_full_resolution_vs_oracle():
    """640x480 room frames, skipped neighbour frames, window clipping at both ends."""
    from mqr import synthetic
    from mqr.confidence import confidence_maps
    seq = synthetic.make_sequence("room", n=14, height=480, width=640, noise=True, seed=5)
    Ti = np.linalg.inv(seq["T_cw"])
    ok = np.ones(14, np.uint8)
    ok[4] = 0
    conf, valid = confidence_maps(seq["depth"], seq["K"], seq["T_cw"], Ti, 0, 14, 10, 4.0, 0.08, frame_ok=ok)
    for i in (0, 5, 13):
        oc, ov = oracle.confidence(seq["depth"], seq["K"], seq["T_cw"], Ti, i, 10, 4.0, 0.08, frame_valid=ok)
        assert np.array_equal(valid[i], ov)
        assert np.array_equal(conf[i], oc)
    assert valid.max() > 0


@pytest.mark.parametrize("thr,dmax", [(0.08, 4.0), (0.0, 4.0), (-1.0, 4.0), (np.inf, 4.0), (1e30, 4.0),
                                      (0.002, 4.0), (0.08, np.inf)])
def test_confidence_band_edges_vs_oracle(thr, dmax):
    """The consistency band (pixel_decide) against the oracle's full computation: thresholds at the
    extremes (nothing / everything consistent, +inf) and small enough that many pairs fall inside the
    band, unbounded depth_max, a non-rigid pose (large R^T R - I), a pose with a NaN entry, a NaN in
    T_cw with a finite separately supplied inverse (the error is NaN: not valid) and an inverse off by
    1 mm (large dT)."""
    from mqr import synthetic
    from mqr.confidence import confidence_maps
    n = 16  # reference frames 5..8 see only finite-band neighbours (the band path proper)
    seq = synthetic.make_sequence("room", n=n, height=120, width=160, f=131.25, noise=True, seed=11)
    T = seq["T_cw"].astype(np.float32).copy()
    T[1, :3, :3] *= np.float32(1.001)  # scaled rotation
    T[14, 0, 3] = np.nan
    Ti = np.linalg.inv(T.astype(np.float64)).astype(np.float32)
    Ti[8, 1, 3] += np.float32(1e-3)
    T[12, 2, 3] = np.nan  # after the inverse: T_cw non-finite, T_cw_inv finite
    conf, valid = confidence_maps(seq["depth"], seq["K"], T, Ti, 0, n, 3, dmax, thr)
    for i in range(n):
        oc, ov = oracle.confidence(seq["depth"], seq["K"], T, Ti, i, 3, dmax, thr)
        assert np.array_equal(valid[i], ov), i
        assert np.array_equal(conf[i], oc), i
    if thr == 0.08:
        assert valid.max() > 0 and 0 < conf.mean() < 1


def test_confidence_float32_prefilter_stages_and_static_camera():
    """The float32 prefilter (pixel_decide32) decides most pairs and defers the uncertain ones: the
    stage counts add up, the maps are identical with counting on or off, and a static camera (every
    neighbour's projection lands exactly on integer pixel coordinates: every floor() is uncertain in
    float32, so every pair must take the float64 path) still matches the oracle bit for bit."""
    import ctypes
    from mqr import _lib, synthetic
    from mqr.confidence import confidence_maps
    seq = synthetic.make_sequence("room", n=12, height=120, width=160, f=131.25, noise=True, seed=21)
    Ti = np.linalg.inv(seq["T_cw"])
    last = np.zeros(4, np.int64)
    base = confidence_maps(seq["depth"], seq["K"], seq["T_cw"], Ti, 0, 12, 10, 4.0, 0.08)
    _lib.call("mqr_confidence_stats", 0, 1, None)
    try:
        counted = confidence_maps(seq["depth"], seq["K"], seq["T_cw"], Ti, 0, 12, 10, 4.0, 0.08)
        _lib.call("mqr_confidence_stats", 0, -1, _lib.ptr(last, _lib._i64p))
    finally:
        _lib.call("mqr_confidence_stats", 0, 0, None)
    assert np.array_equal(base[0], counted[0]) and np.array_equal(base[1], counted[1])
    pairs, f32, f64, tail = (int(x) for x in last)
    assert pairs > 0 and f32 + f64 + tail == pairs and f64 >= 0
    assert f32 > 0.9 * pairs, last
    # static camera: all poses equal (noise differs per frame)
    T = np.repeat(seq["T_cw"][:1], 6, axis=0).astype(np.float32)
    Ts = np.linalg.inv(T.astype(np.float64)).astype(np.float32)
    d = seq["depth"][:6]
    conf, valid = confidence_maps(d, seq["K"][:6], T, Ts, 0, 6, 3, 4.0, 0.08)
    for i in range(6):
        oc, ov = oracle.confidence(d, seq["K"][:6], T, Ts, i, 3, 4.0, 0.08)
        assert np.array_equal(valid[i], ov), i
        assert np.array_equal(conf[i], oc), i
    assert valid.max() > 0


def test_confidence_wide_window_vs_oracle():
    """r > 31 (a window of more than 64 frames): the chunked float64-deferral path (k_confidence<WIDE>)
    over 70 small frames against the oracle, reference frames at both ends and in the middle."""
    from mqr import synthetic
    from mqr.confidence import confidence_maps
    seq = synthetic.make_sequence("room", n=70, height=48, width=64, f=52.5, noise=True, seed=23)
    Ti = np.linalg.inv(seq["T_cw"])
    conf, valid = confidence_maps(seq["depth"], seq["K"], seq["T_cw"], Ti, 0, 70, 40, 4.0, 0.08)
    for i in (0, 35, 69):
        oc, ov = oracle.confidence(seq["depth"], seq["K"], seq["T_cw"], Ti, i, 40, 4.0, 0.08)
        assert np.array_equal(valid[i], ov), i
        assert np.array_equal(conf[i], oc), i
    assert valid.max() > 0  # (ref frame 35 reads a 70-frame window: two 64-neighbour chunks)
