"""The CPU oracle vs golden vectors produced by running the reference's own numpy code."""
import os

import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "confidence_golden.npz"))


@pytest.mark.parametrize("name", ["sphere", "room"])
@pytest.mark.parametrize("tag,params", [("a", (3, 3.0, 0.05)), ("b", (10, 4.0, 0.08))])
def test_oracle_confidence_bit_exact(golden, name, tag, params):
    r, dmax, thr = params
    d = golden[f"{name}_depth"]
    for i in range(d.shape[0]):
        c, v = oracle.confidence(d, golden[f"{name}_K"], golden[f"{name}_T_cw"], golden[f"{name}_T_cw_inv"], i, r,
                                 dmax, thr)
        assert np.array_equal(v, golden[f"{name}_valid_{tag}"][i])
        assert np.array_equal(c, golden[f"{name}_conf_{tag}"][i])


@pytest.mark.parametrize("name", ["sphere", "room"])
def test_oracle_pixel_error_map_bit_exact(golden, name):
    d = golden[f"{name}_depth"]
    for (a, b), e in zip(golden[f"{name}_pairs"], golden[f"{name}_err"]):
        g = oracle.pixel_error_map(golden[f"{name}_K"], golden[f"{name}_T_cw"], golden[f"{name}_T_cw_inv"], a, d[a],
                                   b, d[b], 3.0)
        assert np.array_equal(np.isnan(g), np.isnan(e))
        assert np.array_equal(g[~np.isnan(e)], e[~np.isnan(e)])


def test_oracle_confidence_skips_failed_frames(golden):
    """A neighbour whose load failed contributes nothing (estimate_depth_confidences.py:53-54):
    counts equal the sum of the per-pair error maps over the remaining window frames."""
    d = golden["sphere_depth"]
    K, Tc, Ti = golden["sphere_K"], golden["sphere_T_cw"], golden["sphere_T_cw_inv"]
    fv = np.ones(len(d), np.uint8)
    fv[3] = 0
    c, v = oracle.confidence(d, K, Tc, Ti, 4, 2, 3.0, 0.05, frame_valid=fv)
    valid = np.zeros(d.shape[1:], np.int32)
    cons = np.zeros(d.shape[1:], np.int32)
    for t in (2, 5, 6):
        e = oracle.pixel_error_map(K, Tc, Ti, 4, d[4], t, d[t], 3.0)
        valid += ~np.isnan(e)
        cons += (~np.isnan(e)) & (e <= np.float32(0.05))
    assert np.array_equal(v, valid)
    with np.errstate(invalid="ignore", divide="ignore"):
        want = np.where(valid == 0, 0.0, cons / np.maximum(valid, 1))
    assert np.array_equal(c, want)


@pytest.mark.parametrize("tag,params", [("a", (3, 3.0, 0.05)), ("b", (10, 4.0, 0.08))])
def test_zero_canvas_reproduces_reference_on_mixed_frame_sizes(tmp_path, golden_dir, tag, params):
    """The confidence driver stacks a window of differently sized frames on a zero canvas
    (mqr.confidence._canvas_stack).  The oracle run on that canvas, cropped to the reference frame,
    equals the reference's own build_confidence_map on the ragged capture bit for bit
    (confidence_ragged_golden.npz; the reference interpolates each neighbour within its own h, w)."""
    from test_gpu_confidence_driver import _ragged_capture
    from mqr.confidence import _canvas_stack
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    g = np.load(os.path.join(golden_dir, "confidence_ragged_golden.npz"))
    r, dmax, thr = params
    _ragged_capture(tmp_path, g)
    io = DepthDataIO(tmp_path)
    ds = io.build_depth_dataset(Side.LEFT)
    n = int(g["n"])
    frames = [io.load_depth_map_by_index(Side.LEFT, ds, i) for i in range(n)]
    for i in range(n):
        lo, hi = max(0, i - r), min(n, i + r + 1)
        canvas = _canvas_stack(frames[lo:hi])
        c, v = oracle.confidence(canvas, g["K"][lo:hi], g["T_cw"][lo:hi], g["T_cw_inv"][lo:hi], i - lo, r, dmax, thr)
        h, w = frames[i].shape
        assert np.array_equal(v[:h, :w], g[f"valid_{tag}_{i}"]), i
        assert np.array_equal(c[:h, :w], g[f"conf_{tag}_{i}"]), i
