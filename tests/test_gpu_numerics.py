"""Exhaustive check that the device's division shortcut is bit-identical to IEEE float division,
and that the R-specialised integrate kernel equals the generic one bit for bit."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return int(np.array([x], np.float32).view(np.uint32)[0])


def _check(which, b, lo, hi):
    from mqr import _lib
    mm, first = ctypes.c_uint32(), ctypes.c_uint32()
    _lib.call("mqr_check_division", 0, which, float(b), _bits(lo), _bits(hi) - _bits(lo), ctypes.byref(mm),
              ctypes.byref(first))
    return mm.value, first.value


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_reciprocal_shortcut_exact_over_all_floats(sign):
    lo, hi = (2.0 ** -80, 2.0 ** 80) if sign > 0 else (-(2.0 ** -80), -(2.0 ** 80))
    mm, first = _check(0, 0.0, lo, hi)
    assert mm == 0, f"{mm} mismatches, first bit pattern {first:#x}"


@pytest.mark.parametrize("b", [0.05, 0.04, 0.1, 0.08, 0.02, 0.16, 0.0375, 1.0, 1000.0, 3.3333333])
def test_division_shortcut_exact(b):
    b = float(np.float32(0.005) * np.float32(10.0)) if b == 0.05 else b
    for lo, hi in ((2.0 ** -45, 2.0 ** 12), (-(2.0 ** -45), -(2.0 ** 12))):
        mm, first = _check(1, b, lo, hi)
        assert mm == 0, f"b={b}: {mm} mismatches, first bit pattern {first:#x}"


def test_specialised_integrate_equals_generic():
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=20, height=240, width=320, f=262.5, noise=True, seed=21)
    out = []
    for R, variant in ((16, 0), (16, 1), (8, 0), (8, 1), (16, 2), (16, 0x100), (8, 0x101)):
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=R, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                           trunc_voxel_multiplier=10.0)
        out.append(v.export())
    assert compare_volumes(out[0], out[1], 0.0) == 0.0
    assert compare_volumes(out[2], out[3], 0.0) == 0.0
    assert compare_volumes(out[0], out[4], 0.0) == 0.0
    assert compare_volumes(out[0], out[5], 0.0) == 0.0
    assert compare_volumes(out[2], out[6], 0.0) == 0.0


def test_division_core_on_positive_zero():
    """The branch-free update divides s = +0 (d == zc) through the core sequence: must give +0."""
    for b in (0.05, 1.0, 3.0):
        mm, _ = _check(2, b, 0.0, 2.0 ** -149)  # bit pattern 0 only
        assert mm == 0
