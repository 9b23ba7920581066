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


@pytest.mark.parametrize("which,lo,hi", [(3, 2.0 ** -60, 2.0 ** 60), (4, 1.0, 2.0 ** 24), (4, 2.0 ** -60, 2.0 ** 60)])
def test_shortened_reciprocals_exact(which, lo, hi):
    """Lean integrate kernel: rcp_nm (v_rcp + Newton + Markstein; 1 / zc) and rcp_m (v_rcp +
    Markstein; 1 / (w + 1), and 1 / zc in the RZ = 2 variants) equal IEEE 1.0f / b on every float
    of the range they are used on."""
    mm, first = _check(which, 0.0, lo, hi)
    assert mm == 0, f"mode {which}: {mm} mismatches, first bit pattern {first:#x}"


INTEGRATE_VARIANTS = {16: (0, 2, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 22, 23, 24, 25, 0x100, 0x106,
                          0x108, 26, 27, 28, 29, 0x200, 0x300, 30, 31, 32, 33, 0x21e, 34, 35, 36, 37,
                          40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 56, 57, 58, 59, 0x128, 0x228, 0x130, 0x400, 0x436, 0x500),
                      8: (0, 6, 8, 0x101, 0x200, 40, 48)}


def test_specialised_integrate_equals_generic():
    """Every integrate-kernel variant (R-specialised, packed f32, 256/512/1024 threads, fast
    division with exact re-run, serial or pipelined) equals the generic kernel (variant 1) bit for bit."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=20, height=240, width=320, f=262.5, noise=True, seed=21)
    for R, variants in INTEGRATE_VARIANTS.items():
        out = {}
        for variant in (1,) + variants:
            v = VoxelBlockGrid(voxel_size=0.01, block_resolution=R, block_count=64)
            _lib.call("mqr_vbg_set_variant", v.handle, variant)
            v.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                               trunc_voxel_multiplier=10.0)
            out[variant] = v.export()
        for variant in variants:
            assert compare_volumes(out[1], out[variant], 0.0) == 0.0, (R, variant)


def test_fast_integrate_exact_fallback():
    """Operands outside the division core's exact range (a tiny non-zero depth read in millimetres,
    weights near 2^61 from an imported volume) make the fast kernel redo the block exactly."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=8, height=240, width=320, f=262.5, noise=True, seed=5)
    depth_mm = [np.asarray(d, np.float32) * 1000.0 for d in seq["depth"]]
    for d in depth_mm:
        d[::7, ::5] = np.float32(1e-30)   # in-image, > 0, below 2^-60 -> fallback
    out = []
    # 34 / 37: fast kernel handing out-of-range blocks to the exact fix-up launch
    for R, variant in ((16, 1), (16, 0), (16, 6), (16, 7), (16, 18), (16, 34), (16, 37), (8, 1), (8, 6), (16, 54)):
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=R, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(depth_mm[:4], seq["K"][:4], seq["T_wc"][:4], depth_scale=1000.0, depth_max=4.0,
                           trunc_voxel_multiplier=10.0)
        keys, tsdf, wgt = v.export()
        wgt = wgt.copy()
        wgt[keys.sum(axis=1) % 3 == 0] = np.float32(2.0 ** 61)   # w + 1 out of range (key-chosen blocks)
        v.reset()
        v.import_blocks(keys, tsdf, wgt)
        v.integrate_frames(depth_mm[4:], seq["K"][4:], seq["T_wc"][4:], depth_scale=1000.0, depth_max=4.0,
                           trunc_voxel_multiplier=10.0)
        out.append(v.export())
    for i in (1, 2, 3, 4, 5, 6, 9):
        assert compare_volumes(out[0], out[i], 0.0) == 0.0
    assert compare_volumes(out[7], out[8], 0.0) == 0.0


def test_division_core_on_positive_zero():
    """The branch-free update divides s = +0 (d == zc) through the core sequence: must give +0."""
    for b in (0.05, 1.0, 3.0):
        mm, _ = _check(2, b, 0.0, 2.0 ** -149)  # bit pattern 0 only
        assert mm == 0


def test_packed_integrate_exact_fallback():
    """Packed kernel (variants 8/9): a camera at the origin looking at a 1 cm plane touches the block
    holding voxels with zc == 0 (block re-run), imported weights of 2^61 force the exact pass."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=6, height=240, width=320, f=262.5, noise=True, seed=9)
    near = np.full((240, 320), 0.01, np.float32)
    depths = [near] + [np.asarray(d, np.float32) for d in seq["depth"]]
    Ks = np.concatenate([seq["K"][:1], seq["K"]])
    Ts = np.concatenate([np.eye(4)[None], seq["T_wc"]])
    out = []
    for R, variant in ((16, 1), (16, 8), (16, 9), (16, 14), (16, 15), (8, 1), (8, 8)):
        v = VoxelBlockGrid(voxel_size=0.005, block_resolution=R, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(depths[:4], Ks[:4], Ts[:4], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        keys, tsdf, wgt = v.export()
        assert (keys == 0).all(axis=1).any(), "origin block not touched"
        wgt = wgt.copy()
        wgt[keys.sum(axis=1) % 3 == 1] = np.float32(2.0 ** 61)
        v.reset()
        v.import_blocks(keys, tsdf, wgt)
        v.integrate_frames(depths[3:], Ks[3:], Ts[3:], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        out.append(v.export())
    for i in (1, 2, 3, 4):
        assert compare_volumes(out[0], out[i], 0.0) == 0.0
    assert compare_volumes(out[5], out[6], 0.0) == 0.0


def test_lean_integrate_exact_fallback():
    """Lean kernel (variants 40-53, column and cube lane mappings): the block holding zc == 0 voxels (camera at the origin looking at
    a 1 cm plane) and blocks with imported weights of 2^61 or non-integer weights are handed to the
    exact fix-up launch; every volume equals the generic kernel's bit for bit."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=6, height=240, width=320, f=262.5, noise=True, seed=9)
    near = np.full((240, 320), 0.01, np.float32)
    depths = [near] + [np.asarray(d, np.float32) for d in seq["depth"]]
    Ks = np.concatenate([seq["K"][:1], seq["K"]])
    Ts = np.concatenate([np.eye(4)[None], seq["T_wc"]])
    cases = ((16, 1), (16, 40), (16, 41), (16, 42), (16, 43), (16, 44), (16, 45), (16, 46), (16, 47), (16, 48),
             (16, 49), (16, 50), (16, 51), (16, 52), (16, 53), (16, 56), (16, 57), (16, 58), (8, 1), (8, 40), (8, 48))
    out = []
    for R, variant in cases:
        v = VoxelBlockGrid(voxel_size=0.005, block_resolution=R, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(depths[:4], Ks[:4], Ts[:4], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        keys, tsdf, wgt = v.export()
        assert (keys == 0).all(axis=1).any(), "origin block not touched"
        wgt = wgt.copy()
        sel = keys.sum(axis=1) % 3
        wgt[sel == 1] = np.float32(2.0 ** 61)
        wgt[sel == 2] *= np.float32(1.5)  # odd counts become non-integer
        v.reset()
        v.import_blocks(keys, tsdf, wgt)
        v.integrate_frames(depths[3:], Ks[3:], Ts[3:], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        out.append(v.export())
    for i in range(1, 18):
        assert compare_volumes(out[0], out[i], 0.0) == 0.0, cases[i]
    assert compare_volumes(out[18], out[19], 0.0) == 0.0
    assert compare_volumes(out[18], out[20], 0.0) == 0.0
