"""Exhaustive check that the device's division shortcut is bit-identical to IEEE float division,
and that the R-specialised integrate kernel equals the generic one bit for bit."""
import ctypes
import os

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


# MQR_AB_TEST=1 (tests/test_gpu_ab_variants.py, with MQR_HIP_LIB = tools/_ab/libmqr_ab.so): the integrate
# tests below also cover the A/B kernels the shipped library leaves out (variants 3 and 5, bit 0x8000)
AB = os.environ.get("MQR_AB_TEST") == "1"
# 0x10000: one pixel per touch thread, 0x40000: no speculative first-batch integrate, 0x100000: 64-frame
# batches, 0x200000 / 0x400000 / 0x800000: a first batch of 64 / 32 / 16 frames, 0x4000000: the default
# kernel without its LDS weight table (k_integrate_win)
INTEGRATE_VARIANTS = {16: (0, 2, 4, 0x100, 0x104, 0x200, 0x400, 0x800, 0x10000, 0x40000, 0x100000, 0x200000,
                           0x400000, 0x800000, 0x4000000, 0x8000000),
                      8: (0, 2, 0x100)}
if AB:
    INTEGRATE_VARIANTS = {16: (0, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                               26, 27, 28, 29, 30, 31, 36, 37, 38, 39, 40, 41, 44, 45, 46, 47, 48, 49, 50, 64, 0x4000000, 0x105, 0x605, 0x106, 0x108, 0x10b, 0x10d, 0x111, 0x8000, 0x8003, 0x8008, 0x800a, 0x800b, 0x800d, 0x8011), 8: (0, 0x8000)}


def test_specialised_integrate_equals_generic():
    """Every integrate-kernel variant (lean default, LDS block-tiled, exact R-specialised; pipelined or
    serial touch, longest-first or touch order, 64- or 32-frame batches) equals the generic kernel
    (variant 1) bit for bit."""
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
        bad = []
        for variant in variants:  # every variant checked, the failures reported together
            try:
                compare_volumes(out[1], out[variant], 0.0)
            except AssertionError as e:
                bad.append((R, hex(variant), str(e)[:120]))
        assert not bad, bad


def test_special_depth_values_equal_generic():
    """Depth frames holding NaN (both signs), +-inf, -0.0, negative depths, values at and just past
    depth_max and denormals, seen by a camera whose principal point is -0.0 in one frame: every
    integrate variant equals the generic kernel bit for bit, and the generic kernel equals the oracle
    (Open3D's strict `d > 0`, `d <= depth_max` tests: a NaN depth passes both and updates with
    sdf clamped to the truncation, as the oracle restates it)."""
    import sys
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    seq = synthetic.make_sequence("room", n=8, height=240, width=320, f=262.5, noise=True, seed=77)
    rng = np.random.default_rng(77)
    specials = np.array([np.nan, -np.nan, np.inf, -np.inf, -0.0, 0.0, -1.0, 4.0, np.nextafter(np.float32(4.0), np.float32(5)),
                         1e-40, np.float32(-1e-40)], np.float32)
    depths = []
    for d in seq["depth"]:
        d = np.array(d, np.float32)
        m = rng.random(d.shape) < 0.05
        d[m] = specials[rng.integers(0, len(specials), int(m.sum()))]
        depths.append(d)
    K = np.array(seq["K"], np.float64)
    K[2, 0, 2] = -0.0
    K[2, 1, 2] = -0.0
    args = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    ref = oracle.OracleVBG(0.01, 16, 64)
    for i in range(len(depths)):
        ref.integrate_frame(depths[i], K[i], seq["T_wc"][i], 1.0, 4.0, 10.0)
    for R, variants in INTEGRATE_VARIANTS.items():
        out = {}
        for variant in (1,) + variants:
            v = VoxelBlockGrid(voxel_size=0.01, block_resolution=R, block_count=64)
            _lib.call("mqr_vbg_set_variant", v.handle, variant)
            v.integrate_frames(depths, K, seq["T_wc"], **args)
            out[variant] = v.export()
        if R == 16:
            compare_volumes(ref.export(), out[1], 0.0)
        bad = []
        for variant in variants:
            try:
                compare_volumes(out[1], out[variant], 0.0)
            except AssertionError as e:
                bad.append((R, hex(variant), str(e)[:120]))
        assert not bad, bad


def test_window_reads_fallback_frames():
    """The default kernel reads 8-byte depth windows only from frame stacks with an even pixel count
    and an 8-byte aligned base; odd-sized frames and a device stack starting 4 bytes into its
    allocation take the dword-gather kernel (variant 4).  Every case equals the generic kernel."""
    import ctypes
    import torch
    from gpu_helpers import compare_volumes
    from mqr import synthetic
    from mqr import _lib
    from mqr.vbg import VoxelBlockGrid
    args = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)

    def run(variant, depths, K, T):
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(depths, K, T, **args)
        return v.export()

    odd = synthetic.make_sequence("room", n=10, height=241, width=321, f=262.5, noise=True, seed=44)
    ref = run(1, odd["depth"], odd["K"], odd["T_wc"])
    for variant in (0, 4):
        compare_volumes(ref, run(variant, odd["depth"], odd["K"], odd["T_wc"]), 0.0)
    even = synthetic.make_sequence("room", n=10, height=240, width=320, f=262.5, noise=True, seed=45)
    d = np.ascontiguousarray(np.stack(even["depth"]), np.float32)
    B, H, W = d.shape
    flat = torch.zeros(B * H * W + 1, dtype=torch.float32, device="cuda:0")
    flat[1:] = torch.from_numpy(d.reshape(-1)).to("cuda:0")
    torch.cuda.synchronize()

    class Shifted:  # the stack 4 bytes into the allocation
        ptr = ctypes.c_void_p(flat.data_ptr() + 4)

    ref = run(1, even["depth"], even["K"], even["T_wc"])
    for variant in (0, 4):
        compare_volumes(ref, run(variant, (Shifted, B, H, W), even["K"], even["T_wc"]), 0.0)
        compare_volumes(ref, run(variant, even["depth"], even["K"], even["T_wc"]), 0.0)


def test_table_full_retry_equals_default():
    """The batch touch probes a bounded number of table slots per new key; a batch that fills the
    table is undone and touched again on a table grown to the worst case.  Variant bit 0x1000 probes
    one slot, so nearly every fresh volume takes that path -- on an empty volume and on one that
    already holds blocks (the undo must keep those): results equal the default path bit for bit."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=20, height=240, width=320, f=262.5, noise=True, seed=33)
    args = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    ref = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
    ref.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], **args)
    ref_out = ref.export()
    a = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
    _lib.call("mqr_vbg_set_variant", a.handle, 0x1000)
    a.stats(reset=True)
    a.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], **args)
    assert a.stats()["table_retries"] >= 1
    assert compare_volumes(ref_out, a.export(), 0.0) == 0.0
    b = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
    b.integrate_frames(seq["depth"][:10], seq["K"][:10], seq["T_wc"][:10], **args)
    _lib.call("mqr_vbg_set_variant", b.handle, 0x1000)
    b.stats(reset=True)
    b.integrate_frames(seq["depth"][10:], seq["K"][10:], seq["T_wc"][10:], **args)
    assert b.stats()["table_retries"] >= 1
    assert compare_volumes(ref_out, b.export(), 0.0) == 0.0


def test_fast_integrate_exact_fallback():
    """Depth in millimetres (depth_scale 1000: the exact kernel runs alone) with tiny non-zero
    depths, and weights near 2^61 from an imported volume: every variant equals the generic kernel."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=8, height=240, width=320, f=262.5, noise=True, seed=5)
    depth_mm = [np.asarray(d, np.float32) * 1000.0 for d in seq["depth"]]
    for d in depth_mm:
        d[::7, ::5] = np.float32(1e-30)   # in-image, > 0, below 2^-60: exact division path
    out = []
    cases = ((16, 1), (16, 0), (16, 2), (16, 6 if AB else 0x100), (8, 1), (8, 0), (8, 2))
    for R, variant in cases:
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
    for i in (1, 2, 3):
        assert compare_volumes(out[0], out[i], 0.0) == 0.0, cases[i]
    for i in (5, 6):
        assert compare_volumes(out[4], out[i], 0.0) == 0.0, cases[i]


def test_division_core_on_positive_zero():
    """The branch-free update divides s = +0 (d == zc) through the core sequence: must give +0."""
    for b in (0.05, 1.0, 3.0):
        mm, _ = _check(2, b, 0.0, 2.0 ** -149)  # bit pattern 0 only
        assert mm == 0


def test_lean_integrate_exact_fallback():
    """Fast kernels (lean default, block-tiled): the block holding zc == 0 voxels (camera at the origin
    looking at a 1 cm plane: the tiled kernel's corner test sends that frame to direct gathers, whose
    zc check hands the block off) and blocks with imported weights of 2^61 or non-integer weights go
    to the exact fix-up launch; every volume equals the generic kernel's bit for bit."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=6, height=240, width=320, f=262.5, noise=True, seed=9)
    near = np.full((240, 320), 0.01, np.float32)
    depths = [near] + [np.asarray(d, np.float32) for d in seq["depth"]]
    Ks = np.concatenate([seq["K"][:1], seq["K"]])
    Ts = np.concatenate([np.eye(4)[None], seq["T_wc"]])
    # (the default redoes such blocks in-kernel; variant 4 and, in the A/B library, 15 hand them to the
    # fix-up launch)
    cases = ((16, 1), (16, 0), (16, 5 if AB else 0x200), (16, 2), (16, 0x100), (16, 9 if AB else 0x400),
             (16, 8 if AB else 0x800), (16, 13 if AB else 0x100), (16, 17 if AB else 0x200), (16, 15 if AB else 4),
             (8, 1), (8, 0), (8, 2))
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
    for i in range(1, 10):
        assert compare_volumes(out[0], out[i], 0.0) == 0.0, cases[i]
    for i in (11, 12):
        assert compare_volumes(out[10], out[i], 0.0) == 0.0, cases[i]


@pytest.mark.parametrize("mode,a_max,b_lo,b_hi", [
    (0, 2.0e3 * 700.0, 1e-3, 8.0),        # (X fx) / Z: pixel-scale numerators, depths up to 8 m
    (0, 1.0e12, 2.0 ** -480, 2.0 ** 60),  # the guarded range edges
    (1, 4.0e3, 50.0, 2000.0),             # ((u - cx) z) / fx: focal lengths of real and synthetic cameras
    (1, 1.0e9, 1e-3, 1e6),
])
def test_confidence_float64_quotients_match_ieee(mode, a_max, b_lo, b_hi):
    """The confidence kernel's float64 quotients (shared refined reciprocal; host-rounded reciprocal
    with a Markstein correction) equal IEEE division on 2^31 hashed operand pairs per case."""
    import ctypes
    from mqr import _lib
    mm = ctypes.c_uint64()
    bad = np.zeros(2, np.float64)
    _lib.call("mqr_check_div64", 0, mode, 12345 + mode, 1 << 31, a_max, b_lo, b_hi, ctypes.byref(mm),
              _lib.ptr(bad, _lib._f64p))
    assert mm.value == 0, f"{mm.value} mismatches, e.g. a={bad[0]!r} b={bad[1]!r}"


def test_weight_table_across_calls_and_unknown_bounds():
    """The default kernel's LDS table of (w, 1 / (w + 1)) is sized per batch from the weights before the call
    plus the frames up to the batch's end.  Weights carried over several calls (one of them two batches long,
    the second batch starting at the previous batches' bound), a volume whose weights are unknown after an
    import (no bound: k_integrate_win runs) and the table-less kernel (bit 26) all equal the generic kernel."""
    from gpu_helpers import compare_volumes
    from mqr import _lib, synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=70, height=120, width=160, f=131.25, noise=True, seed=23)
    d, K, T = seq["depth"], seq["K"], seq["T_wc"]
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    calls = [(slice(0, 20),), (slice(10, 30),), (slice(0, 70), slice(0, 70))]  # the last: 140 frames, two batches
    out = {}
    for variant in (1, 0, 0x4000000, 0x8000000):
        v = VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        for parts in calls:
            dd = np.concatenate([d[p] for p in parts])
            v.integrate_frames(dd, np.concatenate([K[p] for p in parts]), np.concatenate([T[p] for p in parts]), **kw)
        out[variant] = v.export()
        # then through an import (weight bound unknown) and two more calls
        w = VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
        _lib.call("mqr_vbg_set_variant", w.handle, variant)
        w.import_blocks(*out[variant])
        for _ in range(2):
            w.integrate_frames(d[:40], K[:40], T[:40], **kw)
        out[(variant, "imported")] = w.export()
    assert float(out[1][2].max()) > 30  # weights carried past the first two calls' frame counts
    for variant in (0, 0x4000000, 0x8000000):
        compare_volumes(out[1], out[variant], 0.0)
        compare_volumes(out[(1, "imported")], out[(variant, "imported")], 0.0)
