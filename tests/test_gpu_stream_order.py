"""Stream ordering at the C-ABI boundary (include/mqr.h "stream ordering", mqr_set_stream).

libmqr runs on its own non-blocking HIP streams.  A caller that hands it a device tensor torch has
just written on a side stream -- with no synchronize in between -- must get the result of the
written frames, never of the bytes that were there before.  Each test delays the side stream by a
spin kernel, enqueues the write behind it and calls the library at once (inside
``torch.cuda.stream(s)``, so the Python layer passes s as the caller stream); the outputs are
compared with the CPU oracle.  Without the ordering the library would read the frames ~50 ms before
they land (round 4's N>1 rehearsal abort, gpurun_out/r04a_bench2.err: "No block is touched")."""
import ctypes

import numpy as np
import pytest

import oracle  # the test-only checker (tests/conftest.py puts oracle/ on the path)

pytestmark = pytest.mark.gpu

_SPIN = 100_000_000  # spin-kernel cycles (~40-50 ms at the MI355X shader clock)


class _Dev:
    def __init__(self, t):
        self.ptr = ctypes.c_void_p(t.data_ptr())


def _late_copy(torch, host, s):
    """A device tensor whose contents land on stream `s` only after a spin kernel: poisoned first
    (NaN, which touches nothing), then the host frames copied in behind the spin."""
    dev = torch.full(host.shape, float("nan"), dtype=torch.float32, device="cuda")
    pinned = torch.from_numpy(host).pin_memory()
    torch.cuda.synchronize()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        torch.cuda._sleep(_SPIN)
        dev.copy_(pinned, non_blocking=True)
    dev.record_stream(s)
    return dev


def test_integrate_frames_after_side_stream_write():
    import torch
    from gpu_helpers import compare_volumes
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=24, height=240, width=320, f=262.5, noise=True, seed=7)
    B, H, W = seq["depth"].shape
    K, T = seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    s = torch.cuda.Stream()
    dev = _late_copy(torch, np.ascontiguousarray(seq["depth"], np.float32), s)
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
    with torch.cuda.stream(s):  # no synchronize: the library orders itself after s
        vbg.integrate_frames((_Dev(dev), B, H, W), K, T, depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    ref = oracle.OracleVBG(0.01, 16, 256)
    for i in range(B):
        ref.integrate_frame(seq["depth"][i], K[i], T[i], 1.0, 4.0, 10.0)
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0


def test_default_stream_write_is_ordered_too():
    """The same with torch's default stream as the writer (the caller stream is then the null stream)."""
    import torch
    from gpu_helpers import compare_volumes
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("sphere", n=8, height=120, width=160, f=131.25, noise=True, seed=3)
    B, H, W = seq["depth"].shape
    K, T = seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    dev = torch.full((B, H, W), float("nan"), dtype=torch.float32, device="cuda")
    pinned = torch.from_numpy(np.ascontiguousarray(seq["depth"], np.float32)).pin_memory()
    torch.cuda.synchronize()
    torch.cuda._sleep(_SPIN)
    dev.copy_(pinned, non_blocking=True)
    vbg = VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64, device="cuda:0")
    vbg.integrate_frames((_Dev(dev), B, H, W), K, T, depth_scale=1.0, depth_max=3.0, trunc_voxel_multiplier=4.0)
    ref = oracle.OracleVBG(0.02, 16, 64)
    for i in range(B):
        ref.integrate_frame(seq["depth"][i], K[i], T[i], 1.0, 3.0, 4.0)
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0


def test_confidence_and_decode_after_side_stream_write():
    import torch
    from mqr import _lib, synthetic
    seq = synthetic.make_sequence("room", n=6, height=120, width=160, f=131.25, noise=True, seed=5)
    B, H, W = seq["depth"].shape
    Tcw = seq["T_cw"].astype(np.float32)
    Tci = np.linalg.inv(seq["T_cw"]).astype(np.float32)
    K32 = np.ascontiguousarray(seq["K"], np.float32)
    s = torch.cuda.Stream()
    # confidence maps of frames that land late on s, written into tensors torch still clears on s
    dev = _late_copy(torch, np.ascontiguousarray(seq["depth"], np.float32), s)
    with torch.cuda.stream(s):
        conf = torch.full((B, H, W), -1.0, dtype=torch.float64, device="cuda")
        valid = torch.full((B, H, W), -1, dtype=torch.int32, device="cuda")
        _lib.call("mqr_confidence", 0, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, B, H, W,
                  _lib.ptr(K32, _lib._f32p), _lib.ptr(np.ascontiguousarray(Tcw.reshape(B, 16)), _lib._f32p),
                  _lib.ptr(np.ascontiguousarray(Tci.reshape(B, 16)), _lib._f32p), None, 0, B, 2, 3.0, 0.05,
                  ctypes.c_void_p(conf.data_ptr()), ctypes.c_void_p(valid.data_ptr()), _lib.MQR_DEVICE)
        c, v = conf.cpu().numpy(), valid.cpu().numpy()
    for i in (0, B // 2, B - 1):
        oc, ov = oracle.confidence(seq["depth"], seq["K"], seq["T_cw"], np.linalg.inv(seq["T_cw"]), i, 2, 3.0, 0.05)
        assert np.array_equal(v[i], ov) and np.array_equal(c[i], oc), f"confidence of frame {i} differs"
    # device ingestion of raw NDC buffers that land late on s
    raw = np.ascontiguousarray(seq["raw"], np.float32)
    draw = _late_copy(torch, raw, s)
    nears = np.full(B, 0.1, np.float64)
    fars = np.full(B, np.inf, np.float64)
    ok = np.zeros(B, np.uint8)
    with torch.cuda.stream(s):
        out = torch.zeros((B, H, W), dtype=torch.float32, device="cuda")
        _lib.call("mqr_decode_depth", 0, ctypes.c_void_p(draw.data_ptr()), _lib.MQR_DEVICE, B, H, W,
                  _lib.ptr(nears, _lib._f64p), _lib.ptr(fars, _lib._f64p), None, None, None, None, _lib.MQR_HOST,
                  0.0, 0, ctypes.c_void_p(out.data_ptr()), _lib.MQR_DEVICE, _lib.ptr(ok, _lib._u8p))
        got = out.cpu().numpy()
    ref = np.empty_like(got)
    ref_ok = np.zeros(B, np.uint8)
    _lib.call("mqr_decode_depth", 0, _lib.ptr(raw), _lib.MQR_HOST, B, H, W, _lib.ptr(nears, _lib._f64p),
              _lib.ptr(fars, _lib._f64p), None, None, None, None, _lib.MQR_HOST, 0.0, 0, _lib.ptr(ref),
              _lib.MQR_HOST, _lib.ptr(ref_ok, _lib._u8p))
    assert np.array_equal(ok, ref_ok)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_caller_stream_is_set_per_call():
    """The Python layer passes torch's current stream before every ordered entry point."""
    import torch
    from mqr import _lib
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _lib.set_stream(_lib.torch_stream())
        got = ctypes.c_void_p()
        _lib.call("mqr_get_stream", ctypes.byref(got))
        assert (got.value or 0) == s.cuda_stream
    _lib.set_stream(_lib.torch_stream())
    _lib.call("mqr_get_stream", ctypes.byref(got))
    assert (got.value or 0) == torch.cuda.current_stream().cuda_stream


def test_confidence_counts_after_side_stream_write():
    """mqr_confidence_counts (the maps as (valid, consistent) byte pairs, csrc/confpack.hip) on frames that
    land late on a side stream: the pairs expand to the oracle's maps exactly -- confidence_map =
    consistent / valid in float64, 0 where valid is 0 -- for every reference frame."""
    import torch
    from mqr import _lib, synthetic
    seq = synthetic.make_sequence("room", n=9, height=120, width=160, f=131.25, noise=True, seed=6)
    B, H, W = seq["depth"].shape
    Tcw = np.ascontiguousarray(seq["T_cw"].astype(np.float32).reshape(B, 16))
    Tci = np.ascontiguousarray(np.linalg.inv(seq["T_cw"]).astype(np.float32).reshape(B, 16))
    K32 = np.ascontiguousarray(seq["K"], np.float32)
    s = torch.cuda.Stream()
    dev = _late_copy(torch, np.ascontiguousarray(seq["depth"], np.float32), s)
    r, a, b = 3, 1, B - 1
    counts = np.full((b - a, H, W), 0xFFFF, np.uint16)
    packed = ctypes.c_int(-1)
    with torch.cuda.stream(s):
        _lib.call("mqr_confidence_counts", 0, ctypes.c_void_p(dev.data_ptr()), _lib.MQR_DEVICE, B, H, W,
                  _lib.ptr(K32, _lib._f32p), _lib.ptr(Tcw, _lib._f32p), _lib.ptr(Tci, _lib._f32p), None, a, b, r,
                  3.0, 0.05, _lib.ptr(counts), ctypes.byref(packed))
    assert packed.value == 1
    valid = (counts & 0xFF).astype(np.int32)
    cons = (counts >> 8).astype(np.int32)
    assert (cons <= valid).all() and valid.max() <= 2 * r
    for i in range(a, b):
        oc, ov = oracle.confidence(seq["depth"], seq["K"], seq["T_cw"], np.linalg.inv(seq["T_cw"]), i, r, 3.0, 0.05)
        with np.errstate(divide="ignore", invalid="ignore"):
            c = np.true_divide(cons[i - a], valid[i - a])
        c[valid[i - a] == 0] = 0.0
        assert np.array_equal(valid[i - a], ov) and np.array_equal(c.view(np.uint64), oc.view(np.uint64)), i


# ---- the other direction: mqr_integrate_frames on device frames returns with its last integrate queued
def _room(n=127, seed=11):
    from mqr import synthetic
    seq = synthetic.make_sequence("room", n=n, height=240, width=320, f=262.5, noise=True, seed=seed)
    return np.ascontiguousarray(seq["depth"], np.float32), seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)


def _oracle(depth, K, T, vs=0.01, dmax=4.0, tm=10.0, ref=None):
    ref = ref if ref is not None else oracle.OracleVBG(vs, 16, 256)
    for i in range(len(depth)):
        ref.integrate_frame(depth[i], K[i], T[i], 1.0, dmax, tm)
    return ref


@pytest.mark.parametrize("side_stream", [False, True])
def test_caller_overwrite_right_after_integrate_frames_is_ordered(side_stream):
    """The caller poisons the frames on its stream the moment integrate_frames returns (no
    synchronize): the write must wait for the library's reads, so the volume is the oracle's over the
    frames as they were.  A long call (254 frames, two batches in flight at the return) makes the
    race wide if the ordering were missing."""
    import torch
    from gpu_helpers import compare_volumes
    from mqr.vbg import VoxelBlockGrid
    depth, K, T = _room(254)
    B, H, W = depth.shape
    dev = torch.from_numpy(depth).cuda()
    torch.cuda.synchronize()
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
    s = torch.cuda.Stream() if side_stream else torch.cuda.current_stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        vbg.integrate_frames((_Dev(dev), B, H, W), K, T, depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        dev.fill_(0.7)  # a wall at 0.7 m in every frame: touches other blocks than the room
    dev.record_stream(s)
    ref = _oracle(depth, K, T)
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0
    torch.cuda.synchronize()
    assert float(dev.max()) == float(np.float32(0.7))


def test_reset_extract_and_second_call_after_an_unfinished_integrate():
    """reset, a second integrate_frames and extraction issued while the previous integrate still runs:
    each orders itself behind it on the device (no host wait), and the results are the oracle's."""
    import torch
    from gpu_helpers import compare_volumes
    from mqr.vbg import VoxelBlockGrid
    d1, K1, T1 = _room(127, seed=11)
    d2, K2, T2 = _room(100, seed=12)
    B1, H, W = d1.shape
    t1, t2 = torch.from_numpy(d1).cuda(), torch.from_numpy(d2).cuda()
    torch.cuda.synchronize()
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
    # (a) reset behind an unfinished integrate, then the second sequence alone
    vbg.integrate_frames((_Dev(t1), B1, H, W), K1, T1, **kw)
    vbg.reset()
    vbg.integrate_frames((_Dev(t2), len(d2), H, W), K2, T2, **kw)
    ref2 = _oracle(d2, K2, T2)
    assert compare_volumes(vbg.export(), ref2.export(), 0.0) == 0.0
    # (b) two calls back to back (the second's touch behind the first's integrate), then the mesh at once
    vbg.reset()
    vbg.integrate_frames((_Dev(t1), B1, H, W), K1, T1, **kw)
    vbg.integrate_frames((_Dev(t2), len(d2), H, W), K2, T2, **kw)
    mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
    ref12 = _oracle(d2, K2, T2, ref=_oracle(d1, K1, T1))
    assert compare_volumes(vbg.export(), ref12.export(), 0.0) == 0.0
    _, _, otri = ref12.extract_mesh(1.5)
    assert mesh.triangles.shape[0] == otri.shape[0]


def test_synchronous_return_variant_is_identical():
    """Variant bit 24 (the A/B of the asynchronous return) drains the streams before returning: same volume."""
    import torch
    from mqr import _lib
    from mqr.vbg import VoxelBlockGrid
    depth, K, T = _room(60, seed=13)
    B, H, W = depth.shape
    t = torch.from_numpy(depth).cuda()
    torch.cuda.synchronize()
    out = []
    for variant in (0, 0x1000000):
        vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
        _lib.call("mqr_vbg_set_variant", vbg.handle, variant)
        vbg.integrate_frames((_Dev(t), B, H, W), K, T, depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        out.append(vbg.export())
    from gpu_helpers import compare_volumes
    assert compare_volumes(out[0], out[1], 0.0) == 0.0  # (block order is the touch's arrival order)


def test_device_buffer_freed_right_after_integrate_frames():
    """A library-allocated frame buffer (mqr_device_alloc) freed the moment integrate_frames returns:
    mqr_device_free waits for the device, so the in-flight integrate still reads the frames."""
    from gpu_helpers import compare_volumes
    from mqr._lib import DeviceBuffer
    from mqr.vbg import VoxelBlockGrid
    depth, K, T = _room(200, seed=14)
    B, H, W = depth.shape
    buf = DeviceBuffer.from_array(depth)
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
    vbg.integrate_frames((buf, B, H, W), K, T, depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    buf.free()
    assert compare_volumes(vbg.export(), _oracle(depth, K, T).export(), 0.0) == 0.0


def _flips(vbg):
    from mqr import _lib
    n = ctypes.c_int64(-1)
    _lib.call("mqr_vbg_flips", vbg.handle, ctypes.byref(n))
    return n.value


@pytest.mark.parametrize("variant", [0, 0x2000000])
def test_reset_behind_an_unfinished_integrate_swaps_sets(variant):
    """reset while an integrate is in flight swaps in the volume's second table / pool set instead of waiting
    (variant 0; bit 25 waits).  The calls alternate a long and a short sequence with no synchronize, so each
    reset finds the previous call's last integrate running: a set swapped back in must be cleared only after
    the integrate that last read it (the long one, two calls earlier), and the second set -- allocated at the
    capacities of the first, which grows in the first call -- must be replaced when the first grows past it.
    Every volume and mesh is the oracle's, the capacity is kept across the swaps, and the swap count says
    which path ran."""
    import torch
    from gpu_helpers import compare_volumes
    from mqr.vbg import VoxelBlockGrid
    from mqr import _lib
    d1, K1, T1 = _room(254, seed=21)
    d2, K2, T2 = _room(90, seed=22)
    B1, H, W = d1.shape
    t1, t2 = torch.from_numpy(d1).cuda(), torch.from_numpy(d2).cuda()
    torch.cuda.synchronize()
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    a = (_Dev(t1), B1, H, W), K1, T1
    b = (_Dev(t2), len(d2), H, W), K2, T2
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64, device="cuda:0")
    _lib.call("mqr_vbg_set_variant", vbg.handle, variant)
    for frames, K, T in (a, b, a, b, a):  # resets 2-5 each behind the previous call's unfinished integrate
        vbg.reset()
        vbg.integrate_frames(frames, K, T, **kw)
    ref1, ref2 = _oracle(d1, K1, T1), _oracle(d2, K2, T2)
    mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
    assert compare_volumes(vbg.export(), ref1.export(), 0.0) == 0.0
    assert mesh.triangles.shape[0] == ref1.extract_mesh(1.5)[2].shape[0]
    cap = vbg.capacity()
    assert cap >= vbg.size()
    vbg.integrate_frames(*b, **kw)  # onto the first sequence (the mask / counter state after the swaps)
    assert compare_volumes(vbg.export(), _oracle(d2, K2, T2, ref=_oracle(d1, K1, T1)).export(), 0.0) == 0.0
    vbg.reset()  # nothing in flight (export drained): an in-place clear
    vbg.integrate_frames(*b, **kw)
    vbg.reset()
    vbg.integrate_frames(*a, **kw)
    assert compare_volumes(vbg.export(), ref1.export(), 0.0) == 0.0
    assert vbg.capacity() >= cap
    flips = _flips(vbg)
    if variant:
        assert flips == 0
    else:
        assert flips == 5, flips  # 4 in the loop + the one behind the short call
    del ref2


def test_resident_frames_back_to_back_passes():
    """MQR_DEVICE_RESIDENT frames (integrate_frames(resident=True)): the caller stream is not made to wait
    for the call's integrates, so the next call's touch may run beside the previous call's last integrate
    (the overlap itself is measured by tools/ab_async.py and the bench trace, not here).  Reset passes over
    resident frames -- mixed with an MQR_DEVICE pass, on a side caller stream and the default one, two
    captures alternating with no synchronize -- leave the oracle's volumes."""
    import torch
    from gpu_helpers import compare_volumes
    from mqr.vbg import VoxelBlockGrid
    d1, K1, T1 = _room(254, seed=31)
    d2, K2, T2 = _room(127, seed=32)
    B1, H, W = d1.shape
    t1, t2 = torch.from_numpy(d1).cuda(), torch.from_numpy(d2).cuda()
    torch.cuda.synchronize()
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0, resident=True)
    a = (_Dev(t1), B1, H, W), K1, T1
    b = (_Dev(t2), len(d2), H, W), K2, T2
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=256, device="cuda:0")
    s = torch.cuda.Stream()  # a side caller stream, then the default one
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        vbg.integrate_frames(*a, **kw)
        vbg.reset()
        vbg.integrate_frames(*a, **dict(kw, resident=False))
        vbg.reset()
        vbg.integrate_frames(*a, **kw)
    torch.cuda.current_stream().wait_stream(s)
    for frames, K, T in (b, a, b, a):
        vbg.reset()
        vbg.integrate_frames(frames, K, T, **kw)
    vbg.integrate_frames(*b, **kw)  # onto the first capture, still without a synchronize
    torch.cuda.synchronize()
    ref = _oracle(d2, K2, T2, ref=_oracle(d1, K1, T1))
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0
    assert _flips(vbg) >= 5
