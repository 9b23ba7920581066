"""Device depth ingestion (mqr_decode_depth) against the reference's own decode.

Golden vectors: tests/golden/decode_golden.npz, produced by the reference's
convert_depth_to_linear / is_depth_map_valid (make_golden.py) with near/far as Python floats
(`linear`, float32 decode) and as numpy float64 scalars (`linear64`, what the pipeline passes).
Bit-exact.  Masking and full-size frames are checked against mqr.depth_utils, the numpy mirror
pinned by the same vectors (tests/test_dataio_golden.py)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_decode_matches_reference_golden(golden_dir):
    from mqr.ingest import decode_depth_frames
    g = np.load(os.path.join(golden_dir, "decode_golden.npz"))
    raw, params = g["raw"], g["params"]
    N = raw.shape[0]
    for k, (near, far) in enumerate(params):
        d32, ok = decode_depth_frames(raw, [float(near)] * N, [float(far)] * N)
        assert np.array_equal(ok, g["valid"])
        assert np.array_equal(d32.view(np.uint32), g["linear"][k].view(np.uint32)), (near, far)
        d64, ok64 = decode_depth_frames(raw, [np.float64(near)] * N, [np.float64(far)] * N)
        assert np.array_equal(ok64, g["valid"])
        assert np.array_equal(d64.view(np.uint32), g["linear64"][k].view(np.uint32)), (near, far)


def test_decode_full_frames_and_mask_match_numpy():
    from mqr.depth_utils import convert_depth_to_linear
    from mqr.ingest import decode_depth_frames
    rng = np.random.default_rng(3)
    N, H, W = 5, 480, 640
    raw = rng.random((N, H, W)).astype(np.float32)
    raw[:, ::17, ::13] = 1.0                    # decodes to 0 (denominator 0)
    raw[0, 7, 9] = 0.0
    raw[3] = 0.0                                # invalid frame
    conf = rng.random((N, H, W))
    conf[1, 0, :5] = np.nan
    vc = rng.integers(0, 6, (N, H, W)).astype(np.int32)
    has = np.array([1, 1, 0, 1, 1], bool)
    nears = [np.float64(0.1), np.float64(0.05), 0.1, np.float64(0.1), np.float64(0.2)]
    fars = [np.float64(np.inf), np.float64(50.0), np.inf, np.float64(np.inf), 100.0]
    out, ok = decode_depth_frames(raw, nears, fars, conf=conf, valid_count=vc, has_mask=has,
                                  confidence_threshold=0.3, valid_count_threshold=2)
    assert ok.tolist() == [True, True, True, False, True]
    for f in range(N):
        ref = convert_depth_to_linear(raw[f], nears[f], fars[f])
        if has[f]:
            ref[conf[f] < 0.3] = 0.0
            ref[vc[f] < 2] = 0.0
        assert np.array_equal(out[f].view(np.uint32), ref.view(np.uint32)), f


def test_decode_device_in_out():
    from mqr._lib import DeviceBuffer
    from mqr.depth_utils import convert_depth_to_linear
    from mqr.ingest import decode_depth_frames
    rng = np.random.default_rng(4)
    raw = rng.random((3, 120, 160)).astype(np.float32)
    r_buf = DeviceBuffer.from_array(raw)
    o_buf = DeviceBuffer(raw.nbytes)
    out, ok = decode_depth_frames((r_buf, 3, 120, 160), [np.float64(0.1)] * 3, [np.float64(np.inf)] * 3,
                                  out_ptr=o_buf)
    assert out is None and ok.all()
    got = o_buf.to_array(raw.shape, np.float32)
    for f in range(3):
        assert np.array_equal(got[f], convert_depth_to_linear(raw[f], np.float64(0.1), np.float64(np.inf)))


def test_decode_rejects_unsupported_scalar_types():
    from mqr.ingest import decode_depth_frames
    with pytest.raises(TypeError):
        decode_depth_frames(np.zeros((1, 4, 4), np.float32), [np.float32(0.1)], [np.inf])


@pytest.mark.parametrize("shape", [(480, 640), (37, 53)])   # vector path, and the scalar path (H*W % 4 != 0)
def test_decode_byte_mask_equals_the_map_mask(shape):
    """mqr_decode_depth_masked with the mask byte (conf < thr) | (count < thr) gives the bits and the
    validity of mqr_decode_depth with the maps; a float count threshold compares as numpy does."""
    from mqr.depth_utils import convert_depth_to_linear
    from mqr.ingest import decode_depth_frames
    rng = np.random.default_rng(9)
    H, W = shape
    N = 5
    raw = rng.random((N, H, W)).astype(np.float32)
    raw[:, ::7, ::5] = 1.0
    raw[2] = 0.0
    conf = rng.random((N, H, W))
    conf[0, 0, :5] = np.nan
    vc = rng.integers(0, 6, (N, H, W)).astype(np.int32)
    has = np.array([1, 0, 1, 1, 1], bool)
    nears = [np.float64(0.1), 0.1, np.float64(0.1), np.float64(0.05), 0.2]
    fars = [np.float64(np.inf), np.inf, np.float64(np.inf), np.float64(50.0), 100.0]
    for vthr in (2, 2.5):
        m8 = ((conf < 0.3) | (vc < vthr)).astype(np.uint8)
        a, ok_a = decode_depth_frames(raw, nears, fars, conf=conf, valid_count=vc, has_mask=has,
                                      confidence_threshold=0.3, valid_count_threshold=vthr)
        b, ok_b = decode_depth_frames(raw, nears, fars, mask=m8, has_mask=has)
        assert np.array_equal(ok_a, ok_b) and ok_b.tolist() == [True, True, False, True, True]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        for f in range(N):
            ref = convert_depth_to_linear(raw[f], nears[f], fars[f])
            if has[f]:
                ref[conf[f] < 0.3] = 0.0
                ref[vc[f] < vthr] = 0.0
            assert np.array_equal(b[f].view(np.uint32), ref.view(np.uint32)), (vthr, f)
    c, ok_c = decode_depth_frames(raw, nears, fars, mask=np.ones((N, H, W), np.uint8), has_mask=None)
    d, _ = decode_depth_frames(raw, nears, fars)
    assert np.array_equal(c.view(np.uint32), d.view(np.uint32)) and np.array_equal(ok_c, ok_a)


def test_decode_byte_mask_device_resident():
    """mqr_decode_depth_masked with raw frames, mask bytes and output all in HBM (MQR_DEVICE)."""
    import ctypes
    from mqr import _lib
    from mqr._lib import DeviceBuffer
    from mqr.ingest import decode_depth_frames
    rng = np.random.default_rng(12)
    N, H, W = 3, 60, 80
    raw = rng.random((N, H, W)).astype(np.float32)
    m8 = (rng.random((N, H, W)) < 0.3).astype(np.uint8)
    has = np.array([1, 0, 1], np.uint8)
    nears = np.full(N, 0.1, np.float64)
    fars = np.full(N, np.inf, np.float64)
    r_buf, m_buf, o_buf = DeviceBuffer.from_array(raw), DeviceBuffer.from_array(m8), DeviceBuffer(raw.nbytes)
    ok = np.zeros(N, np.uint8)
    _lib.call("mqr_decode_depth_masked", 0, r_buf.ptr, _lib.MQR_DEVICE, N, H, W, _lib.ptr(nears, _lib._f64p),
              _lib.ptr(fars, _lib._f64p), None, m_buf.ptr, _lib.ptr(has, _lib._u8p), _lib.MQR_DEVICE, o_buf.ptr,
              _lib.MQR_DEVICE, _lib.ptr(ok, _lib._u8p))
    got = o_buf.to_array(raw.shape, np.float32)
    ref, ref_ok = decode_depth_frames(raw, [0.1] * N, [np.inf] * N, mask=m8, has_mask=has.astype(bool))
    assert np.array_equal(ok.astype(bool), ref_ok) and np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert (got[0][m8[0] != 0] == 0).all() and np.array_equal(got[1], ref[1])
