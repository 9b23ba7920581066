"""csrc/frameio.hip: mqr_read_frames, the native reader of raw depth files and np.savez confidence npz
(reference dataio/depth_data_io.py:33-53, 91-104), and mqr_write_confidence_npz, the native np.savez of
the confidence maps (depth_data_io.py:106-115) with its CRC-32.  Host-only, so they run here without a
GPU: every frame the reader reports read must equal np.fromfile / np.load of the same file, every file it
cannot take (missing, wrong size, compressed, another dtype or shape, truncated) must be reported, not
guessed; the writer's files must load with np.load and hold the members np.savez writes, byte for byte."""
import ctypes
import os
import zipfile

import numpy as np
import pytest


def _lib():
    from mqr import _lib
    try:
        _lib.load()
    except Exception as e:  # pragma: no cover - the library is built by __graft_entry__.build()
        pytest.skip(f"libmqr_hip.so not loadable here: {e}")
    return _lib


def _read(lib, raws, confs, H, W, threads):
    n = len(raws)
    raw = np.full((n, H, W), np.nan, np.float32)
    conf = np.full((n, H, W), np.nan, np.float64)
    vc = np.full((n, H, W), -7, np.int32)
    st = np.zeros(n, np.uint8)
    rp = (ctypes.c_char_p * n)(*[os.fsencode(str(p)) for p in raws])
    cp = (ctypes.c_char_p * n)(*[None if p is None else os.fsencode(str(p)) for p in confs]) if confs else None
    lib.call("mqr_read_frames", n, rp, cp, H, W, lib.ptr(raw), lib.ptr(conf) if cp else None,
             lib.ptr(vc) if cp else None, lib.ptr(st), threads)
    return raw, conf, vc, st


@pytest.mark.parametrize("threads", [1, 4])
def test_read_frames_matches_numpy_and_reports_the_rest(tmp_path, threads):
    lib = _lib()
    H, W = 24, 40
    rng = np.random.default_rng(3)
    raws, confs, expect = [], [], []
    for i in range(13):
        r = rng.random((H, W), dtype=np.float32)
        c = rng.random((H, W))
        v = rng.integers(0, 9, (H, W)).astype(np.int32)
        rp, cp = tmp_path / f"{i}.raw", tmp_path / f"{i}.npz"
        r.astype("<f4").tofile(rp)
        np.savez(cp, confidence_map=c, valid_count=v)
        raws.append(rp)
        confs.append(cp)
        expect.append((r, c, v))
    os.unlink(raws[1])                                                   # raw missing
    np.zeros(H * W + 3, "<f4").tofile(raws[2])                           # raw of the wrong size
    os.unlink(confs[3])                                                  # confidence missing
    np.savez_compressed(confs[4], confidence_map=expect[4][1], valid_count=expect[4][2])   # compressed
    np.savez(confs[5], confidence_map=expect[5][1].astype(np.float32), valid_count=expect[5][2])  # dtype
    np.savez(confs[6], confidence_map=expect[6][1][:, :-1].copy(), valid_count=expect[6][2])    # shape
    with open(confs[7], "r+b") as f:                                     # truncated
        f.truncate(os.path.getsize(confs[7]) // 2)
    np.savez(confs[8], valid_count=expect[8][2])                         # member missing
    np.savez(confs[9], confidence_map=np.asfortranarray(expect[9][1]), valid_count=expect[9][2])  # F order
    confs[10] = None                                                     # no confidence asked for
    with zipfile.ZipFile(confs[12], "w", zipfile.ZIP_STORED) as z:       # members that are not .npy
        z.writestr("confidence_map.npy", b"\x00" * (128 + 8 * H * W))
        z.writestr("valid_count.npy", b"\x00" * (128 + 4 * H * W))
    raw, conf, vc, st = _read(lib, raws, confs, H, W, threads)
    ok_raw, miss_raw, oth_raw = lib.MQR_FRAME_RAW_OK, lib.MQR_FRAME_RAW_MISSING, lib.MQR_FRAME_RAW_OTHER
    ok_c, miss_c, oth_c = lib.MQR_FRAME_CONF_OK, lib.MQR_FRAME_CONF_MISSING, lib.MQR_FRAME_CONF_OTHER
    want = {0: ok_raw | ok_c, 1: miss_raw | ok_c, 2: oth_raw | ok_c, 3: ok_raw | miss_c, 4: ok_raw | oth_c,
            5: ok_raw | oth_c, 6: ok_raw | oth_c, 7: ok_raw | oth_c, 8: ok_raw | oth_c, 9: ok_raw | oth_c,
            10: ok_raw, 11: ok_raw | ok_c, 12: ok_raw | oth_c}
    assert {i: int(s) for i, s in enumerate(st)} == want
    for i, (r, c, v) in enumerate(expect):
        if st[i] & ok_raw:
            assert np.array_equal(raw[i], np.fromfile(raws[i], "<f4").reshape(H, W))
        else:
            assert (raw[i] == 0).all()  # no frame: zeros (decoded invalid)
        if st[i] & ok_c:
            d = np.load(confs[i])
            assert np.array_equal(conf[i], d["confidence_map"]) and np.array_equal(vc[i], d["valid_count"])


def test_read_frames_without_confidence_and_empty(tmp_path):
    lib = _lib()
    H, W = 8, 8
    p = tmp_path / "a.raw"
    np.arange(64, dtype="<f4").tofile(p)
    raw, _, _, st = _read(lib, [p], None, H, W, 2)
    assert st[0] == lib.MQR_FRAME_RAW_OK and np.array_equal(raw[0].ravel(), np.arange(64, dtype=np.float32))
    lib.call("mqr_read_frames", 0, None, None, H, W, None, None, None, None, 2)


def test_crc32_matches_zlib():
    import zlib
    lib = _lib()
    rng = np.random.default_rng(5)
    for n in list(range(0, 200)) + [1000, 4095, 65536 + 17, 3 << 20]:
        b = rng.integers(0, 256, n, dtype=np.uint8)
        for start in (0, 0x12345678):
            got = lib.load().mqr_crc32(start, b.ctypes.data if n else None, n)
            assert got == zlib.crc32(b.tobytes(), start), (n, start)


@pytest.mark.parametrize("threads", [1, 3])
def test_write_confidence_npz_roundtrip(tmp_path, threads):
    """The native writer's files load with np.load (CRC-checked by zipfile), hold the arrays bit for bit,
    pass zipfile's own test, and read back through mqr_read_frames; an unwritable path is reported."""
    import zipfile
    lib = _lib()
    H, W, n = 30, 50, 5
    rng = np.random.default_rng(7)
    conf = rng.random((n, H, W))
    conf[0, 0, 0] = np.nan
    valid = rng.integers(-5, 30, (n, H, W)).astype(np.int32)
    paths = [tmp_path / f"{i}.npz" for i in range(n)]
    paths[3] = tmp_path / "no_such_dir" / "3.npz"
    st = np.full(n, -1, np.int32)
    pp = (ctypes.c_char_p * (n + 1))(*[os.fsencode(str(p)) for p in paths], None)  # null path: skipped
    conf = np.concatenate([conf, conf[:1]])
    valid = np.concatenate([valid, valid[:1]])
    st = np.full(n + 1, -1, np.int32)
    lib.call("mqr_write_confidence_npz", n + 1, pp, lib.ptr(conf), lib.ptr(valid), H, W, lib.ptr(st), threads)
    assert st[3] != 0 and all(st[i] == 0 for i in range(n + 1) if i != 3)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["0.npz", "1.npz", "2.npz", "4.npz"]
    for i in (0, 1, 2, 4):
        with zipfile.ZipFile(paths[i]) as z:
            assert z.testzip() is None and z.namelist() == ["confidence_map.npy", "valid_count.npy"]
        d = np.load(paths[i])
        assert d["confidence_map"].dtype == np.float64 and d["valid_count"].dtype == np.int32
        assert np.array_equal(d["confidence_map"], conf[i], equal_nan=True)
        assert np.array_equal(d["valid_count"], valid[i])
        ref = tmp_path / f"ref{i}.npz"
        np.savez(ref, confidence_map=conf[i], valid_count=valid[i])
        with zipfile.ZipFile(ref) as a, zipfile.ZipFile(paths[i]) as b:  # same members, same bytes
            for name in a.namelist():
                assert a.read(name) == b.read(name)
    ok = [0, 1, 2, 4]
    raws = [tmp_path / f"r{i}.raw" for i in ok]
    for r in raws:
        np.zeros((H, W), "<f4").tofile(r)
    _, c2, v2, st2 = _read(lib, raws, [paths[i] for i in ok], H, W, 2)
    assert (st2 & lib.MQR_FRAME_CONF_OK).all()
    assert np.array_equal(c2, conf[ok], equal_nan=True) and np.array_equal(v2, valid[ok])


@pytest.mark.parametrize("shape", [(24, 40), (210, 330)])   # the second spans several 32768-pixel read blocks
def test_read_frames_masked_matches_the_decode_mask(tmp_path, shape):
    """mqr_read_frames_masked: the same statuses and raw frames as mqr_read_frames, and per frame read the
    mask byte (confidence_map < conf_thr) | (valid_count < count_thr) that load_depth_map applies
    (reference o3d_utils.py:131-142) -- NaN confidence never masks, as in the comparison numpy makes."""
    lib = _lib()
    H, W = shape
    rng = np.random.default_rng(11)
    raws, confs = [], []
    for i in range(6):
        c = rng.random((H, W))
        c[rng.random((H, W)) < 0.05] = np.nan
        c[0, :3] = (-np.inf, np.inf, 0.02)
        v = rng.integers(-2, 6, (H, W)).astype(np.int32)
        rp, cp = tmp_path / f"{i}.raw", tmp_path / f"{i}.npz"
        rng.random((H, W), dtype=np.float32).astype("<f4").tofile(rp)
        np.savez(cp, confidence_map=c, valid_count=v)
        raws.append(rp)
        confs.append(cp)
    os.unlink(confs[2])
    np.savez_compressed(confs[3], confidence_map=np.zeros((H, W)), valid_count=np.zeros((H, W), np.int32))
    confs[4] = None
    raw0, _, _, st0 = _read(lib, raws, confs, H, W, 2)
    n = len(raws)
    raw = np.full((n, H, W), np.nan, np.float32)
    mask = np.full((n, H, W), 7, np.uint8)
    st = np.zeros(n, np.uint8)
    rp = (ctypes.c_char_p * n)(*[os.fsencode(str(p)) for p in raws])
    cp = (ctypes.c_char_p * n)(*[None if p is None else os.fsencode(str(p)) for p in confs])
    thr, vthr = 0.02, 2
    lib.call("mqr_read_frames_masked", n, rp, cp, H, W, thr, vthr, lib.ptr(raw), lib.ptr(mask), lib.ptr(st), 3)
    assert np.array_equal(st, st0) and np.array_equal(raw, raw0)
    for i in range(n):
        if st[i] & lib.MQR_FRAME_CONF_OK:
            d = np.load(confs[i])
            want = (d["confidence_map"] < thr) | (d["valid_count"] < vthr)
            assert np.array_equal(mask[i], want.astype(np.uint8))


@pytest.mark.parametrize("threads", [1, 4])
def test_write_confidence_npz_counts_equals_np_savez_of_the_maps(tmp_path, threads):
    """mqr_write_confidence_npz_counts: files byte-identical (members) to np.savez of the maps the
    reference builds from the two counts -- confidence_map = np.true_divide(consistent, valid), 0 where
    valid is 0, valid_count int32 (estimate_depth_confidences.py:41-79) -- for every (valid, consistent)
    pair of the byte range; a null path writes nothing."""
    import zipfile
    lib = _lib()
    H, W = 256, 257
    v, k = np.meshgrid(np.arange(256), np.arange(257), indexing="ij")
    k = np.minimum(k, v)
    n = 3
    valid = np.stack([v, np.roll(v, 1, 0), np.roll(v, 5, 1)]).astype(np.int32)
    cons = np.stack([k, np.roll(k, 1, 0), np.roll(k, 5, 1)]).astype(np.int32)
    counts = (valid | cons << 8).astype(np.uint16)
    paths = [tmp_path / f"{i}.npz" for i in range(n)]
    pp = (ctypes.c_char_p * (n + 1))(*[os.fsencode(str(p)) for p in paths], None)
    counts = np.concatenate([counts, counts[:1]])
    st = np.full(n + 1, -1, np.int32)
    lib.call("mqr_write_confidence_npz_counts", n + 1, pp, lib.ptr(counts), H, W, lib.ptr(st), threads)
    assert (st == 0).all() and sorted(p.name for p in tmp_path.iterdir()) == ["0.npz", "1.npz", "2.npz"]
    for i in range(n):
        with np.errstate(divide="ignore", invalid="ignore"):
            conf = np.true_divide(cons[i], valid[i])
        conf[valid[i] == 0] = 0.0
        ref = tmp_path / f"ref{i}.npz"
        np.savez(ref, confidence_map=conf, valid_count=valid[i])
        with zipfile.ZipFile(ref) as a, zipfile.ZipFile(paths[i]) as b:
            assert b.testzip() is None and a.namelist() == b.namelist()
            for name in a.namelist():
                assert a.read(name) == b.read(name)
