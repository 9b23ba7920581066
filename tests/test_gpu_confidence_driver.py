"""Row a10: the confidence driver ``mqr.confidence.estimate_depth_confidences`` end to end on a
capture in the reference's layout (estimate_depth_confidences.py:82-153), every written npz
compared with the CPU oracle's build_confidence_map restatement (pinned by the reference's golden
vectors, tests/test_oracle_golden.py).

Covers: the dir-level skip (``skip_if_output_dir_exists``), an existing per-frame file kept as is
(resume rule :94-96), a frame missing / invalid after the dataset was cached (no output for it,
skipped as a neighbour), reference-frame chunks that cross the 64-frame REF_CHUNK boundary and
windows clipped at both ends of the sequence -- on the device-resident path (native reads, frames
decoded once into HBM, native npz writes) and on the standard one (MQR_NATIVE_IO=0), and a write
failure on each, reported per frame with the reference's message.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

N, H, W = 150, 120, 160
R_WIN, DMAX, ERR = 10, 4.0, 0.08


@pytest.fixture()
def capture(tmp_path):
    from mqr import _lib, synthetic
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    _lib.load()
    seq = synthetic.make_sequence("room", n=N, height=H, width=W, f=131.25, noise=True, seed=21)
    synthetic.write_capture(tmp_path, seq)
    io = DepthDataIO(tmp_path)
    ds = io.load_depth_dataset(Side.LEFT)  # builds and caches the dataset (dataset/left_depth_dataset.npz)
    assert len(ds) == N
    return tmp_path, seq, io, ds, Side


def _inputs(io, ds, Side):
    """What the driver sees: the DataIO decode of every frame (None -> zeros), K with the cx flip,
    Open3D camera->world poses and their float32 inverse (estimate_depth_confidences.py:129-136)."""
    from mqr.models import CoordinateSystem
    from mqr.o3d_utils import compute_o3d_intrinsic_matrices
    frames = [io.load_depth_map_by_index(side=Side.LEFT, dataset=ds, index=i) for i in range(len(ds))]
    ok = np.array([f is not None for f in frames], np.uint8)
    depth = np.stack([f if f is not None else np.zeros((H, W), np.float32) for f in frames])
    K = compute_o3d_intrinsic_matrices(ds)
    Tcw = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                  is_camera=True).extrinsics_cw
    return depth, ok, K, Tcw, np.linalg.inv(Tcw)


def _config(skip):
    from mqr.confidence import DepthConfidenceEstimationConfig
    return DepthConfidenceEstimationConfig(target_frame_range=R_WIN, depth_max=DMAX, error_threshold=ERR,
                                           skip_if_output_dir_exists=skip)


@pytest.mark.parametrize("native_io", [True, False])
def test_driver_outputs_match_oracle(capture, native_io, monkeypatch):
    from mqr.confidence import REF_CHUNK, estimate_depth_confidences
    if not native_io:
        monkeypatch.setenv("MQR_NATIVE_IO", "0")
    from mqr.dataio import DepthDataIO
    from mqr.models import ConfidenceMap
    path, seq, io, ds, Side = capture
    assert REF_CHUNK < N
    files = sorted((path / "left_depth").glob("*.raw"))
    files[63].unlink()                                # missing after caching, at the chunk edge
    np.zeros((H, W), "<f4").tofile(files[64])         # all-zero buffer: invalid
    kept = ConfidenceMap(np.full((H, W), 0.25), np.full((H, W), 7, np.int32))
    io.save_confidence_map(Side.LEFT, int(ds.timestamps[5]), kept)  # existing file: kept
    io2 = DepthDataIO(path)  # a fresh DataIO: the cached dataset is read back from disk
    estimate_depth_confidences(io2, _config(skip=False), sides=[Side.LEFT])

    depth, ok, K, Tcw, Ti = _inputs(io2, ds, Side)
    assert list(np.nonzero(ok == 0)[0]) == [63, 64]
    written = 0
    for i, ts in enumerate(ds.timestamps):
        cm = io2.load_confidence_map(Side.LEFT, int(ts))
        if i in (63, 64):
            assert cm is None, "a frame that fails to load gets no confidence map"
            continue
        if i == 5:
            assert np.array_equal(cm.confidence_map, kept.confidence_map)
            assert np.array_equal(cm.valid_count, kept.valid_count)
            continue
        oc, ov = oracle.confidence(depth, K, Tcw, Ti, i, R_WIN, DMAX, ERR, frame_valid=ok)
        assert cm.confidence_map.dtype == np.float64 and cm.valid_count.dtype == np.int32
        assert np.array_equal(cm.valid_count, ov), i
        assert np.array_equal(cm.confidence_map, oc), i
        written += 1
    assert written == N - 3


def test_driver_skips_existing_output_dir(capture):
    from mqr.confidence import estimate_depth_confidences
    path, seq, io, ds, Side = capture
    conf_dir = path / "left_depth_confidence"
    conf_dir.mkdir()
    estimate_depth_confidences(io, _config(skip=True), sides=[Side.LEFT])
    assert list(conf_dir.iterdir()) == []
    estimate_depth_confidences(io, _config(skip=False), sides=[Side.LEFT])
    assert len(list(conf_dir.glob("*.npz"))) == N


def test_build_confidence_map_wrapper(capture):
    """build_confidence_map (estimate_depth_confidences.py:15-79) for single reference frames."""
    from mqr.confidence import build_confidence_map
    path, seq, io, ds, Side = capture
    depth, ok, K, Tcw, Ti = _inputs(io, ds, Side)
    for i in (0, 70, N - 1):
        cm = build_confidence_map(io, ds, K, Tcw, Ti, Side.LEFT, i, R_WIN, DMAX, ERR)
        oc, ov = oracle.confidence(depth, K, Tcw, Ti, i, R_WIN, DMAX, ERR)
        assert np.array_equal(cm.valid_count, ov)
        assert np.array_equal(cm.confidence_map, oc)


def _ragged_capture(tmp, g):
    """The reference-generated ragged capture (two frame sizes) written back to disk."""
    import pandas as pd
    cols = [str(c) for c in g["descriptor_cols"]]
    df = pd.DataFrame(g["descriptor"], columns=cols)
    for c in ("timestamp_ms", "width", "height"):
        df[c] = df[c].astype(np.int64)
    (tmp / "left_depth").mkdir(parents=True)
    for i, ts in enumerate(df["timestamp_ms"]):
        g[f"raw_{i}"].astype("<f4").tofile(tmp / "left_depth" / f"{ts}.raw")
    df.to_csv(tmp / "left_depth_descriptors.csv", index=False)


@pytest.mark.parametrize("tag,params", [("a", (3, 3.0, 0.05)), ("b", (10, 4.0, 0.08))])
def test_driver_mixed_frame_sizes_match_reference_golden(tmp_path, golden_dir, tag, params):
    """Windows that mix two frame sizes: the reference interpolates each neighbour within its own
    (h, w) (compute_pixel_error_map.py:4-60), so such a neighbour counts; the driver and the
    build_confidence_map wrapper reproduce the reference's maps bit for bit
    (tests/golden/confidence_ragged_golden.npz, generated by the reference itself)."""
    import os
    from mqr import _lib
    from mqr.confidence import DepthConfidenceEstimationConfig, build_confidence_map, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    _lib.load()
    g = np.load(os.path.join(golden_dir, "confidence_ragged_golden.npz"))
    r, dmax, thr = params
    _ragged_capture(tmp_path, g)
    io = DepthDataIO(tmp_path)
    estimate_depth_confidences(io, DepthConfidenceEstimationConfig(target_frame_range=r, depth_max=dmax,
                                                                   error_threshold=thr,
                                                                   skip_if_output_dir_exists=False),
                               sides=[Side.LEFT])
    ds = io.load_depth_dataset(Side.LEFT)
    n = int(g["n"])
    assert len(ds) == n and len(set(zip(ds.widths, ds.heights))) == 2
    for i, ts in enumerate(ds.timestamps):
        cm = io.load_confidence_map(Side.LEFT, int(ts))
        assert cm is not None and cm.confidence_map.shape == g[f"conf_{tag}_{i}"].shape, i
        assert np.array_equal(cm.valid_count, g[f"valid_{tag}_{i}"]), i
        assert np.array_equal(cm.confidence_map, g[f"conf_{tag}_{i}"]), i
    for i in (0, 5, 8, n - 1):
        cm = build_confidence_map(io, ds, g["K"], g["T_cw"], g["T_cw_inv"], Side.LEFT, i, r, dmax, thr)
        assert np.array_equal(cm.valid_count, g[f"valid_{tag}_{i}"]), i
        assert np.array_equal(cm.confidence_map, g[f"conf_{tag}_{i}"]), i


def test_driver_reports_a_failing_frame_and_goes_on(capture, capsys, monkeypatch):
    """estimate_depth_confidences.py:98-117: an error while saving one reference frame's map is
    printed with the reference's message and that frame is skipped; every other frame is written."""
    from mqr.confidence import estimate_depth_confidences
    path, seq, io, ds, Side = capture
    bad = int(ds.timestamps[7])
    orig = io.save_confidence_map

    def flaky(side, timestamp, confidence_map):
        if int(timestamp) == bad:
            raise OSError("disk full")
        return orig(side=side, timestamp=timestamp, confidence_map=confidence_map)

    monkeypatch.setattr(io, "save_confidence_map", flaky)
    estimate_depth_confidences(io, _config(skip=False), sides=[Side.LEFT])
    out = capsys.readouterr().out
    assert f"[Error] build_and_save_confidence_map failed for LEFT frame 7 (timestamp {bad}): disk full" in out
    conf_dir = path / "left_depth_confidence"
    assert len(list(conf_dir.glob("*.npz"))) == N - 1
    assert io.load_confidence_map(Side.LEFT, bad) is None


def test_driver_native_write_failure_reported(capture, capsys):
    """On the device-resident path a file that cannot be written (here a directory in its place) is
    reported with the reference's message and errno, and every other frame is written."""
    from mqr.confidence import estimate_depth_confidences
    path, seq, io, ds, Side = capture
    bad = int(ds.timestamps[9])
    (path / "left_depth_confidence" / f"{bad}.npz").mkdir(parents=True)
    estimate_depth_confidences(io, _config(skip=False), sides=[Side.LEFT])
    out = capsys.readouterr().out
    assert f"[Error] build_and_save_confidence_map failed for LEFT frame 9 (timestamp {bad}): [Errno 21]" in out
    conf_dir = path / "left_depth_confidence"
    assert len(list(conf_dir.glob("*.npz"))) == N  # N - 1 files and the directory named like the 10th
    assert io.load_confidence_map(Side.LEFT, int(ds.timestamps[10])) is not None
