"""Row a10: the confidence driver ``mqr.confidence.estimate_depth_confidences`` end to end on a
capture in the reference's layout (estimate_depth_confidences.py:82-153), every written npz
compared with the CPU oracle's build_confidence_map restatement (pinned by the reference's golden
vectors, tests/test_oracle_golden.py).

Covers: the dir-level skip (``skip_if_output_dir_exists``), an existing per-frame file kept as is
(resume rule :94-96), a frame missing / invalid after the dataset was cached (no output for it,
skipped as a neighbour), reference-frame chunks that cross the 64-frame REF_CHUNK boundary and
windows clipped at both ends of the sequence.
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


def test_driver_outputs_match_oracle(capture):
    from mqr.confidence import REF_CHUNK, estimate_depth_confidences
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
