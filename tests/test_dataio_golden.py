"""mqr's DataIO / models / decode restatement vs outputs of the reference code (golden fixtures)."""
import os

import numpy as np
import pandas as pd
import pytest

from mqr.dataio import DepthDataIO
from mqr.depth_utils import convert_depth_to_linear, encode_linear_to_ndc
from mqr.models import CoordinateSystem, Side
from mqr.o3d_utils import compute_o3d_intrinsic_matrices


@pytest.fixture(scope="module")
def decode(golden_dir):
    return np.load(os.path.join(golden_dir, "decode_golden.npz"))


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "confidence_golden.npz"))


def test_decode_matches_reference(decode):
    raw, params, lin = decode["raw"], decode["params"], decode["linear"]
    for p, (near, far) in enumerate(params):
        for i in range(raw.shape[0]):
            got = convert_depth_to_linear(raw[i], float(near), float(far))
            assert got.dtype == np.float32
            assert np.array_equal(got, lin[p, i], equal_nan=True)


def test_validity_rule_matches_reference(decode):
    got = [DepthDataIO.is_depth_map_valid(r) for r in decode["raw"]]
    assert got == list(decode["valid"])


def test_ndc_encode_roundtrip():
    z = np.array([[0.0, 0.1, 0.5, 1.0, 3.999, 4.0]], np.float32)
    back = convert_depth_to_linear(encode_linear_to_ndc(z, 0.1, np.inf), 0.1, np.inf)
    assert back[0, 0] == 0.0
    assert np.allclose(back[0, 1:], z[0, 1:], rtol=2e-5)


def _write_capture_from_fixture(tmp, g, name):
    cols = [str(c) for c in g[f"{name}_descriptor_cols"]]
    df = pd.DataFrame(g[f"{name}_descriptor"], columns=cols)
    for c in ("timestamp_ms", "width", "height"):
        df[c] = df[c].astype(np.int64)
    ddir = tmp / "left_depth"
    ddir.mkdir(parents=True)
    for ts, raw in zip(df["timestamp_ms"], g[f"{name}_raw"]):
        raw.astype("<f4").tofile(ddir / f"{ts}.raw")
    df.to_csv(tmp / "left_depth_descriptors.csv", index=False)


@pytest.mark.parametrize("name", ["sphere", "room"])
def test_dataset_intrinsics_and_poses_match_reference(tmp_path, golden, name):
    _write_capture_from_fixture(tmp_path, golden, name)
    io = DepthDataIO(tmp_path)
    ds = io.build_depth_dataset(Side.LEFT)
    assert np.array_equal(ds.fx, golden[f"{name}_fx"]) and np.array_equal(ds.cx, golden[f"{name}_cx"])
    K = compute_o3d_intrinsic_matrices(ds)
    assert K.dtype == np.float32 and np.array_equal(K, golden[f"{name}_K"])
    o3d = ds.transforms.convert_coordinate_system(CoordinateSystem.OPEN3D, is_camera=True)
    assert np.array_equal(o3d.extrinsics_cw, golden[f"{name}_T_cw"])
    assert np.array_equal(o3d.extrinsics_wc, golden[f"{name}_T_wc"])
    assert np.array_equal(np.linalg.inv(o3d.extrinsics_cw), golden[f"{name}_T_cw_inv"])
    depths = np.stack([io.load_depth_map_by_index(Side.LEFT, ds, i) for i in range(len(ds))])
    assert np.array_equal(depths, golden[f"{name}_depth"])
    # dataset cache round trip (npz, allow_pickle=False like the reference)
    p = tmp_path / "dataset" / "left_depth_dataset.npz"
    ds.save(p)
    ds2 = type(ds).load(p)
    assert np.array_equal(ds2.timestamps, ds.timestamps) and ds2.transforms.coordinate_system == CoordinateSystem.UNITY


def test_missing_and_invalid_frames_are_dropped(tmp_path, golden):
    _write_capture_from_fixture(tmp_path, golden, "sphere")
    files = sorted((tmp_path / "left_depth").glob("*.raw"))
    files[2].unlink()                                   # missing file
    np.zeros((120, 160), "<f4").tofile(files[5])        # all-zero buffer -> invalid
    ds = DepthDataIO(tmp_path).build_depth_dataset(Side.LEFT)
    assert len(ds) == 10


def test_confidence_map_io(tmp_path):
    from mqr.models import ConfidenceMap
    io = DepthDataIO(tmp_path)
    cm = ConfidenceMap(np.random.default_rng(0).random((4, 5)), np.arange(20, dtype=np.int32).reshape(4, 5))
    io.save_confidence_map(Side.LEFT, 123, cm)
    back = io.load_confidence_map(Side.LEFT, 123)
    assert np.array_equal(back.confidence_map, cm.confidence_map) and back.valid_count.dtype == np.int32
    assert io.load_confidence_map(Side.LEFT, 124) is None
    assert io.exists_depth_confidence_map_dir(Side.LEFT)
