"""The drop-in functions called with a DataIO shaped like the reference's own (scripts/dataio/depth_data_io.py:
a `depth_path_config` with get_depth_map_path / get_depth_confidence_map_path, loaders and savers of its
own, no load_raw_depth): `integrate()` must read the frames through the path config (native reader) and
`estimate_depth_confidences()` must write to the config's paths, with results identical to those made
through this package's DepthDataIO -- and identical again with the Python readers (MQR_NATIVE_IO=0)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _PathConfig:
    """The two path methods of the reference's DepthPathConfig (config/project_path_config.py:148-161)."""

    def __init__(self, paths):
        self._p = paths

    def get_depth_map_path(self, side, timestamp):
        return self._p.depth_map_path(side, timestamp)

    def get_depth_confidence_map_path(self, side, timestamp):
        return self._p.confidence_path(side, timestamp)


class _RefShapedIO:
    """Duck type of the reference's DepthDataIO: the methods its callers use, delegating to this
    package's implementation, and `depth_path_config` -- but no load_raw_depth."""

    def __init__(self, io):
        self._io = io
        self.depth_path_config = _PathConfig(io.paths)

    def load_depth_dataset(self, side, use_cache=True):
        return self._io.load_depth_dataset(side)

    def exists_depth_confidence_map_dir(self, side):
        return self._io.exists_depth_confidence_map_dir(side)

    def load_depth_map(self, side, timestamp, width, height, near, far):
        return self._io.load_depth_map(side, timestamp, width, height, near, far)

    def load_depth_map_by_index(self, side, dataset, index):
        return self._io.load_depth_map_by_index(side, dataset, index)

    def load_confidence_map(self, side, timestamp):
        return self._io.load_confidence_map(side, timestamp)

    def save_confidence_map(self, side, timestamp, confidence_map):
        return self._io.save_confidence_map(side, timestamp, confidence_map)


def _capture(path, n=40):
    from mqr import synthetic
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    seq = synthetic.make_sequence("room", n=n, height=120, width=160, f=131.25, noise=True, seed=8)
    synthetic.write_capture(path, seq)
    io = DepthDataIO(path)
    ds = io.load_depth_dataset(Side.LEFT)
    return io, ds, Side


@pytest.mark.parametrize("native_io", [True, False])
def test_reference_shaped_dataio(tmp_path, native_io, monkeypatch):
    from gpu_helpers import compare_volumes
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.models import CoordinateSystem
    from mqr.o3d_utils import _frame_paths, integrate
    if not native_io:
        monkeypatch.setenv("MQR_NATIVE_IO", "0")
    a, b = tmp_path / "a", tmp_path / "b"
    io_a, ds_a, Side = _capture(a)
    io_b, ds_b, _ = _capture(b)
    ref_b = _RefShapedIO(io_b)
    assert (_frame_paths(ref_b, Side.LEFT) is not None) == native_io
    cfg = DepthConfidenceEstimationConfig(target_frame_range=5, depth_max=4.0, error_threshold=0.08,
                                          skip_if_output_dir_exists=False)
    estimate_depth_confidences(io_a, cfg, sides=[Side.LEFT])
    estimate_depth_confidences(ref_b, cfg, sides=[Side.LEFT])
    for ts in ds_a.timestamps:
        ca, cb = io_a.load_confidence_map(Side.LEFT, int(ts)), DepthDataIO(b).load_confidence_map(Side.LEFT, int(ts))
        assert (ca is None) == (cb is None)
        if ca is not None:
            assert np.array_equal(ca.confidence_map, cb.confidence_map) and np.array_equal(ca.valid_count, cb.valid_count)
    kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2, voxel_size=0.01,
              block_resolution=16, block_count=800, depth_max=4.0, trunc_voxel_multiplier=10.0, device=0)
    for ds in (ds_a, ds_b):
        ds.transforms = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                                is_camera=True)
    va = integrate(ds_a, io_a, Side.LEFT, **kw)
    vb = integrate(ds_b, ref_b, Side.LEFT, **kw)
    assert compare_volumes(va.export(), vb.export(), 0.0) == 0.0
