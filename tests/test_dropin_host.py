"""Host logic of the drop-in integrate() (mqr.o3d_utils.integrate, reference o3d_utils.py:153-238)
without a GPU: the device decode and the volume are replaced by recorders, the file reads are the
real ones (native mqr_read_frames_masked and the Python readers).  What is checked is which frames
reach the volume, in which order, and what is printed -- in particular the reference's failure
prefix: a frame whose read raises leaves every earlier frame integrated, nothing of it or after it,
and only the earlier frames' messages printed (verdict r05 item 6).  The volume itself is checked
against the oracle by tests/test_gpu_pipeline.py."""
import numpy as np
import pytest


class _Vol:
    device_id = 0

    def __init__(self, extrinsics):
        self.T = extrinsics
        self.frames = []

    def integrate_frames(self, depths, K, T, frame_ok=None, **kw):
        B = len(T)
        ok = np.ones(B, bool) if frame_ok is None else np.asarray(frame_ok, bool)
        for j in range(B):
            if ok[j]:
                i = int(np.flatnonzero((self.T == T[j].astype(self.T.dtype)).all(axis=(1, 2)))[0])
                self.frames.append(i)


class _Buf:
    def __init__(self, nbytes, device=0):
        self.ptr = 0

    def free(self):
        pass


@pytest.fixture()
def fakes(monkeypatch):
    from mqr import _lib, ingest
    from mqr.dataio import DepthDataIO

    def decode(raw, nears, fars, **kw):
        raw = raw if not isinstance(raw, tuple) else None
        return None, np.array([DepthDataIO.is_depth_map_valid(r) for r in raw], bool)

    monkeypatch.setattr(ingest, "decode_depth_frames", decode)
    monkeypatch.setattr(_lib, "DeviceBuffer", _Buf)


def _capture(tmp_path, n=14, seed=31):
    from mqr import synthetic
    from mqr.dataio import DepthDataIO
    from mqr.models import ConfidenceMap, Side
    seq = synthetic.make_sequence("sphere", n=n, height=24, width=32, f=26.25, noise=True, seed=seed)
    synthetic.write_capture(tmp_path, seq)
    io = DepthDataIO(tmp_path)
    ds = io.build_depth_dataset(Side.LEFT)
    for i, ts in enumerate(ds.timestamps):
        if i not in (6, 9):
            io.save_confidence_map(Side.LEFT, int(ts), ConfidenceMap(np.ones((24, 32)), np.ones((24, 32), np.int32)))
    files = sorted((tmp_path / "left_depth").glob("*.raw"))
    files[3].unlink()                                 # missing: skipped
    np.ones((24, 32), "<f4").tofile(files[9])         # invalid: dropped, no confidence message
    return io, ds, Side, files


def _run(tmp_path, capsys, monkeypatch, chunk, native_io, fail=None):
    from mqr import o3d_utils
    monkeypatch.setattr(o3d_utils, "CHUNK", chunk)
    monkeypatch.setenv("MQR_NATIVE_IO", "1" if native_io else "0")
    io, ds, Side, files = _capture(tmp_path)
    if fail is not None:
        f = [p for p in files if p.exists() and int(p.stem) == ds.timestamps[fail]][0]
        np.zeros(24 * 32 + 5, "<f4").tofile(f)        # wrong size: the reference's reshape raises ValueError
    vol = _Vol(ds.transforms.extrinsics_wc)
    capsys.readouterr()
    err = None
    try:
        o3d_utils.integrate(ds, io, Side.LEFT, use_confidence_filtered_depth=True, confidence_threshold=0.5,
                            valid_count_threshold=1, voxel_size=0.01, block_resolution=16, block_count=10,
                            depth_max=4.0, trunc_voxel_multiplier=10.0, device=0, vbg_opt=vol)
    except ValueError as e:
        err = e
    return vol.frames, capsys.readouterr().out, err


@pytest.mark.parametrize("native_io", [True, False])
@pytest.mark.parametrize("chunk", [4, 127])
def test_dropin_frames_and_messages(tmp_path, capsys, monkeypatch, fakes, chunk, native_io):
    frames, out, err = _run(tmp_path, capsys, monkeypatch, chunk, native_io)
    assert err is None
    assert frames == [i for i in range(14) if i not in (3, 9)]
    assert out.count("[Warning] Confidence map not found") == 1  # frame 6 (9 is invalid)


@pytest.mark.parametrize("native_io", [True, False])
@pytest.mark.parametrize("chunk", [4, 127])
@pytest.mark.parametrize("fail", [0, 5, 7, 13])
def test_dropin_failure_prefix(tmp_path, capsys, monkeypatch, fakes, chunk, native_io, fail):
    frames, out, err = _run(tmp_path, capsys, monkeypatch, chunk, native_io, fail=fail)
    assert isinstance(err, ValueError)
    assert frames == [i for i in range(fail) if i not in (3, 9)]
    assert out.count("[Warning] Confidence map not found") == (1 if fail > 6 else 0)


def test_native_paths_respect_subclass_overrides(tmp_path):
    """A subclass of the reference's DepthDataIO that overrides a loader or the saver at class level
    keeps its override: the native readers / writers are not used for it."""
    from mqr.confidence import _native_paths
    from mqr.o3d_utils import _frame_paths
    io, ds, Side, _ = _capture(tmp_path)

    class _Paths:
        def get_depth_map_path(self, side, timestamp):
            return io.paths.depth_map_path(side, timestamp)

        def get_depth_confidence_map_path(self, side, timestamp):
            return io.paths.confidence_path(side, timestamp)

    class DepthDataIO:  # the reference's class name (scripts/dataio/depth_data_io.py)
        def __init__(self):
            self.depth_path_config = _Paths()

        def load_depth_map(self, side, timestamp, width, height, near, far):
            return io.load_depth_map(side, timestamp, width, height, near, far)

        def load_depth_map_by_index(self, side, dataset, index):
            return io.load_depth_map_by_index(side, dataset, index)

        def is_depth_map_valid(self, depth_map):
            return io.is_depth_map_valid(depth_map)

        def load_confidence_map(self, side, timestamp):
            return io.load_confidence_map(side, timestamp)

        def save_confidence_map(self, side, timestamp, confidence_map):
            return io.save_confidence_map(side, timestamp, confidence_map)

    class Loads(DepthDataIO):
        def load_confidence_map(self, side, timestamp):
            return None

    class Saves(DepthDataIO):
        def save_confidence_map(self, side, timestamp, confidence_map):
            pass

    assert _frame_paths(DepthDataIO(), Side.LEFT) is not None
    assert _frame_paths(Loads(), Side.LEFT) is None
    assert _frame_paths(Saves(), Side.LEFT) is not None       # integrate() reads only
    assert _native_paths(DepthDataIO(), Side.LEFT, ds) is not None
    assert _native_paths(Saves(), Side.LEFT, ds) is None
    inst = DepthDataIO()
    inst.load_confidence_map = lambda side, timestamp: None   # replaced on the instance
    assert _frame_paths(inst, Side.LEFT) is None
