"""The drop-in boundary end to end: mqr.o3d_utils.integrate(dataset, depth_data_io, side, ...)
(reference o3d_utils.py:153-238) on a capture written in the reference's layout, with native file
reads (mqr_read_frames) and device ingestion (raw files -> mqr_decode_depth -> batched touch/integrate),
against the CPU oracle fed by the numpy decode path frame by frame.  Covers missing files, invalid
buffers, confidence masking, missing confidence maps (warned only for valid frames) and the Python
readers (MQR_NATIVE_IO=0).  Bit-identical volumes."""
import numpy as np
import pytest

import oracle  # the test-only checker (tests/conftest.py puts oracle/ on the path)

pytestmark = pytest.mark.gpu


def _capture(tmp_path, n=14, seed=31):
    from mqr import synthetic
    from mqr.dataio import DepthDataIO
    from mqr.models import ConfidenceMap, Side
    seq = synthetic.make_sequence("room", n=n, height=240, width=320, f=262.5, noise=True, seed=seed)
    synthetic.write_capture(tmp_path, seq)
    io = DepthDataIO(tmp_path)
    ds = io.build_depth_dataset(Side.LEFT)
    assert len(ds) == n
    rng = np.random.default_rng(seed)
    for i, ts in enumerate(ds.timestamps):
        if i in (6, 9):
            continue  # no confidence map: warn (6) and integrate unmasked; 9 is invalid, so no warning
        conf = rng.random((240, 320))
        vc = rng.integers(0, 8, (240, 320)).astype(np.int32)
        io.save_confidence_map(Side.LEFT, int(ts), ConfidenceMap(conf, vc))
    files = sorted((tmp_path / "left_depth").glob("*.raw"))
    files[3].unlink()                                 # missing after the dataset was built
    np.ones((240, 320), "<f4").tofile(files[9])       # all-one buffer: invalid, dropped
    return io, ds, Side


@pytest.mark.parametrize("native_io", [True, False])
@pytest.mark.parametrize("chunk", [4, 127])
@pytest.mark.parametrize("use_conf", [False, True])
def test_integrate_dropin_matches_oracle(tmp_path, use_conf, chunk, native_io, capsys, monkeypatch):
    """chunk 4: several hand-offs, so both alternating host staging sets are reused (and the missing
    file / invalid buffer / missing confidence map land in different chunks)."""
    from gpu_helpers import compare_volumes
    from mqr import o3d_utils
    from mqr.o3d_utils import _masked_depth, compute_o3d_intrinsic_matrices, integrate
    monkeypatch.setattr(o3d_utils, "CHUNK", chunk)
    if not native_io:
        monkeypatch.setenv("MQR_NATIVE_IO", "0")
    io, ds, Side = _capture(tmp_path)
    kw = dict(use_confidence_filtered_depth=use_conf, confidence_threshold=0.2, valid_count_threshold=2)
    vbg = integrate(ds, io, Side.LEFT, voxel_size=0.01, block_resolution=16, block_count=500, depth_max=4.0,
                    trunc_voxel_multiplier=10.0, device="CUDA:0", **kw)
    out = capsys.readouterr().out
    # the reference reads a frame's confidence map only after its depth map passed is_depth_map_valid
    assert out.count("[Warning] Confidence map not found") == (1 if use_conf else 0)
    ref = oracle.OracleVBG(0.01, 16, 256)
    K = compute_o3d_intrinsic_matrices(ds).astype(np.float64)
    T = ds.transforms.extrinsics_wc.astype(np.float64)
    used = 0
    for i in range(len(ds)):
        d = _masked_depth(io, Side.LEFT, i, ds, **kw)
        if d is None:
            continue
        ref.integrate_frame(d, K[i], T[i], 1.0, 4.0, 10.0)
        used += 1
    assert used == len(ds) - 2
    capsys.readouterr()
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0


def test_integrate_dropin_chains_volumes(tmp_path):
    """vbg_opt chaining (reconstruct_scene.py:65-81): a second call continues the same volume."""
    from gpu_helpers import compare_volumes
    from mqr.o3d_utils import integrate
    io, ds, Side = _capture(tmp_path, n=10, seed=5)
    kw = dict(use_confidence_filtered_depth=False, confidence_threshold=0.0, valid_count_threshold=0,
              voxel_size=0.01, block_resolution=8, block_count=100, depth_max=4.0, trunc_voxel_multiplier=10.0,
              device=0)
    a = integrate(ds[list(range(5))], io, Side.LEFT, **kw)
    a = integrate(ds[list(range(5, 10))], io, Side.LEFT, vbg_opt=a, **kw)
    b = integrate(ds, io, Side.LEFT, **kw)
    assert compare_volumes(a.export(), b.export(), 0.0) == 0.0


@pytest.mark.parametrize("chunk", [4, 127])
def test_integrate_dropin_ragged_frame_sizes(tmp_path, chunk, monkeypatch):
    """Frames of different sizes in one capture (the descriptor CSV gives each frame's width and
    height, depth_data_io.py:187-188): runs of one size go to the device in dataset order, and the
    volume equals frame-by-frame integration.  chunk 4 mixes one-size chunks (staged path) with a
    chunk that spans both sizes (list path)."""
    import pandas as pd
    from gpu_helpers import compare_volumes
    from mqr import synthetic
    from mqr.dataio import DepthDataIO
    from mqr.models import Side
    from mqr import o3d_utils
    from mqr.o3d_utils import _masked_depth, compute_o3d_intrinsic_matrices, integrate
    monkeypatch.setattr(o3d_utils, "CHUNK", chunk)
    parts = [("a", 240, 320, 262.5, 1_000_000, 5), ("b", 120, 160, 131.25, 2_000_000, 4),
             ("c", 240, 320, 262.5, 3_000_000, 3)]
    frames = []
    for name, h, w, f, t0, n in parts:
        seq = synthetic.make_sequence("room", n=n, height=h, width=w, f=f, noise=True, seed=len(frames) + 3)
        synthetic.write_capture(tmp_path / name, seq, t0=t0)
        frames.append(pd.read_csv(tmp_path / name / "left_depth_descriptors.csv"))
        (tmp_path / "left_depth").mkdir(exist_ok=True)
        for raw in (tmp_path / name / "left_depth").glob("*.raw"):
            raw.rename(tmp_path / "left_depth" / raw.name)
    pd.concat(frames).to_csv(tmp_path / "left_depth_descriptors.csv", index=False)
    io = DepthDataIO(tmp_path)
    ds = io.build_depth_dataset(Side.LEFT)
    assert len(ds) == 12 and len(set(zip(ds.widths, ds.heights))) == 2
    kw = dict(use_confidence_filtered_depth=False, confidence_threshold=0.0, valid_count_threshold=0)
    vbg = integrate(ds, io, Side.LEFT, voxel_size=0.01, block_resolution=16, block_count=300, depth_max=4.0,
                    trunc_voxel_multiplier=10.0, device="CUDA:0", **kw)
    ref = oracle.OracleVBG(0.01, 16, 256)
    K = compute_o3d_intrinsic_matrices(ds).astype(np.float64)
    T = ds.transforms.extrinsics_wc.astype(np.float64)
    for i in range(len(ds)):
        d = _masked_depth(io, Side.LEFT, i, ds, **kw)
        assert d is not None and d.shape == (ds.heights[i], ds.widths[i])
        ref.integrate_frame(d, K[i], T[i], 1.0, 4.0, 10.0)
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0


@pytest.mark.parametrize("native_io", [True, False])
@pytest.mark.parametrize("chunk", [4, 127])
def test_integrate_dropin_failure_prefix(tmp_path, chunk, native_io, capsys, monkeypatch):
    """A frame whose read raises mid-chunk (a raw file of the wrong size: the reference's
    np.fromfile(...).reshape raises ValueError, depth_data_io.py:46): the exception leaves integrate()
    with every earlier frame integrated and nothing of it or after it, and only the earlier frames'
    messages printed -- the reference's per-frame loop (o3d_utils.py:188-236).  Frame 6 (after the
    failing frame 5) has no confidence map: its warning must not appear."""
    from gpu_helpers import compare_volumes
    from mqr import o3d_utils
    from mqr.o3d_utils import _masked_depth, compute_o3d_intrinsic_matrices, integrate
    from mqr.vbg import VoxelBlockGrid
    monkeypatch.setattr(o3d_utils, "CHUNK", chunk)
    if not native_io:
        monkeypatch.setenv("MQR_NATIVE_IO", "0")
    io, ds, Side = _capture(tmp_path)
    files = sorted((tmp_path / "left_depth").glob("*.raw"))
    fail = 5
    np.zeros(240 * 320 + 7, "<f4").tofile(files[fail - 1])  # files[3] was deleted: index fail - 1 is frame 5
    assert ds.timestamps[fail] == int(files[fail - 1].stem)
    kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.2, valid_count_threshold=2)
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=500, device=0)
    capsys.readouterr()
    with pytest.raises(ValueError):
        integrate(ds, io, Side.LEFT, voxel_size=0.01, block_resolution=16, block_count=500, depth_max=4.0,
                  trunc_voxel_multiplier=10.0, device="CUDA:0", vbg_opt=vbg, **kw)
    assert "Confidence map not found" not in capsys.readouterr().out
    ref = oracle.OracleVBG(0.01, 16, 256)
    K = compute_o3d_intrinsic_matrices(ds).astype(np.float64)
    T = ds.transforms.extrinsics_wc.astype(np.float64)
    used = 0
    for i in range(fail):
        d = _masked_depth(io, Side.LEFT, i, ds, **kw)
        if d is not None:
            ref.integrate_frame(d, K[i], T[i], 1.0, 4.0, 10.0)
            used += 1
    assert used == fail - 1  # frame 3 is missing
    assert vbg.size() > 0
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0
