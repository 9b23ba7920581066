"""GPU parity: libmqr_hip.so (through the C ABI) vs the CPU oracle on the same seeded inputs.

Bar (north star): identical touched-block sets and integer weights, TSDF within 1e-4 on w>0
voxels (bit-exact in practice: both sides compile without FP contraction), identical
marching-cubes vertex/triangle sets.
"""
import numpy as np
import pytest

import oracle
from gpu_helpers import compare_meshes, compare_points_normals, compare_volumes

pytestmark = pytest.mark.gpu

TOL = 1e-4  # voxel TSDF tolerance from BASELINE.json north_star


@pytest.fixture(scope="module")
def mqr_mod():
    from mqr import _lib
    _lib.load()
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    import mqr.vbg
    return mqr.vbg


@pytest.fixture(scope="module")
def sphere_seq():
    from mqr import synthetic
    return synthetic.make_sequence("sphere", n=8, height=120, width=160, f=131.25, noise=True, seed=11)


@pytest.fixture(scope="module")
def room_seq():
    from mqr import synthetic
    return synthetic.make_sequence("room", n=40, height=240, width=320, f=262.5, noise=True, seed=12)


def _oracle_run(seq, vs, R, dmax, tm, frames=None):
    ref = oracle.OracleVBG(vs, R, 256)
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)
    for i in (range(len(K)) if frames is None else frames):
        ref.integrate_frame(seq["depth"][i], K[i], T[i], 1.0, dmax, tm)
    return ref


def test_touch_matches_oracle(mqr_mod, room_seq):
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=128)
    K = room_seq["K"].astype(np.float64)
    T = room_seq["T_wc"].astype(np.float64)
    for i in (0, 7, 23):
        g = vbg.compute_unique_block_coordinates(room_seq["depth"][i], K[i], T[i], 1.0, 4.0, 10.0).numpy()
        o = oracle.touch(room_seq["depth"][i], K[i], T[i], 0.01, 16, 1.0, 4.0, 10.0)
        assert len(g) == len(np.unique(g, axis=0))
        assert np.array_equal(np.unique(g, axis=0), np.unique(o, axis=0))
    assert vbg.size() == 0  # touch does not allocate (Open3D uses a separate frustum map)


@pytest.mark.parametrize("scene,vs,R,dmax,tm", [("sphere", 0.02, 16, 3.0, 4.0), ("sphere", 0.01, 8, 3.0, 8.0),
                                                ("room", 0.01, 16, 4.0, 10.0)])
def test_integrate_frames_matches_oracle(mqr_mod, sphere_seq, room_seq, scene, vs, R, dmax, tm):
    seq = sphere_seq if scene == "sphere" else room_seq
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=vs, block_resolution=R, block_count=16)  # forces pool growth
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=dmax,
                         trunc_voxel_multiplier=tm)
    ref = _oracle_run(seq, vs, R, dmax, tm)
    err = compare_volumes(vbg.export(), ref.export(), TOL)
    assert err == 0.0, f"expected bit-exact TSDF, got {err}"


def test_per_frame_api_equals_batched(mqr_mod, room_seq):
    K = room_seq["K"].astype(np.float64)
    T = room_seq["T_wc"].astype(np.float64)
    a = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
    for i in range(12):
        keys = a.compute_unique_block_coordinates(room_seq["depth"][i], K[i], T[i], 1.0, 4.0, 10.0)
        a.integrate(keys, room_seq["depth"][i], K[i], T[i], 1.0, 4.0, 10.0)
    b = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
    b.integrate_frames(room_seq["depth"][:12], K[:12], T[:12], depth_scale=1.0, depth_max=4.0,
                       trunc_voxel_multiplier=10.0)
    assert compare_volumes(a.export(), b.export(), 0.0) == 0.0


def test_skipped_frames_and_empty_frame_error(mqr_mod, sphere_seq):
    K = sphere_seq["K"].astype(np.float64)
    T = sphere_seq["T_wc"].astype(np.float64)
    ok = np.array([1, 0, 1, 1, 0, 1, 1, 1], np.uint8)
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
    vbg.integrate_frames(sphere_seq["depth"], K, T, frame_ok=ok, depth_scale=1.0, depth_max=3.0,
                         trunc_voxel_multiplier=4.0)
    ref = _oracle_run(sphere_seq, 0.02, 16, 3.0, 4.0, frames=np.nonzero(ok)[0])
    compare_volumes(vbg.export(), ref.export(), 0.0)
    empty = np.zeros_like(sphere_seq["depth"][:1])
    with pytest.raises(RuntimeError, match="No block is touched"):
        vbg.integrate_frames(empty, K[:1], T[:1], depth_scale=1.0, depth_max=3.0, trunc_voxel_multiplier=4.0)


# R = 16 / 8: bit-row kernels (k_mc_count / k_mc_emit); R = 12: runtime-R per-voxel kernels
@pytest.mark.parametrize("R,thr", [(16, 0.0), (16, 1.5), (16, 3.0), (8, 1.5), (8, 0.0), (12, 1.5)])
def test_mesh_matches_oracle(mqr_mod, room_seq, R, thr):
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=R, block_count=512)
    vbg.integrate_frames(room_seq["depth"], room_seq["K"], room_seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    ref = _oracle_run(room_seq, 0.01, R, 4.0, 10.0)
    mesh = vbg.extract_triangle_mesh(weight_threshold=thr)
    ov, on, ot = ref.extract_mesh(thr)
    assert len(ot) > 1000
    compare_meshes(mesh.vertices, mesh.triangles, ov, ot, pos_tol=0.0)
    compare_points_normals(mesh.vertices, mesh.vertex_normals, ov, on, 1e-6)


@pytest.mark.parametrize("thr", [0.0, 3.0])
def test_points_match_oracle(mqr_mod, room_seq, thr):
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=512)
    vbg.integrate_frames(room_seq["depth"], room_seq["K"], room_seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    ref = _oracle_run(room_seq, 0.01, 16, 4.0, 10.0)
    pcd = vbg.extract_point_cloud(weight_threshold=thr)
    op, on = ref.extract_points(thr)
    assert pcd.point.positions.shape[0] == op.shape[0] > 100
    compare_points_normals(pcd.points, pcd.normals, op, on, 1e-6)


def test_repeated_extraction_speculative_capacity(mqr_mod, room_seq):
    """The second and later extractions of a volume emit into buffers sized from the previous
    extraction's counts without waiting for the totals: a mesh / point cloud that grew past that
    capacity (2 frames, then 40) is re-emitted into exact buffers, one that fits (same volume again,
    a higher threshold) is kept.  Every result equals the oracle."""
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=512)
    args = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    vbg.integrate_frames(room_seq["depth"][:1], room_seq["K"][:1], room_seq["T_wc"][:1], **args)
    small = vbg.extract_triangle_mesh(weight_threshold=0.0)
    small_p = vbg.extract_point_cloud(weight_threshold=0.0)
    vbg.integrate_frames(room_seq["depth"][1:], room_seq["K"][1:], room_seq["T_wc"][1:], **args)
    cap = lambda n: n + n // 4 + 4096  # extract.hip spec_cap
    ref = _oracle_run(room_seq, 0.01, 16, 4.0, 10.0)
    for i, thr in enumerate((0.0, 0.0, 3.0)):  # grown past the hint, then equal, then smaller
        mesh = vbg.extract_triangle_mesh(weight_threshold=thr)
        ov, on, ot = ref.extract_mesh(thr)
        if i == 0:
            assert len(ot) > cap(len(small.triangles)), "the re-emission path is not exercised"
        compare_meshes(mesh.vertices, mesh.triangles, ov, ot, pos_tol=0.0)
        compare_points_normals(mesh.vertices, mesh.vertex_normals, ov, on, 1e-6)
        pcd = vbg.extract_point_cloud(weight_threshold=thr)
        op, onn = ref.extract_points(thr)
        if i == 0:
            assert op.shape[0] > cap(small_p.point.positions.shape[0]), "the re-emission path is not exercised"
        compare_points_normals(pcd.points, pcd.normals, op, onn, 1e-6)


def test_save_load_roundtrip(mqr_mod, sphere_seq, tmp_path):
    vbg = mqr_mod.VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
    vbg.integrate_frames(sphere_seq["depth"], sphere_seq["K"], sphere_seq["T_wc"], depth_scale=1.0, depth_max=3.0,
                         trunc_voxel_multiplier=4.0)
    p = tmp_path / "colorless_vbg.npz"
    vbg.save(str(p))
    d = np.load(p)
    assert set(d.files) >= {"voxel_size", "block_resolution", "key", "tsdf", "weight"}
    assert d["tsdf"].shape[1:] == (16, 16, 16, 1)
    vbg2 = mqr_mod.VoxelBlockGrid.load(str(p))
    compare_volumes(vbg.export(), vbg2.export(), 0.0)
    m1 = vbg.extract_triangle_mesh(1.5)
    m2 = vbg2.extract_triangle_mesh(1.5)
    compare_meshes(m1.vertices, m1.triangles, m2.vertices, m2.triangles)


def test_sharded_merge_matches_single_pass(mqr_mod, room_seq):
    """N-way frame split merged by the multi-GPU pack/reduce/unpack code path (the reduce done
    on the host here), vs one sequential pass: same keys and weights, tsdf within 1e-4."""
    from mqr import _lib
    from mqr.distributed import shard_range
    n = len(room_seq["K"])
    full = _oracle_run(room_seq, 0.01, 16, 4.0, 10.0)
    for world in (2, 3):
        vols = []
        for r in range(world):
            lo, hi = shard_range(n, r, world)
            v = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
            v.integrate_frames(room_seq["depth"][lo:hi], room_seq["K"][lo:hi], room_seq["T_wc"][lo:hi],
                               depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
            vols.append(v)
        union = np.unique(np.concatenate([v.export_keys() for v in vols]), axis=0).astype(np.int32)
        U = len(union)
        dkeys = _lib.DeviceBuffer.from_array(union)
        total = np.zeros((U, 4096, 2), np.float32)
        for v in vols:
            buf = _lib.DeviceBuffer(total.nbytes)
            v.pack_weighted(dkeys.ptr.value, U, buf.ptr.value)
            total += buf.to_array(total.shape, np.float32)
        merged = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
        dsum = _lib.DeviceBuffer.from_array(total)
        merged.unpack_weighted(dkeys.ptr.value, U, dsum.ptr.value)
        err = compare_volumes(merged.export(), full.export(), TOL)
        assert err < 1e-5


def test_speculative_first_batch_gate(mqr_mod, room_seq):
    """The first batch of a call is integrated right behind its touch, gated on the device by the
    touch's counters (k_gate).  A volume that has integrated before (so the gate path is taken) gives
    the same volume with the speculative head on and off (variant bit 18); a first batch whose pool
    overflows (capacity 1 block) or holds a frame that touches nothing falls back to the ordinary path:
    the result equals the oracle's and the error is raised as upstream does."""
    from mqr import _lib
    K = room_seq["K"].astype(np.float64)
    T = room_seq["T_wc"].astype(np.float64)
    d = room_seq["depth"]
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    vols = []
    for variant in (0, 0x40000):
        v = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=4096)
        _lib.call("mqr_vbg_set_variant", v.handle, variant)
        v.integrate_frames(d[:4], K[:4], T[:4], **kw)  # sets the speculative grid estimate
        v.reset()
        v.integrate_frames(d, K, T, **kw)
        vols.append(v)
    assert compare_volumes(vols[0].export(), vols[1].export(), 0.0) == 0.0
    ref = _oracle_run(room_seq, 0.01, 16, 4.0, 10.0)
    compare_volumes(vols[0].export(), ref.export(), 0.0)
    # pool overflow inside the speculative first batch: capacity 1 block
    small = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=1)
    small.integrate_frames(d[:1], K[:1], T[:1], **kw)
    small.reset()
    small.integrate_frames(d, K, T, **kw)
    compare_volumes(small.export(), ref.export(), 0.0)
    # a frame that touches nothing inside the first batch: frames before it integrated, then the error
    dd = d.copy()
    dd[3] = 0.0
    vols[0].reset()
    with pytest.raises(RuntimeError, match="No block is touched"):
        vols[0].integrate_frames(dd, K, T, **kw)
    compare_volumes(vols[0].export(), _oracle_run(room_seq, 0.01, 16, 4.0, 10.0, frames=[0, 1, 2]).export(), 0.0)


def test_released_grid_is_reused_as_a_new_one(mqr_mod, room_seq):
    """A released grid of the same configuration is handed to the next VoxelBlockGrid (mqr.vbg SPARE_GRIDS):
    it must come back empty, with the default integrate configuration, and integrate exactly as a new grid;
    a grid that grew is not kept."""
    from mqr import vbg as vbg_mod
    from mqr import _lib
    vbg_mod.release_spare_grids()
    K = room_seq["K"].astype(np.float64)
    T = room_seq["T_wc"].astype(np.float64)
    kw = dict(depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    a = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=4096)
    _lib.call("mqr_vbg_set_variant", a.handle, 0x400)  # 32-frame batches: must not carry over
    a.integrate_frames(room_seq["depth"][:20], K[:20], T[:20], **kw)
    ref = a.export()
    h = a.handle.value
    del a
    b = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=4096)
    assert b.handle.value == h and b.size() == 0  # the released grid, emptied
    b.integrate_frames(room_seq["depth"][:20], K[:20], T[:20], **kw)
    assert compare_volumes(b.export(), ref, 0.0) == 0.0
    c = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=4096)
    assert c.handle.value != h  # (b still alive: a new grid)
    del b, c
    g = mqr_mod.VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=16)  # grows past 16 blocks
    g.integrate_frames(room_seq["depth"][:20], K[:20], T[:20], **kw)
    vbg_mod.release_spare_grids()
    del g
    assert not vbg_mod._spares  # grown: destroyed, not kept
    vbg_mod.release_spare_grids()
