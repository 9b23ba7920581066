"""Parity at the BASELINE.json configurations' own sizes, GPU vs the CPU
oracle on the same inputs:

* C1: 32 x 640x480 procedural sphere, 2 cm voxels, R = 16, the 128^3 region (o3d_utils.py:153-238);
* C2: 500 x 640x480 procedural room walk, 5 mm voxels, R = 16, trunc 10, depth_max 4 m;
* C3: C2 + estimate_depth_confidences (r = 10, depth_max 4, err 0.08) -> mask (0.02 / 2) -> integrate
  (estimate_depth_confidences.py:15-79, o3d_utils.py:109-150);
* C4: 1000 LEFT + 1000 RIGHT frames (stereo baseline 0.064 m) chained into ONE volume, LEFT then
  RIGHT as two integrate calls (reconstruct_scene.py:64-81, vbg_opt threaded through);
* C5: 1000 + 1000 frames of the 8 x 8 x 3 m hall at 3 mm, 640x480, the volume grown from 4096
  blocks to ~10^5 (multi-GB pool growth), mesh at 1.5 and point cloud at 3.0.

Point clouds (extract_point_cloud, reconstruct_scene.py:90 / refine_fragment_poses.py:39, default
weight_threshold 3.0) are compared at C2, C4 and C5 sizes.  Config-size meshes and point clouds are
compared as exact multisets through 64-bit position hashes (gpu_helpers.compare_meshes_fast).

Bar (north_star): identical touched-block sets and weights, |dtsdf| <= 1e-4 on w > 0 voxels
(bit-exact in practice), identical marching-cubes vertex and triangle sets at the pipeline's mesh
threshold 1.5 and the point-cloud default 3.0.  The oracle itself is parity-unpinned against Open3D
(Open3D is absent offline); the confidence path is pinned by reference golden vectors.
"""
import numpy as np
import pytest

import oracle
from gpu_helpers import compare_meshes, compare_meshes_fast, compare_points_fast, compare_volumes

pytestmark = pytest.mark.gpu

TOL = 1e-4  # voxel TSDF tolerance, BASELINE.json north_star


@pytest.fixture(scope="module")
def vbg_mod():
    import torch  # initialise torch's HIP first: the in-process runtime then serves both
    assert torch.cuda.is_available()
    from mqr import _lib
    _lib.load()
    import mqr.vbg
    return mqr.vbg


def _oracle_volume(depth, K, T, vs, R, dmax, tm, block_count=4096):
    ref = oracle.OracleVBG(vs, R, block_count)
    K = np.asarray(K, np.float64)
    T = np.asarray(T, np.float64)
    for i in range(len(depth)):
        ref.integrate_frame(depth[i], K[i], T[i], 1.0, dmax, tm)
    return ref


def _check_mesh(vbg, ref, thr, fast=False):
    mesh = vbg.extract_triangle_mesh(weight_threshold=thr)
    ov, _, ot = ref.extract_mesh(thr)
    assert len(ot) > 1000
    if fast:
        compare_meshes_fast(mesh.vertices, mesh.triangles, ov, ot)
    else:
        compare_meshes(mesh.vertices, mesh.triangles, ov, ot, pos_tol=0.0)
    return len(ot)


def _check_points(vbg, ref, thr=3.0):
    """extract_point_cloud() at the reference's default threshold (reconstruct_scene.py:90)."""
    pcd = vbg.extract_point_cloud(weight_threshold=thr)
    op, on = ref.extract_points(thr)
    assert len(op) > 1000
    compare_points_fast(pcd.points, pcd.normals, op, on, tol=1e-6)
    return len(op)


def _integrate_sides(vbg, ref, sides, vs, dmax=4.0, tm=10.0):
    """reconstruct_scene.py:64-81: one integrate call per side into the same volume (vbg_opt),
    LEFT first; the oracle runs the same frames one by one."""
    for depth, K, T in sides:
        vbg.integrate_frames(depth, K, T, depth_scale=1.0, depth_max=dmax, trunc_voxel_multiplier=tm)
        K = np.asarray(K, np.float64)
        T = np.asarray(T, np.float64)
        for i in range(len(depth)):
            ref.integrate_frame(depth[i], K[i], T[i], 1.0, dmax, tm)


def test_c1_sphere_32_frames_2cm(vbg_mod):
    """C1: 32 frames 640x480 on a 1.5 m ring around a r = 0.5 m sphere, 2 cm voxels (128^3 = 512
    blocks of 16^3), noisy depth (sigma 0.002 z, 1 % dropout)."""
    from mqr import synthetic
    seq = synthetic.make_sequence("sphere", n=32, height=480, width=640, noise=True, seed=0)
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=512)
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    ref = _oracle_volume(seq["depth"], seq["K"], seq["T_wc"], 0.02, 16, 4.0, 10.0, 512)
    keys = vbg.export_keys()
    assert np.abs(keys).max() <= 4  # inside the 128^3 region around the sphere
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    for thr in (1.5, 3.0):
        _check_mesh(vbg, ref, thr)


@pytest.fixture(scope="module")
def c2_seq(vbg_mod):
    """The bench's C2 sequence (mqr.synthetic.make_sequence_fast, GPU ray cast) as host arrays."""
    from mqr import synthetic
    seq = synthetic.make_sequence_fast("room", n=500, height=480, width=640, seed=0, device="cuda:0")
    seq["depth"] = seq.pop("depth_t").cpu().numpy()
    return seq


@pytest.fixture(scope="module")
def c2_pair(vbg_mod, c2_seq):
    seq = c2_seq
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=4096)  # grows
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    ref = _oracle_volume(seq["depth"], seq["K"], seq["T_wc"], 0.005, 16, 4.0, 10.0, 8192)
    return vbg, ref


def test_c2_room_500_frames_5mm(c2_pair):
    vbg, ref = c2_pair
    assert ref.size() > 5000
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    n15 = _check_mesh(vbg, ref, 1.5)
    n30 = _check_mesh(vbg, ref, 3.0)
    assert n15 >= n30 > 1_000_000


def test_c2_point_cloud_threshold_3(c2_pair):
    """extract_point_cloud() with its default weight_threshold 3.0 on the C2 volume: the file
    reconstruct_scene.py:90-91 persists, and what the fragment path extracts."""
    vbg, ref = c2_pair
    assert _check_points(vbg, ref, 3.0) > 1_000_000


def test_c2_room_320x320(vbg_mod):
    """C2's second frame size (the Quest depth size is not recorded in the reference,
    so C2 also runs at 320 x 320): 500 frames, 5 mm, against the oracle."""
    from mqr import synthetic
    seq = synthetic.make_sequence_fast("room", n=500, height=320, width=320, f=262.5, seed=1, device="cuda:0")
    depth = seq.pop("depth_t").cpu().numpy()
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=4096)
    vbg.integrate_frames(depth, seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    ref = _oracle_volume(depth, seq["K"], seq["T_wc"], 0.005, 16, 4.0, 10.0, 8192)
    assert ref.size() > 3000
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    _check_mesh(vbg, ref, 1.5)


def test_c3_confidence_mask_integrate(vbg_mod, c2_seq):
    """C3: confidence of every frame (r = 10) on the GPU, checked against the oracle on ALL 500
    reference frames (the float32 prefilter decides ~99.6 % of the (pixel, neighbour) pairs: every
    frame's maps must stay bit-identical, not a sample); then the masked sequence integrates
    identically on both sides."""
    from mqr.confidence import confidence_maps
    seq = c2_seq
    depth, K, Tcw = seq["depth"], seq["K"], seq["T_cw"]
    Ti = np.linalg.inv(Tcw)
    conf, valid = confidence_maps(depth, K, Tcw, Ti, 0, len(depth), 10, 4.0, 0.08)
    bad = []
    for i in range(len(depth)):
        oc, ov = oracle.confidence(depth, K, Tcw, Ti, i, 10, 4.0, 0.08)
        if not (np.array_equal(valid[i], ov) and np.array_equal(conf[i], oc)):
            bad.append(i)
    assert not bad, f"confidence maps differ from the oracle at reference frames {bad[:20]}"
    masked = depth.copy()
    masked[conf < 0.02] = 0.0  # o3d_utils.py:141-142 with the pipeline's thresholds
    masked[valid < 2] = 0.0
    assert 0.01 < (masked == 0).mean() < 0.9
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=8192)
    vbg.integrate_frames(masked, K, seq["T_wc"], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
    ref = _oracle_volume(masked, K, seq["T_wc"], 0.005, 16, 4.0, 10.0, 8192)
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    _check_mesh(vbg, ref, 1.5)


def test_empty_frame_mid_batch(vbg_mod):
    """A frame that touches no block in the middle of a device batch: frames before it are
    integrated, nothing of it or after it is (Open3D raises at that frame's touch)."""
    from mqr import synthetic
    seq = synthetic.make_sequence("sphere", n=12, height=120, width=160, f=131.25, noise=True, seed=3)
    depth = seq["depth"].copy()
    depth[7] = 0.0
    K = seq["K"].astype(np.float64)
    T = seq["T_wc"].astype(np.float64)
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
    vbg.integrate_frames(depth[:3], K[:3], T[:3], depth_scale=1.0, depth_max=3.0, trunc_voxel_multiplier=4.0)
    with pytest.raises(RuntimeError, match="No block is touched"):
        vbg.integrate_frames(depth[3:], K[3:], T[3:], depth_scale=1.0, depth_max=3.0, trunc_voxel_multiplier=4.0)
    ref = _oracle_volume(depth[:7], K[:7], T[:7], 0.02, 16, 3.0, 4.0, 64)
    assert vbg.size() == ref.size()
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0
    # the volume stays usable: the remaining frames continue it exactly
    vbg.integrate_frames(depth[8:], K[8:], T[8:], depth_scale=1.0, depth_max=3.0, trunc_voxel_multiplier=4.0)
    for i in range(8, 12):
        ref.integrate_frame(depth[i], K[i], T[i], 1.0, 3.0, 4.0)
    assert compare_volumes(vbg.export(), ref.export(), 0.0) == 0.0


def test_empty_first_frame_of_batch(vbg_mod):
    from mqr import synthetic
    seq = synthetic.make_sequence("sphere", n=4, height=120, width=160, f=131.25, noise=False, seed=3)
    depth = seq["depth"].copy()
    depth[0] = 0.0
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=64)
    with pytest.raises(RuntimeError, match="No block is touched"):
        vbg.integrate_frames(depth, seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=3.0,
                             trunc_voxel_multiplier=4.0)
    assert vbg.size() == 0


def test_c5_structure_hall_3mm(vbg_mod):
    """C5's structure at test size: LEFT then RIGHT (stereo baseline 0.064 m) through the 8 x 8 x 3 m
    hall at 3 mm voxels, volume grown from a small capacity, mesh at 1.5 and per-vertex colour from
    keyframes with ray-cast colour-aligned depth -- all against the oracle."""
    from mqr import synthetic
    from mqr.color import color_map
    from mqr.raycasting import RaycastingScene
    left = synthetic.hall_loop_poses(24)
    right = [(R, t + R[:, 0] * 0.064) for R, t in left]
    seq = synthetic.make_sequence("hall", poses=left + right, height=240, width=320, f=262.5, noise=True, seed=8)
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.003, block_resolution=16, block_count=256)
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    ref = _oracle_volume(seq["depth"], seq["K"], seq["T_wc"], 0.003, 16, 4.0, 10.0, 256)
    assert ref.size() > 4 * 256  # grew several times
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    _check_mesh(vbg, ref, 1.5, fast=True)
    mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
    key = list(range(0, 48, 4))
    K = seq["K"][key].astype(np.float64)
    T = seq["T_wc"][key].astype(np.float64)
    poses = left + right
    imgs = np.stack([synthetic.render_color("hall", K[0], poses[i][0], poses[i][1], 240, 320) for i in key])
    rs = RaycastingScene()
    rs.add_triangles(mesh.vertices, mesh.triangles)
    depth = rs.cast_pinhole(K, T, 320, 240)["t_hit"].numpy()
    gc, gn = color_map(mesh.vertices, imgs, depth, K, T)
    oc, on = oracle.color_map(mesh.vertices, imgs, depth, K, T)
    assert np.array_equal(gn, on) and np.array_equal(gc, oc)
    # colour max depth 2.5 m in an 8 x 8 m hall: only the near walls and floor are coloured
    assert (gn > 0).mean() > 0.02


def _device_sides(seq, n_left):
    """The generated (GPU) sequence split into its LEFT and RIGHT halves as host arrays."""
    depth = seq.pop("depth_t").cpu().numpy()
    K, T = seq["K"], seq["T_wc"]
    return [(depth[:n_left], K[:n_left], T[:n_left]), (depth[n_left:], K[n_left:], T[n_left:])]


def test_c4_left_right_2000_frames_chained(vbg_mod):
    """C4 on one GPU: 1000 LEFT + 1000 RIGHT frames (0.064 m stereo baseline) of the room walk at
    5 mm, chained into one volume LEFT then RIGHT (reconstruct_scene.py:64-81)."""
    from mqr import synthetic
    left = synthetic.room_loop_poses(1000)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    seq = synthetic.make_sequence_fast("room", poses=left + right, height=480, width=640, seed=4, device="cuda:0")
    sides = _device_sides(seq, 1000)
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.005, block_resolution=16, block_count=4096)
    ref = oracle.OracleVBG(0.005, 16, 8192)
    _integrate_sides(vbg, ref, sides, 0.005)
    del sides
    assert ref.size() > 6000
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    assert _check_mesh(vbg, ref, 1.5, fast=True) > 1_500_000
    _check_points(vbg, ref, 3.0)


def test_c5_hall_1000_plus_1000_3mm(vbg_mod):
    """C5 at 1000 + 1000 frames of 640x480 through the 8 x 8 x 3 m hall at 3 mm voxels (R = 16),
    LEFT then RIGHT into one volume grown from 4096 blocks; volume, mesh at 1.5 and point cloud at
    3.0 against the oracle (the 4000-frame bench leg carries the same comparison)."""
    from mqr import synthetic
    left = synthetic.hall_loop_poses(1000)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    seq = synthetic.make_sequence_fast("hall", poses=left + right, height=480, width=640, seed=5, device="cuda:0")
    sides = _device_sides(seq, 1000)
    vbg = vbg_mod.VoxelBlockGrid(voxel_size=0.003, block_resolution=16, block_count=4096)
    ref = oracle.OracleVBG(0.003, 16, 4096)
    _integrate_sides(vbg, ref, sides, 0.003)
    del sides
    assert ref.size() > 20 * 4096  # the pool grew many times over
    assert compare_volumes(vbg.export(), ref.export(), TOL) == 0.0
    assert _check_mesh(vbg, ref, 1.5, fast=True) > 10_000_000
    _check_points(vbg, ref, 3.0)
