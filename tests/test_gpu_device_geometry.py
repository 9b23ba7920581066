"""Device-resident geometry (mqr.geometry DeviceGeom / DeviceArray, mqr_geom_device_ptrs): extraction
results stay in HBM as Open3D's tensor geometry does on a CUDA device (reference reconstruct_scene.py:
105-122, 186-198: extract -> filter_mesh_components -> RaycastingScene -> colour), and the chain
extract -> filter -> ray cast -> colour run on them in place must give exactly what the host-array
calls give.  Also: lazy host copies, .cpu(), pickling, and the lifetime of the device arrays."""
import pickle

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def volume():
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=12, height=240, width=320, f=262.5, noise=True, seed=41)
    vbg = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=2000, device="CUDA:0")
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    return vbg, seq


def test_extraction_stays_in_hbm_until_host_access(volume):
    vbg, _ = volume
    mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
    pos = mesh.vertex.positions
    assert pos.is_cuda and mesh.triangle.indices.is_cuda and pos.dtype == np.float32
    n = pos.shape[0]
    assert n > 1000 and pos.is_cuda  # shape without a copy
    v = mesh.vertices  # first host access copies
    assert isinstance(v, np.ndarray) and v.shape == (n, 3)
    assert mesh.cpu().vertex.positions.is_cuda is False
    back = pickle.loads(pickle.dumps(mesh.vertex.positions))
    assert np.array_equal(back.numpy(), v)
    pcd = vbg.extract_point_cloud(3.0)
    assert pcd.point.positions.is_cuda and pcd.points.shape == (pcd.point.positions.shape[0], 3)


def test_filter_cast_colour_in_place_equal_host_arrays(volume):
    from mqr.color import color_map, project_vertex_colors
    from mqr.geometry import TriangleMesh
    from mqr.meshfilter import filter_mesh_components
    from mqr.raycasting import RaycastingScene
    vbg, seq = volume
    mesh = vbg.extract_triangle_mesh(weight_threshold=1.5)
    host = TriangleMesh(mesh.vertices.copy(), mesh.vertex_normals.copy(), mesh.triangles.copy(), device="CUDA:0")
    fd = filter_mesh_components(mesh, 500)
    fh = filter_mesh_components(host, 500)
    assert fd.vertex.positions.is_cuda and not fh.vertex.positions.is_cuda
    assert np.array_equal(fd.vertices, fh.vertices) and np.array_equal(fd.triangles, fh.triangles)
    assert np.array_equal(fd.vertex_normals, fh.vertex_normals)
    K = seq["K"][:4].astype(np.float64)
    T = seq["T_wc"][:4].astype(np.float64)
    H, W = 240, 320
    imgs = np.random.default_rng(1).integers(0, 256, (4, H, W, 3), np.uint8)
    sd, sh = RaycastingScene(device=0), RaycastingScene(device=0)
    sd.add_triangles(fd)
    sh.add_triangles(fh.vertices, fh.triangles)
    td = sd.cast_pinhole(K, T, W, H)["t_hit"]
    th = sh.cast_pinhole(K, T, W, H)["t_hit"]
    assert td.is_cuda and np.array_equal(td.numpy(), th.numpy())
    cd, nd = color_map(fd.vertex.positions, imgs, td, K, T)          # vertices and depths in HBM
    ch, nh = color_map(fh.vertices, imgs, th.numpy(), K, T)          # host arrays
    assert np.array_equal(cd, ch) and np.array_equal(nd, nh)
    pd, qd = project_vertex_colors(fd, imgs, K, T)
    ph, qh = project_vertex_colors(fh, imgs, K, T)
    assert np.array_equal(pd, ch) and np.array_equal(ph, ch) and np.array_equal(qd, nh) and np.array_equal(qh, nh)


def test_device_arrays_outlive_the_volume_and_each_other():
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=4, height=120, width=160, f=131.25, noise=False, seed=2)
    vbg = VoxelBlockGrid(voxel_size=0.02, block_resolution=16, block_count=500, device="CUDA:0")
    vbg.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                         trunc_voxel_multiplier=10.0)
    meshes = [vbg.extract_triangle_mesh(1.5) for _ in range(3)]
    ref = meshes[0].vertices.copy()
    del vbg
    pos = meshes[1].vertex.positions
    del meshes[1]
    assert np.array_equal(pos.numpy(), ref) and np.array_equal(meshes[-1].vertices, ref)
