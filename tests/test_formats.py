"""On-disk formats: the PLY files the reference writes through
``o3d.io.write_point_cloud`` / ``write_triangle_mesh`` (``reconstruction_data_io.py:57-94``) and the
``colorless_vbg.npz`` of ``vbg.save`` / ``VoxelBlockGrid.load`` (``:42-55``).
Open3D is absent offline, so the layouts follow the recalled upstream writers (VERIFY): these tests
pin our writers against an independent reader, the header text and the App. A.7 key / dtype /
shape contract.  Parity against files Open3D itself produced is unpinned."""
import numpy as np
import pytest

from mqr import geometry


def _mesh(seed=0, nv=50, nt=80):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(nv, 3)).astype(np.float32)
    n = rng.normal(size=(nv, 3)).astype(np.float32)
    t = rng.integers(0, nv, size=(nt, 3)).astype(np.int32)
    return geometry.TriangleMesh(v, n, t)


def _header(path):
    data = open(path, "rb").read()
    return data[:data.index(b"end_header\n")].decode().splitlines()


def test_triangle_mesh_ply_layout_and_round_trip(tmp_path):
    m = _mesh()
    p = tmp_path / "mesh.ply"
    assert geometry.write_triangle_mesh(str(p), m)
    assert _header(p) == ["ply", "format binary_little_endian 1.0", "comment Created by Open3D", "element vertex 50",
                          "property double x", "property double y", "property double z",
                          "property double nx", "property double ny", "property double nz",
                          "element face 80", "property list uchar uint vertex_indices"]
    props, faces = geometry.read_ply(str(p))
    for i, k in enumerate("xyz"):
        assert props[k].dtype == np.float64
        assert np.array_equal(props[k], m.vertices[:, i].astype(np.float64))  # float32 -> float64 exact
        assert np.array_equal(props["n" + k], m.vertex_normals[:, i].astype(np.float64))
    assert np.array_equal(faces, m.triangles)
    back = geometry.read_triangle_mesh(str(p))
    assert np.array_equal(back.vertices, m.vertices) and np.array_equal(back.triangles, m.triangles)
    # exact file size: header + 48 B per vertex + 13 B per face
    assert p.stat().st_size == len(open(p, "rb").read().split(b"end_header\n")[0]) + 11 + 50 * 48 + 80 * 13


def test_point_cloud_ply_and_empty(tmp_path):
    rng = np.random.default_rng(1)
    pc = geometry.PointCloud(rng.normal(size=(7, 3)).astype(np.float32), rng.normal(size=(7, 3)).astype(np.float32))
    p = tmp_path / "pcd.ply"
    assert geometry.write_point_cloud(str(p), pc, write_ascii=False, compressed=True)
    props, faces = geometry.read_ply(str(p))
    assert faces is None and len(props["x"]) == 7
    assert np.array_equal(np.stack([props["x"], props["y"], props["z"]], 1), pc.points.astype(np.float64))
    empty = geometry.TriangleMesh(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32), np.zeros((0, 3), np.int32))
    q = tmp_path / "empty.ply"
    geometry.write_triangle_mesh(str(q), empty)
    props, faces = geometry.read_ply(str(q))
    assert len(props["x"]) == 0 and faces is not None and len(faces) == 0


def test_ply_rejects_bad_input(tmp_path):
    m = _mesh()
    bad = geometry.TriangleMesh(m.vertices, m.vertex_normals, np.array([[0, 1, 99]], np.int32))
    with pytest.raises(ValueError):
        geometry.write_triangle_mesh(str(tmp_path / "bad.ply"), bad)
    with pytest.raises(ValueError):
        geometry.write_triangle_mesh(str(tmp_path / "bad.obj"), m)
    with pytest.raises(NotImplementedError):
        geometry.write_triangle_mesh(str(tmp_path / "a.ply"), m, write_ascii=True)


@pytest.mark.gpu
def test_vbg_npz_app_a7_contract(tmp_path):
    """vbg.save writes exactly App. A.7's arrays (names, dtypes, shapes); load accepts a file laid out
    that way by hand, including extra metadata keys, and reproduces the volume bit for bit."""
    import torch  # initialise torch's HIP first
    assert torch.cuda.is_available()
    import oracle
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("sphere", n=6, height=120, width=160, f=131.25, noise=True, seed=2)
    ref = oracle.OracleVBG(0.02, 16, 64)
    for i in range(6):
        ref.integrate_frame(seq["depth"][i], seq["K"][i].astype(np.float64), seq["T_wc"][i].astype(np.float64),
                            1.0, 3.0, 4.0)
    keys, tsdf, wgt = ref.export()
    R = 16
    path = tmp_path / "colorless_vbg.npz"
    np.savez(path, voxel_size=np.array([0.02], np.float32), block_resolution=np.array([R], np.int64),
             key=keys.astype(np.int32), tsdf=tsdf.reshape(-1, R, R, R, 1), weight=wgt.reshape(-1, R, R, R, 1),
             some_metadata=np.array([1, 2, 3]))
    vbg = VoxelBlockGrid.load(str(path))
    assert vbg.voxel_size == np.float32(0.02) and vbg.block_resolution == R
    k2, t2, w2 = vbg.export()
    o = np.lexsort(keys.T[::-1])
    o2 = np.lexsort(k2.T[::-1])
    assert np.array_equal(keys[o], k2[o2])
    assert np.array_equal(tsdf.reshape(-1, R ** 3)[o], t2.reshape(-1, R ** 3)[o2])
    assert np.array_equal(wgt.reshape(-1, R ** 3)[o], w2.reshape(-1, R ** 3)[o2])
    out = tmp_path / "saved.npz"
    vbg.save(str(out))
    d = np.load(out, allow_pickle=False)
    assert sorted(d.files) == ["block_resolution", "key", "tsdf", "voxel_size", "weight"]
    assert d["voxel_size"].dtype == np.float32 and d["voxel_size"].shape == (1,)
    assert d["block_resolution"].dtype == np.int64 and d["block_resolution"].shape == (1,)
    assert d["key"].dtype == np.int32 and d["key"].shape == (len(keys), 3)
    for a in ("tsdf", "weight"):
        assert d[a].dtype == np.float32 and d[a].shape == (len(keys), R, R, R, 1)
