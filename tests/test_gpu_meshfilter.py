"""filter_mesh_components on the device (row f3) vs the CPU restatement (oracle/meshfilter_ref.py):
identical vertices, normals, triangles and statistics, bit for bit."""
import numpy as np
import pytest

import meshfilter_ref as mf
from test_oracle_meshfilter import T as T_KAT, V as V_KAT

pytestmark = pytest.mark.gpu


def _cmp(gpu, ref):
    pv, pn, pt, pst = gpu
    rv, rn, rt, rst = ref
    assert np.array_equal(pt, rt)
    assert np.array_equal(pv.view(np.uint32), rv.view(np.uint32))
    if rn is not None:
        assert np.array_equal(pn.view(np.uint32), rn.view(np.uint32))
    for k, val in rst.items():
        assert pst[k] == val, (k, pst[k], val)


@pytest.mark.parametrize("min_count", [1, 2, 100])
def test_known_answer_mesh(min_count):
    from mqr.meshfilter import filter_mesh_components_gpu
    _cmp(filter_mesh_components_gpu(V_KAT, None, T_KAT, min_count), mf.filter_mesh_components(V_KAT, None, T_KAT,
                                                                                             min_count))


@pytest.fixture(scope="module")
def room_mesh():
    from mqr import synthetic
    from mqr.vbg import VoxelBlockGrid
    seq = synthetic.make_sequence("room", n=16, height=120, width=160, f=131.25, noise=True, seed=43)
    v = VoxelBlockGrid(voxel_size=0.02, block_resolution=8, block_count=512)
    v.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0,
                       trunc_voxel_multiplier=6.0)
    m = v.extract_triangle_mesh(weight_threshold=1.0)
    return m.vertices.copy(), m.vertex_normals.copy(), m.triangles.copy()


@pytest.mark.parametrize("min_count", [1, 50, 2000, 10 ** 9])
def test_extracted_mesh_matches_oracle(room_mesh, min_count):
    from mqr.meshfilter import filter_mesh_components_gpu
    V, N, T = room_mesh
    assert T.shape[0] > 5000
    ref = mf.filter_mesh_components(V, N, T, min_count)
    assert ref[3]["clusters"] > 1  # noisy depth leaves floaters
    _cmp(filter_mesh_components_gpu(V, N, T, min_count), ref)


def test_stress_duplicates_nan_and_shuffled(room_mesh):
    from mqr.meshfilter import filter_mesh_components_gpu
    V, N, T = room_mesh
    rng = np.random.default_rng(0)
    T2 = np.concatenate([T, T[rng.integers(0, len(T), 500)][:, [1, 2, 0]], T[:50][:, [0, 0, 1]]])
    T2 = T2[rng.permutation(len(T2))]
    V2 = V.copy()
    V2[rng.integers(0, len(V), 20)] = np.nan
    V2[rng.integers(0, len(V), 20)] = V2[rng.integers(0, len(V), 20)]  # coincident vertices
    ref = mf.filter_mesh_components(V2, N, T2, 30)
    _cmp(filter_mesh_components_gpu(V2, N, T2, 30), ref)


def test_dropin_messages_and_empty(capsys):
    from mqr.geometry import TriangleMesh
    from mqr.meshfilter import filter_mesh_components
    out = filter_mesh_components(TriangleMesh(V_KAT, np.zeros_like(V_KAT), T_KAT), 2)
    txt = capsys.readouterr().out
    assert "Found 3 connected component(s)" in txt and "Removed 1 small component(s) with < 2" in txt
    assert "Final mesh has 4 triangles (was 8)" in txt
    assert out.triangles.shape == (4, 3)
    empty = TriangleMesh(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32), np.zeros((0, 3), np.int32))
    assert filter_mesh_components(empty) is empty
    assert "no triangles" in capsys.readouterr().out
