"""Multi-GPU merge in libmqr (mqr_reduce_rccl / mqr_merge_local / mqr_xchg_*) on one device.

The exchange of mqr_reduce_rccl (per-rank plan, send segments packed by k_gather_blocks, receive
segments merged in rank order through recv_dst) runs here over two other transports:
* mqr_merge_local -- the n volumes of one process, device copies between the ranks' own send and
  receive buffers; every sender / receiver pair's segment lists are checked entry for entry;
* merge_staged (mqr_xchg_*) -- one PROCESS per rank (2, 3 and 8 processes sharing the GPU), the
  segments carried over gloo through host buffers, each process planning on its own.
Only the ncclSend / ncclRecv call itself is not exercised on a one-GPU box (RCCL refuses two ranks
on one device).

* root mode: N frame shards merged into one volume == one sequential pass (identical keys and
  weights, |dtsdf| <= 1e-4; voxels one shard saw alone are that shard's values bit for bit);
* sharded mode: every rank's owned slice + one-block halo; the shard meshes (owned cubes only)
  concatenate to exactly the merged volume's mesh (same triangle set, counts add up);
* RCCL itself at world size 1 (one GPU on the test box); world size 2 over RCCL when >= 2 GPUs
  are visible (skipped otherwise -- the driver's 8-GPU node runs bench.py --gpus N).
"""
import os

import numpy as np
import pytest

import oracle
from gpu_helpers import canon_triangles, canon_vertices, compare_meshes, compare_volumes

pytestmark = pytest.mark.gpu

TOL = 1e-4


@pytest.fixture(scope="module")
def seq():
    from mqr import _lib, synthetic
    _lib.load()
    return synthetic.make_sequence("room", n=36, height=240, width=320, f=262.5, noise=True, seed=12)


def _shards(seq, world, R=16, vs=0.01, ranks=None):
    from mqr.distributed import shard_range
    from mqr.vbg import VoxelBlockGrid
    vols = []
    n = len(seq["K"])
    for r in (range(world) if ranks is None else ranks):
        lo, hi = shard_range(n, r, world)
        v = VoxelBlockGrid(voxel_size=vs, block_resolution=R, block_count=64)
        v.integrate_frames(seq["depth"][lo:hi], seq["K"][lo:hi], seq["T_wc"][lo:hi], depth_scale=1.0,
                           depth_max=4.0, trunc_voxel_multiplier=10.0)
        vols.append(v)
    return vols


def _oracle(seq, R=16, vs=0.01):
    ref = oracle.OracleVBG(vs, R, 256)
    for i in range(len(seq["K"])):
        ref.integrate_frame(seq["depth"][i], seq["K"][i].astype(np.float64), seq["T_wc"][i].astype(np.float64),
                            1.0, 4.0, 10.0)
    return ref


@pytest.mark.parametrize("world", [2, 3, 8])
def test_root_merge_matches_single_pass(seq, world):
    from mqr.distributed import merge_local
    vols = _shards(seq, world)
    res = merge_local(vols, mode="root", root=world - 1)
    merged, n_owned = res[world - 1]
    assert n_owned == merged.size()
    for r, (o, n) in enumerate(res):
        if r != world - 1:
            assert o.size() == 0 and n == 0
    err = compare_volumes(merged.export(), _oracle(seq).export(), TOL)
    assert err < 1e-5
    # a voxel that only the first shard saw keeps that shard's values exactly
    k0, t0, w0 = vols[0].export()
    km, tm, wm = merged.export()
    pos = {tuple(k): i for i, k in enumerate(km)}
    others = [dict(zip(map(tuple, v.export()[0]), v.export()[2])) for v in vols[1:]]
    for b in range(len(k0)):
        wo = sum(o[tuple(k0[b])] if tuple(k0[b]) in o else 0 for o in others)
        alone = (w0[b] > 0) & (np.asarray(wo) == 0)
        j = pos[tuple(k0[b])]
        assert np.array_equal(tm[j][alone], t0[b][alone]) and np.array_equal(wm[j][alone], w0[b][alone])


@pytest.mark.parametrize("world,R", [(2, 16), (3, 16), (4, 8), (8, 16)])
def test_sharded_meshes_concatenate_to_the_merged_mesh(seq, world, R):
    from mqr.distributed import extract_mesh_owned, merge_local
    vols = _shards(seq, world, R=R)
    root = merge_local(vols, mode="root", root=0)[0][0]
    full = root.extract_triangle_mesh(weight_threshold=1.5)
    shards = merge_local(vols, mode="sharded")
    owned_keys = []
    verts, tris, nt = [], [], 0
    off = 0
    for out, n_owned in shards:
        k = out.export()[0]
        owned_keys.append(k[:n_owned])
        m = extract_mesh_owned(out, n_owned, 1.5)
        verts.append(m.vertices)
        tris.append(m.triangles + off)
        off += len(m.vertices)
        nt += len(m.triangles)
    allk = np.concatenate(owned_keys)
    assert len(allk) == root.size() and len(np.unique(allk, axis=0)) == len(allk)  # owned slices partition U
    assert nt == len(full.triangles) > 1000
    V, T = np.concatenate(verts), np.concatenate(tris)
    assert np.array_equal(canon_triangles(V, T), canon_triangles(full.vertices, full.triangles))
    assert np.array_equal(canon_vertices(np.unique(V, axis=0))[0], canon_vertices(np.unique(full.vertices, axis=0))[0])
    # the halo makes each shard's owned blocks identical to the merged volume's
    rk, rt, rw = root.export()
    rpos = {tuple(k): i for i, k in enumerate(rk)}
    for out, n_owned in shards:
        k, t, w = out.export()
        for b in range(n_owned):
            j = rpos[tuple(k[b])]
            assert np.array_equal(t[b], rt[j]) and np.array_equal(w[b], rw[j])


@pytest.mark.parametrize("world,mode", [(2, "sharded"), (3, "root"), (8, "sharded"), (8, "root")])
def test_fused_merge_equals_per_source_merge(seq, world, mode):
    """The fused merge (one pass per output block, entries folded in rank order) against the round-5 merge
    (one pass over the output per source rank, mqr_merge_set_per_source): every rank's output, bit for bit."""
    from mqr.distributed import merge_local, set_merge_per_source
    vols = _shards(seq, world)
    fused = [(o.export(), n) for o, n in merge_local(vols, mode=mode)]
    set_merge_per_source(True)
    try:
        per_src = [(o.export(), n) for o, n in merge_local(vols, mode=mode)]
    finally:
        set_merge_per_source(False)
    assert len(fused) == len(per_src)
    for (a, na), (b, nb) in zip(fused, per_src):
        assert na == nb
        for x, y in zip(a, b):  # both outputs are activated in plan order: same buffer order
            assert np.array_equal(x, y)


def test_rccl_world_one(seq):
    """mqr_reduce_rccl through a real RCCL communicator (world size 1: the send to self)."""
    from mqr.distributed import RcclComm, merge_rccl
    vol = _shards(seq, 1)[0]
    comm = RcclComm(0, 0, 1, RcclComm.unique_id())
    try:
        out, n = merge_rccl(vol, comm, mode="root")
        assert n == vol.size() == out.size()
        assert compare_volumes(out.export(), vol.export(), 0.0) == 0.0
        out2, n2 = merge_rccl(vol, comm, mode="sharded", out=out)  # reuse: the output is emptied first
        assert n2 == vol.size()
        a = vol.extract_triangle_mesh(1.5)
        from mqr.distributed import extract_mesh_owned
        b = extract_mesh_owned(out2, n2, 1.5)
        compare_meshes(b.vertices, b.triangles, a.vertices, a.triangles)
        ph = comm.timing()
        assert all(v >= 0.0 for v in ph.values()), ph
        # `out` aliasing `local` would empty the volume before it is sent: refused, volume intact
        before = vol.export()
        with pytest.raises(RuntimeError, match="different volume"):
            merge_rccl(vol, comm, mode="root", out=vol)
        assert compare_volumes(vol.export(), before, 0.0) == 0.0
    finally:
        comm.close()


def test_segment_format_follows_the_weight_bounds(seq):
    """Segments carry uint16 weights when every rank's weights are integers <= 65535 (integrated volumes)
    and float32 pairs otherwise (an imported volume's weights are unknown); the RCCL path at world size 1
    reports the format in its counts, and the merged volume is the same either way."""
    from mqr.distributed import RcclComm, merge_rccl
    from mqr.vbg import VoxelBlockGrid
    vol = _shards(seq, 1)[0]
    R3 = 16 ** 3
    comm = RcclComm(0, 0, 1, RcclComm.unique_id())
    try:
        out, _ = merge_rccl(vol, comm, mode="root")
        assert comm.counts()["bytes_per_block"] == 6 * R3  # uint16 weights
        a = out.export()
        imp = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
        imp.import_blocks(*vol.export())
        out2, _ = merge_rccl(imp, comm, mode="root")
        assert comm.counts()["bytes_per_block"] == 8 * R3  # float32 pairs
        assert compare_volumes(out2.export(), a, 0.0) == 0.0
        assert compare_volumes(a, vol.export(), 0.0) == 0.0
    finally:
        comm.close()


@pytest.mark.parametrize("world,mode", [(3, "sharded"), (8, "root")])
def test_uint16_weight_segments_equal_float32_segments(seq, world, mode):
    """merge_local with uint16-weight segments (the default for integrated volumes) against float32 pairs
    (mqr_merge_set_per_source bit 1), fused and per-source merges: every output bit for bit."""
    from mqr.distributed import merge_local, set_merge_per_source
    vols = _shards(seq, world)
    outs = {}
    try:
        for per_source in (False, True):
            for f32 in (False, True):
                set_merge_per_source(per_source, f32)
                outs[(per_source, f32)] = [(o.export(), n) for o, n in merge_local(vols, mode=mode)]
    finally:
        set_merge_per_source(False, False)
    ref = outs[(False, False)]
    for key, got in outs.items():
        for (a, na), (b, nb) in zip(ref, got):
            assert na == nb, key
            for x, y in zip(a, b):
                assert np.array_equal(x, y), key


def _rccl_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mqr import synthetic
        from mqr.distributed import extract_mesh_owned, make_comm, merge_rccl, shard_range
        from mqr.vbg import VoxelBlockGrid
        torch.cuda.set_device(rank)
        s = synthetic.make_sequence("room", n=36, height=240, width=320, f=262.5, noise=True, seed=12)
        lo, hi = shard_range(36, rank, world)
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64, device=rank)
        v.integrate_frames(s["depth"][lo:hi], s["K"][lo:hi], s["T_wc"][lo:hi], depth_scale=1.0, depth_max=4.0,
                           trunc_voxel_multiplier=10.0)
        comm = make_comm(rank)
        out, n = merge_rccl(v, comm, mode="sharded")
        m = extract_mesh_owned(out, n, 1.5)
        got = [None] * world
        dist.all_gather_object(got, (m.vertices, m.triangles))
        comm.close()
        q.put((rank, got if rank == 0 else None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_two_gpus(seq):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (RCCL cannot put two ranks on one device)")
    import socket
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rccl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    assert not isinstance(res[1], str), res[1]
    got = res[0]
    assert not isinstance(got, str), got
    from mqr.distributed import merge_local
    full = merge_local(_shards(seq, 2), mode="root")[0][0].extract_triangle_mesh(1.5)
    off, V, T = 0, [], []
    for v, t in got:
        V.append(v)
        T.append(t + off)
        off += len(v)
    V, T = np.concatenate(V), np.concatenate(T)
    assert np.array_equal(canon_triangles(V, T), canon_triangles(full.vertices, full.triangles))


# ---------------------------------------------------------------- one process per rank (gloo-carried)
def _staged_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mqr import synthetic
        from mqr.distributed import extract_mesh_owned, merge_staged
        vol = _shards(synthetic.make_sequence("room", n=36, height=240, width=320, f=262.5, noise=True, seed=12),
                      world, ranks=[rank])[0]
        root = world - 1
        out, n_root = merge_staged(vol, mode="root", root=root)
        res = {"root": out.export() if rank == root else None, "n_root": n_root, "size_root": out.size()}
        out2, n = merge_staged(vol, mode="sharded", out=out)  # the output volume is reused (emptied first)
        m = extract_mesh_owned(out2, n, 1.5)
        k, t, w = out2.export()
        res.update(owned=(k[:n], t[:n], w[:n]), mesh=(m.vertices, m.triangles))
        q.put((rank, res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, repr(e) + "\n" + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_staged_processes_match_local_twin_and_single_pass(seq, world):
    """`world` processes on the one GPU, each integrating its frame shard and running the exchange
    on its own (plan, send segments, rank-ordered merge); segments over gloo.  The root volume is
    bit-identical to the one-process twin's and within 1e-4 of the single pass; the shard meshes
    concatenate to the merged mesh; owned blocks equal the merged volume's."""
    import socket
    import torch.multiprocessing as mp
    from mqr.distributed import merge_local
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_staged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in ps)
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    twin = merge_local(_shards(seq, world), mode="root", root=world - 1)[world - 1][0]
    tk, tt, tw = twin.export()
    rk, rt, rw = res[world - 1]["root"]
    assert res[world - 1]["n_root"] == len(rk) == len(tk)
    for r in range(world - 1):
        assert res[r]["n_root"] == 0 and res[r]["size_root"] == 0
    assert np.array_equal(rk, tk) and np.array_equal(rt, tt) and np.array_equal(rw, tw)  # same order, same bits
    assert compare_volumes((rk, rt, rw), _oracle(seq).export(), TOL) < 1e-5
    full = twin.extract_triangle_mesh(1.5)
    off, V, T, K = 0, [], [], []
    rpos = {tuple(k): i for i, k in enumerate(rk)}
    for r in range(world):
        v, t = res[r]["mesh"]
        V.append(v)
        T.append(t + off)
        off += len(v)
        k, ot, ow = res[r]["owned"]
        K.append(k)
        for b in range(len(k)):
            j = rpos[tuple(k[b])]
            assert np.array_equal(ot[b], rt[j]) and np.array_equal(ow[b], rw[j])
    allk = np.concatenate(K)
    assert len(allk) == len(rk) and len(np.unique(allk, axis=0)) == len(allk)
    V, T = np.concatenate(V), np.concatenate(T)
    assert len(T) == len(full.triangles) > 1000
    assert np.array_equal(canon_triangles(V, T), canon_triangles(full.vertices, full.triangles))


def test_xchg_create_checks_the_callers_key_row(seq):
    """mqr_xchg_create refuses (status 4) a gathered-keys row that is not the rank's own keys in buffer
    order padded with 0xFF..FF: the plan's send lists index the local pool through it."""
    import ctypes
    from mqr import _lib
    from mqr.distributed import MERGE_MODES, _empty_like, _packed
    vols = _shards(seq, 2)
    mine = _packed(vols[0].export_keys())
    other = _packed(vols[1].export_keys())
    mx = max(len(mine), len(other)) + 3
    out = _empty_like(vols[0])

    def create(row0):
        allk = np.full(2 * mx, -1, np.int64)
        allk[:len(row0)] = row0
        allk[mx:mx + len(other)] = other
        h = ctypes.c_void_p()
        rc = _lib.load().mqr_xchg_create(vols[0].handle, 2, 0, MERGE_MODES["root"], 0, _lib.ptr(allk), mx,
                                          _lib.MQR_HOST, out.handle, ctypes.byref(h))
        if h.value:
            _lib.load().mqr_xchg_destroy(h)
        return rc

    assert create(mine) == 0
    assert create(mine[::-1].copy()) == 4                           # another order
    assert create(mine[:-1]) == 4                                   # a key missing (padding in its place)
    assert create(np.concatenate([mine, other[:1]])) == 4          # a foreign key in the padding
    assert "not this rank's" in _lib.load().mqr_last_error().decode()


def test_rccl_merge_right_after_device_frame_integrate(seq):
    """integrate_frames on device frames returns with its last integrate running; mqr_reduce_rccl issued at
    once overlaps its all-gathers and plan with it and waits only before the send gather: the merged volume
    (world size 1: the volume itself) is the oracle's."""
    import ctypes
    import torch
    from mqr.distributed import RcclComm, merge_rccl
    from mqr.vbg import VoxelBlockGrid

    class _Dev:
        def __init__(self, t):
            self.ptr = ctypes.c_void_p(t.data_ptr())

    d = torch.from_numpy(np.ascontiguousarray(seq["depth"], np.float32)).cuda()
    torch.cuda.synchronize()
    B, H, W = d.shape
    comm = RcclComm(0, 0, 1, RcclComm.unique_id())
    try:
        vol = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
        out = None
        for _ in range(2):  # twice: the second merge follows a reset and re-integration of the same volume
            vol.reset()
            vol.integrate_frames((_Dev(d), B, H, W), seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64),
                                 depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
            out, n = merge_rccl(vol, comm, mode="root", out=out)
            assert compare_volumes(out.export(), _oracle(seq).export(), 0.0) == 0.0
    finally:
        comm.close()
