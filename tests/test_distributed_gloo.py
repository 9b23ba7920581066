"""world_size-2 gloo test of the multi-GPU merge logic (union of keys + one sum-reduce + unpack).

The volume is a numpy stand-in exposing the same pack/unpack pointer interface as
mqr.vbg.VoxelBlockGrid, so the torch.distributed code path of mqr.distributed runs unchanged."""
import ctypes
import os
import socket

import numpy as np
import pytest

R = 4
R3 = R ** 3


class NumpyVolume:
    block_resolution = R
    device_id = 0
    on_device = False

    def __init__(self, blocks):
        self.blocks = {tuple(k): (t.copy(), w.copy()) for k, (t, w) in blocks.items()}

    def export_keys(self):
        return np.array(sorted(self.blocks), np.int32).reshape(-1, 3)

    @staticmethod
    def _view(p, shape, ctype):
        return np.ctypeslib.as_array(ctypes.cast(ctypes.c_void_p(p), ctypes.POINTER(ctype)), shape=shape)

    def pack_weighted(self, keys_ptr, U, out_ptr):
        keys = self._view(keys_ptr, (U, 3), ctypes.c_int32)
        out = self._view(out_ptr, (U, R3, 2), ctypes.c_float)
        for i, k in enumerate(map(tuple, keys)):
            t, w = self.blocks.get(k, (np.zeros(R3, np.float32), np.zeros(R3, np.float32)))
            out[i, :, 0] = w * t
            out[i, :, 1] = w

    def unpack_weighted(self, keys_ptr, U, in_ptr):
        keys = self._view(keys_ptr, (U, 3), ctypes.c_int32)
        src = self._view(in_ptr, (U, R3, 2), ctypes.c_float)
        for i, k in enumerate(map(tuple, keys)):
            s, w = src[i, :, 0], src[i, :, 1]
            self.blocks[k] = (np.where(w > 0, s / np.where(w > 0, w, 1), 0).astype(np.float32), w.copy())


def _make(rank):
    rng = np.random.default_rng(rank)
    keys = [[(0, 0, 0), (1, 0, 0)], [(1, 0, 0), (0, -1, 2)], [(1, 0, 0), (5, 5, -5), (0, 0, 0)]][rank]
    return {k: (rng.uniform(-1, 1, R3).astype(np.float32), rng.integers(0, 5, R3).astype(np.float32))
            for k in keys}


def _worker(rank, world, port, q, method="reduce"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mqr.distributed import merge_to_root, shard_range, union_keys
        vol = NumpyVolume(_make(rank))
        u = union_keys(vol.export_keys())
        U = merge_to_root(vol, root=0, method=method)
        q.put((rank, len(u), U, {k: (t.tolist(), w.tolist()) for k, (t, w) in vol.blocks.items()},
               shard_range(10, rank, world)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_merge_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == 3 and res[0][2] == 3
    assert res[0][4] == (0, 5) and res[1][4] == (5, 10)
    a, b = _make(0), _make(1)
    merged = res[0][3]
    assert set(merged) == {(0, 0, 0), (1, 0, 0), (0, -1, 2)}
    t0, w0 = a[(1, 0, 0)]
    t1, w1 = b[(1, 0, 0)]
    w = w0 + w1
    want = np.where(w > 0, (w0 * t0 + w1 * t1) / np.where(w > 0, w, 1), 0)
    got_t, got_w = map(np.asarray, merged[(1, 0, 0)])
    assert np.array_equal(got_w, w)
    assert np.abs(got_t - want).max() < 1e-6
    # non-root keeps its own partial volume
    assert set(res[1][3]) == {(1, 0, 0), (0, -1, 2)}


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_merge_gloo(world):
    """all-to-all to the union-slice owners + gather to root == the dense reduce (uneven slices at 3)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "sparse")) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = [_make(r) for r in range(world)]
    keys = set().union(*parts)
    assert res[0][2] == len(keys)
    merged = res[0][3]
    assert set(merged) == keys
    for k in keys:
        ws = [p[k][1] for p in parts if k in p]
        ts = [p[k][0] for p in parts if k in p]
        w = np.sum(ws, axis=0)
        want = np.where(w > 0, np.sum([a * b for a, b in zip(ws, ts)], axis=0) / np.where(w > 0, w, 1), 0)
        got_t, got_w = map(np.asarray, merged[k])
        assert np.array_equal(got_w, w)
        assert np.abs(got_t - want).max() < 1e-6
    for r in range(1, world):  # non-root ranks keep their partial volumes
        assert set(res[r][3]) == set(parts[r])
