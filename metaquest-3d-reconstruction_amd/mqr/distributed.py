"""Frame-sharded fusion across the GPUs of one node.

One process per GPU (torchrun).  Each rank integrates a contiguous range of frames into its own
volume (frame order preserved inside the shard).  The single exchange step merges the partial
volumes exactly (up to fp32 rounding), because the reference's unit-weight running average is
``tsdf = sum(sdf_i) / n, weight = n``:

    1. all-gather the per-rank block counts and keys (int32 x3, ~12 B per block);
    2. every rank forms the identical sorted union key table;
    3. each rank packs (w * tsdf, w) float32 for the union blocks (zeros where absent) on device;
    4. ONE sum-reduce over RCCL (xGMI) into the root;
    5. the root unpacks: tsdf = sum(w*tsdf) / sum(w), weight = sum(w), and extracts.

Only step 4 moves volume data (U * R^3 * 8 bytes).  The collective calls go through
``torch.distributed`` (backend "nccl" is RCCL on ROCm; "gloo" for the CPU tests), everything
volumetric goes through libmqr_hip.so.

The production path is ``merge_rccl``: the whole exchange inside libmqr_hip.so (mqr_reduce_rccl,
RCCL resolved at run time, one sparse grouped send/recv of the blocks each rank owns or needs as
halo), with ``torch.distributed`` (any backend, gloo is enough) only handing the RCCL id around.
``merge_local`` runs the same plan and kernels for several volumes of one process (tests on one
GPU), and ``extract_mesh_owned`` extracts a shard's mesh (its owned cubes only).
"""
from __future__ import annotations

import numpy as np


def shard_range(n_frames: int, rank: int, world: int):
    """Contiguous frame range [lo, hi) of `rank` (the first n % world ranks get one more)."""
    base, extra = divmod(n_frames, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def confidence_shard(depths, intrinsics, T_cw, T_cw_inv, rank: int, world: int, target_frame_range=10,
                     depth_max=3.0, error_threshold=0.05, frame_ok=None, device=0):
    """This rank's share of the confidence maps (reference frames are independent):
    reference frames shard_range(n, rank, world), read with a +-r halo of neighbour frames; no
    collective.  The shards of all ranks concatenate, in rank order, to the single-GPU result.
    Returns (lo, hi, conf (hi-lo,H,W) f64, valid (hi-lo,H,W) i32)."""
    from .confidence import confidence_maps
    n = len(depths)
    lo, hi = shard_range(n, rank, world)
    if hi <= lo:
        H, W = np.shape(depths)[1:]
        return lo, hi, np.empty((0, H, W), np.float64), np.empty((0, H, W), np.int32)
    r = int(target_frame_range)
    a, b = max(0, lo - r), min(n, hi + r)  # the window the kernel reads; indices stay global through lo - a
    ok = None if frame_ok is None else np.asarray(frame_ok)[a:b]
    conf, valid = confidence_maps(np.asarray(depths)[a:b], np.asarray(intrinsics)[a:b], np.asarray(T_cw)[a:b],
                                  np.asarray(T_cw_inv)[a:b], lo - a, hi - a, r, depth_max, error_threshold, ok,
                                  device=device)
    return lo, hi, conf, valid


def union_keys(local_keys: np.ndarray, group=None, device=None) -> np.ndarray:
    """All-gather every rank's block keys; return the sorted (lexicographic) union, int32 (U,3)."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cpu")
    local = torch.as_tensor(np.ascontiguousarray(local_keys, dtype=np.int32).reshape(-1, 3), device=dev)
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(max(counts), 1)
    padded = torch.zeros((m, 3), dtype=torch.int32, device=dev)
    padded[: local.shape[0]] = local
    gathered = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(gathered, padded, group=group)
    allk = np.concatenate([g[:c].cpu().numpy() for g, c in zip(gathered, counts)], axis=0)
    if len(allk) == 0:
        return np.zeros((0, 3), np.int32)
    return _unpacked(np.unique(_packed(allk)))  # == np.unique(allk, axis=0), ~30x faster


def _packed(keys: np.ndarray) -> np.ndarray:
    """int64 key with the lexicographic (x, y, z) order of np.unique(axis=0) (the library's pack_key)."""
    k = keys.astype(np.int64) + (1 << 20)
    return (k[:, 0] << 42) | (k[:, 1] << 21) | k[:, 2]


def _unpacked(p: np.ndarray) -> np.ndarray:
    m = (1 << 21) - 1
    k = np.stack([(p >> 42) & m, (p >> 21) & m, p & m], axis=1) - (1 << 20)
    return k.astype(np.int32)


def merge_to_root(vbg, group=None, root: int = 0, all_ranks: bool = False, method: str = "sparse"):
    """Merge every rank's volume into rank `root`'s (or into all ranks' with all_ranks=True).

    method "sparse" (default, root only): every rank sends each of its blocks once, to the rank
    that owns that block's slice of the sorted union (all-to-all), owners sum the contributions in
    rank order, and the root gathers the owned slices -- per-link traffic ~ (own blocks + U / N)
    blocks instead of the U blocks (mostly zeros) a dense ring reduce moves through every link.
    method "reduce": one dense sum-reduce (or all-reduce) of the zero-padded union.

    `vbg` needs: export_keys(), pack_weighted(keys_ptr, U, out_ptr), unpack_weighted(keys_ptr, U, in_ptr),
    block_resolution, device_id -- mqr.vbg.VoxelBlockGrid on a GPU; tests use a numpy double over gloo.
    Returns the union block count."""
    if method == "sparse" and not all_ranks:
        return _merge_sparse(vbg, group, root)
    if method not in ("sparse", "reduce"):
        raise ValueError(f"unknown merge method {method!r}")
    import torch
    import torch.distributed as dist
    nccl = dist.get_backend(group) == "nccl"
    on_device = getattr(vbg, "on_device", True)   # the numpy stand-in of the CPU tests says False
    vdev = torch.device("cuda", vbg.device_id) if on_device else torch.device("cpu")
    cdev = vdev if nccl else torch.device("cpu")  # gloo collectives run on host tensors
    keys = union_keys(vbg.export_keys(), group=group, device=cdev)
    U = len(keys)
    if U == 0:
        return 0
    R3 = vbg.block_resolution ** 3
    dkeys = torch.as_tensor(keys, device=vdev).contiguous()
    packed = torch.empty((U, R3, 2), dtype=torch.float32, device=vdev)
    if on_device:
        torch.cuda.synchronize(vdev)
    vbg.pack_weighted(dkeys.data_ptr(), U, packed.data_ptr())
    buf = packed if cdev == vdev else packed.to(cdev)
    if all_ranks:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.reduce(buf, dst=root, op=dist.ReduceOp.SUM, group=group)
    if all_ranks or dist.get_rank(group) == root:
        if buf is not packed:
            packed.copy_(buf)
        if on_device:
            torch.cuda.synchronize(vdev)
        vbg.unpack_weighted(dkeys.data_ptr(), U, packed.data_ptr())
    return U


def _merge_sparse(vbg, group, root):
    import torch
    import torch.distributed as dist
    nccl = dist.get_backend(group) == "nccl"
    on_device = getattr(vbg, "on_device", True)
    vdev = torch.device("cuda", vbg.device_id) if on_device else torch.device("cpu")
    cdev = vdev if nccl else torch.device("cpu")
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    local = np.ascontiguousarray(vbg.export_keys(), dtype=np.int32).reshape(-1, 3)
    union = union_keys(local, group=group, device=cdev)
    U = len(union)
    if U == 0:
        return 0
    R3 = vbg.block_resolution ** 3
    bounds = np.array([(U * r) // world for r in range(world + 1)], np.int64)  # owner slices of the union
    idx = np.searchsorted(_packed(union), _packed(local)).astype(np.int64)
    owner = np.searchsorted(bounds, idx, side="right") - 1
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    n = len(local)
    send = torch.empty((n, R3, 2), dtype=torch.float32, device=vdev)
    if n:
        dkeys = torch.as_tensor(np.ascontiguousarray(local[order]), device=vdev).contiguous()
        if on_device:
            torch.cuda.synchronize(vdev)
        vbg.pack_weighted(dkeys.data_ptr(), n, send.data_ptr())
    sc = torch.as_tensor(send_counts, device=cdev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(c) for c in rc.cpu().tolist()]
    sbuf = send if cdev == vdev else send.to(cdev)
    rbuf = torch.empty((sum(recv_counts), R3, 2), dtype=torch.float32, device=cdev)
    dist.all_to_all_single(rbuf, sbuf, output_split_sizes=recv_counts, input_split_sizes=send_counts.tolist(),
                           group=group)
    sidx = torch.as_tensor(np.ascontiguousarray(idx[order]), device=cdev)
    ridx = torch.empty(sum(recv_counts), dtype=torch.int64, device=cdev)
    dist.all_to_all_single(ridx, sidx, output_split_sizes=recv_counts, input_split_sizes=send_counts.tolist(),
                           group=group)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    m = int(np.max(np.diff(bounds)))
    owned = torch.zeros((m, R3, 2), dtype=torch.float32, device=cdev)
    off = 0
    for c in recv_counts:  # source-rank order: deterministic sums (indices unique within a source)
        if c:
            owned.index_add_(0, ridx[off:off + c] - lo, rbuf[off:off + c])
        off += c
    del rbuf, sbuf, send
    gathered = [torch.empty_like(owned) for _ in range(world)] if rank == root else None
    dist.gather(owned, gathered, dst=root, group=group)
    if rank == root:
        full = torch.cat([g[: int(bounds[r + 1] - bounds[r])] for r, g in enumerate(gathered)]).to(vdev)
        full = full.contiguous()
        del gathered
        ukeys = torch.as_tensor(union, device=vdev).contiguous()
        if on_device:
            torch.cuda.synchronize(vdev)
        vbg.unpack_weighted(ukeys.data_ptr(), U, full.data_ptr())
        if on_device:
            torch.cuda.synchronize(vdev)
    return U


# ---------------------------------------------------------------- libmqr RCCL path
MERGE_MODES = {"root": 0, "sharded": 1}


class RcclComm:
    """One rank's RCCL communicator inside libmqr_hip.so (mqr_comm_init)."""

    def __init__(self, device: int, rank: int, world: int, uid: bytes):
        import ctypes
        from . import _lib
        _lib.preload_rccl()
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        h = ctypes.c_void_p()
        _lib.call("mqr_comm_init", int(device), int(rank), int(world), buf, ctypes.byref(h))
        self._h, self.device, self.rank, self.world = h, int(device), int(rank), int(world)

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        _lib.preload_rccl()
        buf = (ctypes.c_uint8 * 128)()
        _lib.call("mqr_comm_unique_id", buf)
        return bytes(buf)

    def timing(self) -> dict:
        """Phases of the last merge (ms, HIP events on the merge stream)."""
        import ctypes
        from . import _lib
        ms = (ctypes.c_float * 4)()
        _lib.call("mqr_comm_timing", self._h, ms)
        return {"plan_ms": ms[0], "out_and_gather_ms": ms[1], "exchange_ms": ms[2], "merge_kernels_ms": ms[3]}

    def counts(self) -> dict:
        """Segment sizes of the last merge: blocks sent to / received from each rank (the own rank's
        entry is the local self segment) and bytes per block."""
        import ctypes
        from . import _lib
        sc, rc = np.zeros(self.world, np.int64), np.zeros(self.world, np.int64)
        fpb = ctypes.c_int64()
        _lib.call("mqr_comm_counts", self._h, _lib.ptr(sc, _lib._i64p), _lib.ptr(rc, _lib._i64p), ctypes.byref(fpb))
        return _segment_stats(sc, rc, 4 * fpb.value, self.rank)

    def close(self):
        from . import _lib
        if getattr(self, "_h", None) is not None and self._h.value and _lib._lib is not None:
            _lib._lib.mqr_comm_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _segment_stats(send_blocks, recv_blocks, bytes_per_block, rank) -> dict:
    """What one rank's merge moved between ranks (its self segment excluded)."""
    sc = np.asarray(send_blocks, np.int64).copy()
    rc = np.asarray(recv_blocks, np.int64).copy()
    sc[rank] = rc[rank] = 0
    return {"bytes_per_block": int(bytes_per_block),
            "sent_blocks": int(sc.sum()), "recv_blocks": int(rc.sum()), "sent_bytes": int(sc.sum()) * bytes_per_block,
            "recv_bytes": int(rc.sum()) * bytes_per_block, "peers_sent_to": int((sc > 0).sum()),
            "max_segment_bytes": int(max(sc.max(), rc.max()) * bytes_per_block) if len(sc) else 0}


def make_comm(device: int, group=None) -> RcclComm:
    """Rank 0 makes the RCCL id; torch.distributed (any backend) broadcasts it; every rank inits."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [RcclComm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return RcclComm(device, rank, world, obj[0])


def _empty_like(vbg):
    from .vbg import VoxelBlockGrid
    return VoxelBlockGrid(voxel_size=vbg.voxel_size, block_resolution=vbg.block_resolution, block_count=1,
                          device=vbg.device_id)


def merge_rccl(vbg, comm: RcclComm, mode: str = "sharded", root: int = 0, out=None):
    """mqr_reduce_rccl: returns (out volume, owned block count).  mode "root": rank `root`'s out
    holds the merged volume; "sharded": every out holds its owned union slice first, then halo."""
    import ctypes
    from . import _lib
    out = out if out is not None else _empty_like(vbg)
    n = ctypes.c_int64()
    _lib.call("mqr_reduce_rccl", vbg.handle, comm._h, MERGE_MODES[mode], int(root), out.handle, ctypes.byref(n))
    return out, n.value


def merge_local(vbgs, mode: str = "sharded", root: int = 0, outs=None):
    """mqr_reduce_rccl's exchange for several volumes of one process on one device, with device
    copies as the transport: every rank plans, packs its send segments and merges in rank order as
    it would over RCCL; sender / receiver segment lists are checked pair by pair (mqr_merge_local).
    Returns [(out volume, owned block count)] per input; outputs must not alias inputs."""
    import ctypes
    from . import _lib
    n = len(vbgs)
    outs = outs if outs is not None else [_empty_like(v) for v in vbgs]
    arr = (ctypes.c_void_p * n)(*[v.handle.value for v in vbgs])
    oarr = (ctypes.c_void_p * n)(*[o.handle.value for o in outs])
    owned = np.zeros(n, np.int64)
    _lib.call("mqr_merge_local", arr, n, MERGE_MODES[mode], int(root), oarr, _lib.ptr(owned, _lib._i64p))
    return list(zip(outs, owned.tolist()))


def merge_staged(vbg, group=None, mode: str = "sharded", root: int = 0, out=None, stats=None):
    """mqr_reduce_rccl's exchange with the segments carried by torch.distributed over host buffers
    (gloo): one process per rank, any device (several ranks may share one GPU, which RCCL refuses).
    The plan, the send segments (packed from this rank's pool), the rank-ordered merge and the output
    are libmqr's own (mqr_xchg_*); only the ncclSend / ncclRecv of the segments is replaced by
    isend / irecv of host tensors.  Every rank's send count to each peer is compared with that
    peer's receive count from it (an all-to-all of the counts) before any segment moves, and
    mqr_xchg_create checks that this rank's row of the gathered keys is its own.  Returns (out
    volume, owned block count); `stats` (a dict) receives the segment sizes (_segment_stats)."""
    import ctypes
    import torch
    import torch.distributed as dist
    from . import _lib
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    out = out if out is not None else _empty_like(vbg)
    local = np.ascontiguousarray(vbg.export_keys(), dtype=np.int32).reshape(-1, 3)
    n = torch.tensor([len(local)], dtype=torch.int64)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    mx = max(1, max(int(c.item()) for c in counts))
    mine = np.full(mx, -1, np.int64)  # 0xFFFF...FF padding (the library's empty key)
    mine[:len(local)] = _packed(local)
    gathered = [torch.empty(mx, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(mine), group=group)
    allk = np.ascontiguousarray(torch.cat(gathered).numpy())
    h = ctypes.c_void_p()
    _lib.call("mqr_xchg_create", vbg.handle, world, rank, MERGE_MODES[mode], int(root), _lib.ptr(allk), int(mx),
              _lib.MQR_HOST, out.handle, ctypes.byref(h))
    try:
        sc, rc = np.zeros(world, np.int64), np.zeros(world, np.int64)
        fpb = ctypes.c_int64()
        _lib.call("mqr_xchg_counts", h, _lib.ptr(sc, _lib._i64p), _lib.ptr(rc, _lib._i64p), None, ctypes.byref(fpb))
        theirs = torch.empty(world, dtype=torch.int64)
        dist.all_to_all_single(theirs, torch.from_numpy(sc.copy()), group=group)
        if not np.array_equal(theirs.numpy(), rc):
            raise RuntimeError(f"merge_staged: rank {rank} expects {rc.tolist()} blocks from the ranks, "
                               f"which send it {theirs.numpy().tolist()}")
        if stats is not None:
            stats.update(_segment_stats(sc, rc, 4 * fpb.value, rank))
        ops, recvs = [], []
        for p in range(world):
            if p == rank:
                continue
            if sc[p]:
                buf = np.empty(int(sc[p]) * fpb.value, np.float32)
                _lib.call("mqr_xchg_send_segment", h, p, _lib.ptr(buf), _lib.MQR_HOST)
                ops.append(dist.isend(torch.from_numpy(buf), dst=_global(group, p), group=group))
            if rc[p]:
                t = torch.empty(int(rc[p]) * fpb.value, dtype=torch.float32)
                ops.append(dist.irecv(t, src=_global(group, p), group=group))
                recvs.append((p, t))
        for op in ops:
            op.wait()
        for p, t in recvs:
            _lib.call("mqr_xchg_recv_segment", h, p, ctypes.c_void_p(t.data_ptr()), _lib.MQR_HOST)
        owned = ctypes.c_int64()
        _lib.call("mqr_xchg_finish", h, ctypes.byref(owned))
    finally:
        _lib._lib.mqr_xchg_destroy(h)
    return out, owned.value


def _global(group, r):
    """Global rank of group rank r (torch.distributed's point-to-point calls take global ranks)."""
    import torch.distributed as dist
    return r if group is None else dist.get_global_rank(group, r)


def merge_local_timing(n: int):
    """Per-rank wall ms of the last merge_local (one rank's plan, output volume, send-segment gather
    and merge kernels, without the transfer)."""
    from . import _lib
    ms = np.zeros(n, np.float32)
    _lib.call("mqr_merge_local_timing", _lib.ptr(ms, _lib._f32p), int(n))
    return ms.tolist()


def set_merge_per_source(on: bool, f32_segments: bool = False):
    """Process-wide merge A/B hooks (mqr_merge_set_per_source): on = the round-5 pass per source rank
    instead of one fused pass per output block; f32_segments = merge_local sends float32 weights even
    where uint16 holds them.  Same bits; for A/Bs and tests."""
    from . import _lib
    _lib.call("mqr_merge_set_per_source", (1 if on else 0) | (2 if f32_segments else 0))


def extract_mesh_owned(vbg, n_owned: int, weight_threshold: float = 1.5):
    """A shard's mesh: triangles of the cubes whose origin lies in its owned blocks, the vertices
    they reference (re-indexed; vertices on the shard boundary also appear in the neighbour's mesh)."""
    import ctypes
    from . import _lib
    from ._lib import MQR_HOST, call, ptr
    from .geometry import TriangleMesh
    g = ctypes.c_void_p()
    call("mqr_extract_mesh_owned", vbg.handle, float(weight_threshold), int(n_owned), ctypes.byref(g))
    try:
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        call("mqr_geom_counts", g, ctypes.byref(nv), ctypes.byref(nt))
        pos = np.empty((nv.value, 3), np.float32)
        nrm = np.empty((nv.value, 3), np.float32)
        tri = np.empty((nt.value, 3), np.int32)
        call("mqr_geom_copy", g, ptr(pos), ptr(nrm), ptr(tri) if nt.value else None, MQR_HOST)
    finally:
        _lib._lib.mqr_geom_free(g)
    used = np.zeros(len(pos), bool)
    used[tri.reshape(-1)] = True
    remap = np.cumsum(used) - 1
    return TriangleMesh(pos[used], nrm[used], remap[tri].astype(np.int32), device=vbg.device)
