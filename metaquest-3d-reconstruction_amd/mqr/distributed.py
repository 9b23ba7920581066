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
"""
from __future__ import annotations

import numpy as np


def shard_range(n_frames: int, rank: int, world: int):
    """Contiguous frame range [lo, hi) of `rank` (the first n % world ranks get one more)."""
    base, extra = divmod(n_frames, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


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
    return np.unique(allk, axis=0).astype(np.int32)


def merge_to_root(vbg, group=None, root: int = 0, all_ranks: bool = False):
    """Merge every rank's volume into rank `root`'s (or into all ranks' with all_ranks=True).

    `vbg` needs: export_keys(), pack_weighted(keys_ptr, U, out_ptr), unpack_weighted(keys_ptr, U, in_ptr),
    block_resolution, device_id -- mqr.vbg.VoxelBlockGrid on a GPU; tests use a numpy double over gloo.
    Returns the union block count."""
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
