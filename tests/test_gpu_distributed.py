"""2-3 ranks (gloo, all on GPU 0) run the real multi-GPU merge path: frame-sharded integration
through libmqr_hip.so, key union, then the sparse all-to-all + gather (or the dense sum-reduce) and
unpack; rank 0's volume must equal a single sequential pass (same keys and weights, tsdf within 1e-4)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q, method):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mqr import synthetic
        from mqr.distributed import merge_to_root, shard_range
        from mqr.vbg import VoxelBlockGrid
        seq = synthetic.make_sequence("room", n=24, height=240, width=320, f=262.5, noise=True, seed=31)
        lo, hi = shard_range(24, rank, world)
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64, device=0)
        v.integrate_frames(seq["depth"][lo:hi], seq["K"][lo:hi], seq["T_wc"][lo:hi], depth_scale=1.0,
                           depth_max=4.0, trunc_voxel_multiplier=10.0)
        U = merge_to_root(v, root=0, method=method)
        if rank == 0:
            k, t, w = v.export()
            q.put((rank, U, k, t, w))
        else:
            q.put((rank, U, None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,method", [(2, "sparse"), (2, "reduce"), (3, "sparse")])
def test_multi_rank_merge_on_gpu(world, method):
    import oracle
    import torch.multiprocessing as mp
    from gpu_helpers import compare_volumes
    from mqr import synthetic
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, method)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=300)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    seq = synthetic.make_sequence("room", n=24, height=240, width=320, f=262.5, noise=True, seed=31)
    ref = oracle.OracleVBG(0.01, 16, 256)
    for i in range(24):
        ref.integrate_frame(seq["depth"][i], seq["K"][i].astype(np.float64), seq["T_wc"][i].astype(np.float64),
                            1.0, 4.0, 10.0)
    _, U, k, t, w = res[0]
    assert all(res[r][1] == U for r in range(world)) and U == ref.size()
    assert compare_volumes((k, t, w), ref.export(), 1e-4) < 1e-5


@pytest.mark.parametrize("world", [2, 3])
def test_confidence_shards_concatenate_to_single_pass(world):
    """§8(e) confidence: each rank computes its reference-frame range with a +-r halo, no collective;
    the shards in rank order equal the single-GPU maps bit for bit (an invalid frame included)."""
    import numpy as np
    import torch
    assert torch.cuda.is_available()
    from mqr import synthetic
    from mqr.confidence import confidence_maps
    from mqr.distributed import confidence_shard
    seq = synthetic.make_sequence("room", n=23, height=120, width=160, f=131.25, noise=True, seed=4)
    d, K, Tcw = seq["depth"], seq["K"], seq["T_cw"]
    Ti = np.linalg.inv(Tcw)
    ok = np.ones(len(d), np.uint8)
    ok[7] = 0
    full_c, full_v = confidence_maps(d, K, Tcw, Ti, 0, len(d), 4, 4.0, 0.08, ok)
    parts = [confidence_shard(d, K, Tcw, Ti, r, world, 4, 4.0, 0.08, ok) for r in range(world)]
    assert [p[0] for p in parts] == sorted(p[0] for p in parts) and parts[-1][1] == len(d)
    assert np.array_equal(np.concatenate([p[2] for p in parts]), full_c)
    assert np.array_equal(np.concatenate([p[3] for p in parts]), full_v)
