"""Debug: merge_local vs a numpy merge of the shard exports and vs the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import oracle
from mqr import _lib, synthetic
from mqr.distributed import merge_local, shard_range
from mqr.vbg import VoxelBlockGrid
_lib.load()
seq = synthetic.make_sequence("room", n=36, height=240, width=320, f=262.5, noise=True, seed=12)
ref = oracle.OracleVBG(0.01, 16, 256)
for i in range(36):
    ref.integrate_frame(seq["depth"][i], seq["K"][i].astype(np.float64), seq["T_wc"][i].astype(np.float64), 1.0, 4.0, 10.0)
rk, rt, rw = ref.export()
rmap = {tuple(k): i for i, k in enumerate(rk)}
single = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
single.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
sk, st_, sw = single.export()
print("single vs oracle bad", sum(not np.array_equal(sw[i], rw[rmap[tuple(k)]]) for i, k in enumerate(sk)))
for world, root in ((1, 0), (2, 1), (2, 0)):
    vols = []
    for r in range(world):
        lo, hi = shard_range(36, r, world)
        v = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
        v.integrate_frames(seq["depth"][lo:hi], seq["K"][lo:hi], seq["T_wc"][lo:hi], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
        vols.append(v)
    res = merge_local(vols, mode="root", root=root)
    out, n = res[root]
    k, t, w = out.export()
    acc = {}
    for v in vols:
        kk, tt, ww = v.export()
        for i, key in enumerate(map(tuple, kk)):
            acc[key] = acc[key] + ww[i] if key in acc else ww[i].copy()
    bad = sum(not np.array_equal(acc[key], w[i]) for i, key in enumerate(map(tuple, k)))
    badr = sum(not np.array_equal(rw[rmap[key]], w[i]) for i, key in enumerate(map(tuple, k)))
    bads = sum(not np.array_equal(rw[rmap[key]], acc[key]) for key in acc)
    print("world", world, "root", root, "n", n, "blocks", len(k), "ref blocks", len(rk), "bad vs sum", bad, "bad vs oracle", badr, "sum vs oracle", bads)
