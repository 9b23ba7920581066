import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
import numpy as np
from mqr import _lib, synthetic
from mqr.distributed import merge_local
from mqr.vbg import VoxelBlockGrid
_lib.load()
seq = synthetic.make_sequence("room", n=36, height=240, width=320, f=262.5, noise=True, seed=12)
v = VoxelBlockGrid(voxel_size=0.01, block_resolution=16, block_count=64)
v.integrate_frames(seq["depth"], seq["K"], seq["T_wc"], depth_scale=1.0, depth_max=4.0, trunc_voxel_multiplier=10.0)
lk, lt, lw = v.export()
lmap = {tuple(k): i for i, k in enumerate(lk)}
out, n = merge_local([v], mode="root")[0]
k, t, w = out.export()
bad = [i for i, key in enumerate(map(tuple, k)) if not np.array_equal(lw[lmap[key]], w[i])]
print("n", n, "bad", len(bad), bad[:20], bad[-5:])
wsum = {i: float(w[i].sum()) for i in bad[:5]}
print("out wsum", wsum, "expected", {i: float(lw[lmap[tuple(k[i])]].sum()) for i in bad[:5]})
# is the bad block a copy of some other local block?
sig = {float(lw[j].sum()) * 1e6 + float(lt[j].sum()): j for j in range(len(lk))}
for i in bad[:5]:
    s = float(w[i].sum()) * 1e6 + float(t[i].sum())
    print(i, "matches local block", sig.get(s), "its local index", lmap[tuple(k[i])], "zero?", not w[i].any())
