#!/usr/bin/env python3
"""What the C4 exchange moves, per rank, at 2 / 4 / 8 ranks (verdict r05 item 2): the 2000-frame
LEFT+RIGHT capture split by contiguous frame ranges exactly as bench.py --gpus N splits it, each
shard integrated into its own volume on this one GPU, then the sharded plan of csrc/merge.hip
(sorted union, owner slices [U r / W, U (r+1) / W), destinations = owner + owners of the 26
neighbours) restated in numpy over the exported keys and weights.  For every rank: blocks and bytes
it sends to / receives from peers (the self segment excluded), and the fraction of the sent voxels
whose weight is 0 (those add nothing to sum(w tsdf) / sum(w)).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, ROOT)


def packed(k):
    import numpy as np
    k = k.astype(np.int64) + (1 << 20)
    return (k[:, 0] << 42) | (k[:, 1] << 21) | k[:, 2]


def plan_counts(keys_per_rank, zeros_per_rank, R3):
    """Sharded-mode send / receive block counts and zero-weight voxels per rank (merge.hip's plan)."""
    import numpy as np
    W = len(keys_per_rank)
    pk = [packed(k) for k in keys_per_rank]
    uni = np.unique(np.concatenate(pk))
    U = len(uni)
    lo = np.array([U * r // W for r in range(W + 1)], np.int64)
    owner_of = lambda u: np.searchsorted(lo, u, side="right") - 1  # noqa: E731
    # destination mask per union block: its owner and the owners of its 26 neighbours
    ukeys = np.stack([(uni >> 42) & 0x1FFFFF, (uni >> 21) & 0x1FFFFF, uni & 0x1FFFFF], 1) - (1 << 20)
    dm = np.zeros(U, np.uint64)
    dm |= (np.uint64(1) << owner_of(np.arange(U)).astype(np.uint64))
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dz in (-1, 0, 1):
                if dx == dy == dz == 0:
                    continue
                nk = packed(ukeys + np.array([dx, dy, dz]))
                j = np.searchsorted(uni, nk)
                ok = (j < U) & (uni[np.minimum(j, U - 1)] == nk)
                dm[ok] |= np.uint64(1) << owner_of(j[ok]).astype(np.uint64)
    out = []
    recv = np.zeros(W, np.int64)
    for r in range(W):
        u = np.searchsorted(uni, pk[r])
        m = dm[u] & ~(np.uint64(1) << np.uint64(r))          # peers only
        ndest = np.array([bin(int(x)).count("1") for x in m], np.int64)
        for d in range(W):
            if d != r:
                recv[d] += int(((m >> np.uint64(d)) & np.uint64(1)).sum())
        sent_vox = int(ndest.sum()) * R3
        sent_zero = int((ndest * zeros_per_rank[r]).sum())
        out.append({"blocks": len(pk[r]), "sent_blocks": int(ndest.sum()), "sent_bytes": sent_vox * 8,
                    "sent_zero_weight_frac": sent_zero / max(sent_vox, 1),
                    "zero_weight_frac_all_blocks": float(zeros_per_rank[r].sum()) / max(len(pk[r]) * R3, 1)})
    for r in range(W):
        out[r]["recv_blocks"] = int(recv[r])
        out[r]["recv_bytes"] = int(recv[r]) * R3 * 8
        # the segments as the library sends integrated volumes: tsdf float32 + weight uint16 (6 B per voxel)
        out[r]["sent_bytes_uint16_weights"] = out[r]["sent_bytes"] // 8 * 6
        out[r]["recv_bytes_uint16_weights"] = out[r]["recv_bytes"] // 8 * 6
    return U, out


def main():
    import argparse
    import numpy as np
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--frames-per-side", type=int, default=1000)
    a = ap.parse_args()
    from bench import _DevPtr
    from mqr import synthetic
    from mqr.distributed import merge_local, merge_local_timing, set_merge_per_source, shard_range
    from mqr.vbg import VoxelBlockGrid
    left = synthetic.room_loop_poses(a.frames_per_side)
    right = [(R_, t_ + R_[:, 0] * 0.064) for R_, t_ in left]
    full = synthetic.make_sequence_fast("room", poses=left + right, height=480, width=640, seed=4, device="cuda:0")
    depth = full["depth_t"].contiguous()
    K, T = full["K"].astype(np.float64), full["T_wc"].astype(np.float64)
    n = depth.shape[0]
    R, R3 = 16, 16 ** 3
    res = {"workload": "C4 capture (1000 LEFT + 1000 RIGHT, 640x480, 5 mm, R=16), bench.py's contiguous split",
           "per_world": {}}
    for W in [int(x) for x in a.ranks.split(",")]:
        keys, zeros, vols, int_ms = [], [], [], []
        for r in range(W):
            lo, hi = shard_range(n, r, W)
            d = depth[lo:hi]
            v = VoxelBlockGrid(voxel_size=0.005, block_resolution=R, block_count=16384, device=0)
            ts = []
            for _ in range(4):  # one rank's step work: reset + integrate of its frame range (first = warm-up)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                v.reset()
                v.integrate_frames((_DevPtr(d.data_ptr()), hi - lo, 480, 640), K[lo:hi], T[lo:hi], depth_scale=1.0,
                                   depth_max=4.0, trunc_voxel_multiplier=10.0)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            int_ms.append(sorted(ts[1:])[1] * 1e3)
            k, _, w = v.export()
            keys.append(k)
            zeros.append((w.reshape(len(k), -1) == 0).sum(1).astype(np.int64))
            vols.append(v)
        U, per = plan_counts(keys, zeros, R3)
        # one rank's own share of the exchange without the transfer (plan, output volume, send gather,
        # merge kernels): mqr_merge_local's per-destination wall times, median of 3 after a warm-up
        # (and the same with the round-5 merge, one pass over the output per source: mqr_merge_set_per_source)
        def own_times(per_source):
            set_merge_per_source(per_source)
            try:
                outs_, reps = None, []
                for _ in range(6):
                    got_ = merge_local(vols, mode="sharded", outs=outs_)
                    outs_ = [o for o, _ in got_]
                    reps.append(merge_local_timing(W))
            finally:
                set_merge_per_source(False)
            return [sorted(rr[i] for rr in reps[1:])[2] for i in range(W)], outs_, got_
        own_ps, _, _ = own_times(True)
        own_ms, outs, got = own_times(False)
        sent = sum(p["sent_blocks"] for p in per) * R3
        zf = sum(p["sent_zero_weight_frac"] * p["sent_blocks"] for p in per) * R3 / max(sent, 1)
        for r in range(W):
            per[r]["integrate_ms"] = int_ms[r]
            per[r]["merge_own_ms"] = own_ms[r]
            per[r]["merge_own_ms_per_source"] = own_ps[r]
        res["per_world"][W] = {"union_blocks": U, "ranks": per,
                               "max_sent_bytes": max(p["sent_bytes"] for p in per),
                               "max_sent_bytes_uint16_weights": max(p["sent_bytes_uint16_weights"] for p in per),
                               "max_recv_bytes_uint16_weights": max(p["recv_bytes_uint16_weights"] for p in per),
                               "max_recv_bytes": max(p["recv_bytes"] for p in per),
                               "max_integrate_ms": max(int_ms), "max_merge_own_ms": max(own_ms),
                               "max_merge_own_ms_per_source": max(own_ps),
                               "sent_zero_weight_frac": zf}
        print(f"W={W}: U={U} max sent {res['per_world'][W]['max_sent_bytes'] / 1e6:.1f} MB, "
              f"zero-weight {zf:.3f}, integrate {max(int_ms):.2f} ms, own merge {max(own_ms):.2f} ms "
              f"(per-source merge {max(own_ps):.2f})",
              file=sys.stderr, flush=True)
        del vols, outs, got
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
