#!/usr/bin/env python3
"""What the integrate kernel's voxel-frames do, on one 64-frame batch of the C2 walk (CPU, numpy).

Answers two questions behind the integrate kernel's design:

1. Culling potential: of the voxel-frames of the touched blocks (every voxel of every block a frame
   touches), how many update, lie outside the image, see an invalid depth, or lie behind the
   surface by more than the truncation (sdf < -trunc)?  How many 64-voxel wave bricks (the lean
   kernel's brick map, one gather instruction each) and whole (block, frame) pairs have no
   updating voxel at all -- the most an exact wave- or block-level cull could skip?
2. Address-path cost: the kernel's depth gathers cost about one L1 tag lookup per distinct
   (lane quad, dword) address.  Distinct (quad, pixel) pairs per 64-lane gather for the current
   lane -> voxel map and for alternative quad shapes.

Float32 projection as in the kernel (statistics only; parity is the oracle's job).
Output: JSON on stdout.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

VS, R, DMAX, TAU, H, W = 0.005, 16, 4.0, 0.05, 480, 640
LANE = np.arange(64)


def lane_maps():
    """(wave w, lane l, voxel k) -> (x, y, z) within the 16^3 block."""
    def brick(w, l, k):  # the kernel's map (vbg_kernels.hpp lean_map<..., 1>)
        return (l % 8) + 8 * (w % 2), ((l // 8) % 2) + 2 * (w // 2) + 8 * (k // 4), l // 16 + 4 * (k % 4)

    def quad_xz(w, l, k):
        x = (l & 1) | ((l >> 2) & 3) << 1 | 8 * (w % 2)
        z = ((l >> 1) & 1) | ((l >> 5) & 1) << 1
        return x, ((l >> 4) & 1) + 2 * (w // 2) + 8 * (k // 4), z + 4 * (k % 4)

    def quad_z(w, l, k):
        return ((l >> 2) & 7) + 8 * (w % 2), (l >> 5) + 2 * (w // 2) + 8 * (k // 4), (l & 3) + 4 * (k % 4)

    def quad_xy(w, l, k):
        x = (l & 1) | ((l >> 2) & 3) << 1 | 8 * (w % 2)
        return x, ((l >> 1) & 1) + 2 * (w // 2) + 8 * (k // 4), (l >> 4) + 4 * (k % 4)

    return {"brick (kernel): quads along x": brick, "quads 2x2 in x-z": quad_xz, "quads along z": quad_z,
            "quads 2x2 in x-y": quad_xy}


def project(keys, x, y, z, E, K):
    fx, fy, cx, cy = (np.float32(K[0, 0]), np.float32(K[1, 1]), np.float32(K[0, 2]), np.float32(K[1, 2]))
    X = ((keys[:, 0:1] * R + x[None]) * np.float32(VS)).astype(np.float32)
    Y = ((keys[:, 1:2] * R + y[None]) * np.float32(VS)).astype(np.float32)
    Z = ((keys[:, 2:3] * R + z[None]) * np.float32(VS)).astype(np.float32)
    xc = X * E[0, 0] + Y * E[0, 1] + Z * E[0, 2] + E[0, 3]
    yc = X * E[1, 0] + Y * E[1, 1] + Z * E[1, 2] + E[1, 3]
    zc = X * E[2, 0] + Y * E[2, 1] + Z * E[2, 2] + E[2, 3]
    with np.errstate(divide="ignore", invalid="ignore"):
        u = fx * xc / zc + cx
        v = fy * yc / zc + cy
    inimg = (u >= 0) & (v >= 0) & (u <= W - 1) & (v <= H - 1) & (zc > 0)
    ui = np.clip(np.nan_to_num(u), 0, W - 1).astype(np.int64)
    vi = np.clip(np.nan_to_num(v), 0, H - 1).astype(np.int64)
    return zc, inimg, vi * W + ui, u, v


TILE = int(os.environ.get("MQR_WS_TILE", "16"))


def tile_max_dilated(d):
    """Per TILE x TILE pixel tile: the largest valid depth (0 < d <= DMAX; -inf if none), then the
    maximum over each tile's 3 x 3 tile neighbourhood."""
    th, tw = -(-H // TILE), -(-W // TILE)
    dd = np.where((d > 0) & (d <= DMAX), d, -np.inf).astype(np.float32)
    pad = np.full((th * TILE, tw * TILE), -np.inf, np.float32)
    pad[:H, :W] = dd
    t = pad.reshape(th, TILE, tw, TILE).max(axis=(1, 3))
    p = np.pad(t, 1, constant_values=-np.inf)
    return np.max([p[i:i + th, j:j + tw] for i in range(3) for j in range(3)], axis=0)


def main():
    import oracle
    from mqr import synthetic
    poses = synthetic.room_loop_poses(500)[128:192]
    seq = synthetic.make_sequence("room", poses=poses, height=H, width=W, noise=True, seed=0)
    D, K, T = seq["depth"], seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    zz, yy, xx = (a.ravel() for a in np.meshgrid(np.arange(R), np.arange(R), np.arange(R), indexing="ij"))
    bw = (xx // 8) + 2 * ((yy % 8) // 2)  # brick map: wave of each voxel
    bk = 4 * (yy // 8) + (zz // 4)        # and its voxel slot k
    brick = bw * 8 + bk
    tot = dict(voxel_frames=0, outside_image=0, invalid_depth=0, behind_surface=0, update=0)
    bricks = dead_bricks = out_bricks = pairs = dead_pairs = tile_bricks = 0
    # lane 0 of each wave slot (brick id w * 8 + k): x = 8 (w % 2), y = 2 (w // 2) + 8 (k // 4), z = 4 (k % 4)
    lane0 = np.zeros(64, np.int64)
    for w in range(8):
        for k in range(8):
            x0, y0, z0 = 8 * (w % 2), 2 * (w // 2) + 8 * (k // 4), 4 * (k % 4)
            lane0[w * 8 + k] = (z0 * R + y0) * R + x0
    quad = {name: [0, 0] for name in lane_maps()}
    for f in range(len(poses)):
        keys = oracle.touch(D[f], K[f], T[f], VS, R, 1.0, DMAX, 10.0)
        E = T[f].astype(np.float32)
        tmd = tile_max_dilated(D[f])
        for c in range(0, len(keys), 256):
            kk = keys[c:c + 256]
            zc, inimg, pix, uu, vv = project(kk, xx, yy, zz, E, K[f])
            d = D[f].reshape(-1)[pix]
            dv = inimg & (d > 0) & (d <= DMAX)
            upd = dv & (d - zc >= -TAU)
            tot["voxel_frames"] += upd.size
            tot["outside_image"] += int((~inimg).sum())
            tot["invalid_depth"] += int((inimg & ~dv).sum())
            tot["behind_surface"] += int((dv & ~upd).sum())
            tot["update"] += int(upd.sum())
            rows = np.repeat(np.arange(len(kk)), R ** 3)
            ub = np.zeros((len(kk), 64), bool)
            np.logical_or.at(ub, (rows, np.tile(brick, len(kk))), upd.ravel())
            ib = np.zeros((len(kk), 64), bool)
            np.logical_or.at(ib, (rows, np.tile(brick, len(kk))), inimg.ravel())
            # tile cull: lane 0's pixel picks a tile; a lane is certainly not
            # updating when outside the image, or within 16 px of lane 0's pixel (so its own tile is in
            # the 3 x 3 neighbourhood) with zc - (neighbourhood max depth) > trunc
            l0 = lane0[brick]                                      # per voxel: its slot's lane-0 voxel
            u0, v0, in0 = uu[:, l0], vv[:, l0], inimg[:, l0]
            t0 = np.where(in0, tmd[np.clip(np.nan_to_num(v0), 0, H - 1).astype(np.int64) // TILE,
                                   np.clip(np.nan_to_num(u0), 0, W - 1).astype(np.int64) // TILE], np.inf)
            with np.errstate(invalid="ignore"):
                near = (np.abs(uu - u0) < TILE) & (np.abs(vv - v0) < TILE)
                sure = (~inimg) | (near & (zc - t0 > TAU))
            sb = np.ones((len(kk), 64), bool)
            np.logical_and.at(sb, (rows, np.tile(brick, len(kk))), sure.ravel())
            tile_bricks += int((sb & ib).sum())
            bricks += ub.size
            dead_bricks += int((~ub).sum())
            out_bricks += int((~ib).sum())
            pairs += len(kk)
            dead_pairs += int((~ub.any(1)).sum())
        if f % 4 == 0:  # the quad statistics on every 4th frame, every 7th block
            sub = keys[::7]
            for name, mp in lane_maps().items():
                for w in range(8):
                    for k in range(8):
                        x, y, z = mp(w, LANE, k)
                        _, inimg, pix, _, _ = project(sub, x, y, z, E, K[f])
                        q = np.sort(np.where(inimg, pix, -1).reshape(len(sub), 16, 4), axis=2)
                        distinct = (q[:, :, 1:] != q[:, :, :-1]).sum(2) + 1 - (q[:, :, 0] == -1)
                        quad[name][0] += int(distinct.sum())
                        quad[name][1] += len(sub)
    out = {"workload": "C2 room walk frames 128-191 (one 64-frame batch), 640x480, 5 mm, R 16, trunc 10",
           "voxel_frames": tot["voxel_frames"],
           "fractions": {k: v / tot["voxel_frames"] for k, v in tot.items() if k != "voxel_frames"},
           "wave_bricks_without_update": dead_bricks / bricks,
           "wave_bricks_entirely_outside_image": out_bricks / bricks,
           "wave_bricks_in_image_culled_by_tile_max": tile_bricks / bricks, "cull_tile_px": TILE,
           "block_frame_pairs_without_update": dead_pairs / pairs, "block_frame_pairs": pairs,
           "distinct_quad_pixels_per_64_lane_gather": {n: q / g for n, (q, g) in quad.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
