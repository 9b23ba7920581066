#!/usr/bin/env python3
"""What lane-level tile proofs could take off the integrate kernel's depth reads (verdict r05 item 3),
on frames of the C2 walk (CPU, numpy; statistics only, parity is the oracle's job).

Per T x T pixel tile of a frame, a 16-byte record: a validity bit per pixel (the update's
`!(d <= 0) && !(d > depth_max)`, which NaN passes), lo = min of the valid non-NaN depths, hi = max of
them (+inf when the tile holds a NaN).  A lane whose voxel projects into the image reads its tile's
record first and is decided without its pixel when
  * its bit is 0                      -> no update (exact: the update's own depth test fails);
  * fl(lo - zc) >= trunc              -> the update with s = trunc, sn = 1 exactly (sdf >= trunc for
                                         every valid pixel of the tile by monotone rounding; a NaN
                                         pixel takes s = trunc too);
  * fl(hi - zc) < -trunc              -> no update.
Reported per 64-lane wave slot (the kernel's brick map) and frame: lanes decided, slots whose every
lane is decided or outside the image (their pixel read is skipped), distinct 8-byte windows per
pixel read with and without the proofs, distinct records per record read.  JSON on stdout."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metaquest-3d-reconstruction_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from integrate_work_stats import DMAX, H, R, VS, W, project  # noqa: E402

TAU = np.float32(np.float32(10.0) * np.float32(VS))


def tile_records(d, T):
    th, tw = -(-H // T), -(-W // T)
    valid = ~(d <= 0) & ~(d > DMAX)
    fin = valid & ~np.isnan(d)
    pad = lambda a, v: np.pad(a, ((0, th * T - H), (0, tw * T - W)), constant_values=v)  # noqa: E731
    lo = np.where(pad(fin, False), pad(d, 0), np.inf).reshape(th, T, tw, T).min(axis=(1, 3)).astype(np.float32)
    hi = np.where(pad(fin, False), pad(d, 0), -np.inf).reshape(th, T, tw, T).max(axis=(1, 3)).astype(np.float32)
    hasnan = pad(np.isnan(d), False).reshape(th, T, tw, T).any(axis=(1, 3))
    hi[hasnan] = np.inf
    return valid, lo, hi


def main():
    import oracle
    from mqr import synthetic
    nfr = int(os.environ.get("MQR_TP_FRAMES", "12"))
    poses = synthetic.room_loop_poses(500)[128:128 + nfr]
    seq = synthetic.make_sequence("room", poses=poses, height=H, width=W, noise=True, seed=0)
    D, K, Tw = seq["depth"], seq["K"].astype(np.float64), seq["T_wc"].astype(np.float64)
    zz, yy, xx = (a.ravel() for a in np.meshgrid(np.arange(R), np.arange(R), np.arange(R), indexing="ij"))
    slot = ((xx // 8) + 2 * ((yy % 8) // 2)) * 8 + 4 * (yy // 8) + (zz // 4)  # wave * 8 + k (brick map)
    order = np.argsort(slot, kind="stable")                                  # voxels grouped by slot
    res = {}
    for T in (4, 8):
        acc = dict(lanes=0, in_img=0, dec_invalid=0, dec_clamp=0, dec_behind=0, slots=0, slots_skip=0,
                   slots_skip_in_img=0, win_base=0, win_left=0, rec=0, reads_base=0, reads_left=0)
        for f in range(nfr):
            keys = oracle.touch(D[f], K[f], Tw[f], VS, R, 1.0, DMAX, 10.0)
            E = Tw[f].astype(np.float32)
            valid, lo, hi = tile_records(D[f], T)
            for c in range(0, len(keys), 128):
                kk = keys[c:c + 128]
                zc, inimg, pix, uu, vv = project(kk, xx, yy, zz, E, K[f])
                zc, inimg, pix = zc[:, order], inimg[:, order], pix[:, order]
                pv, pu = pix // W, pix % W
                tix = (pv // T) * (-(-W // T)) + pu // T
                bit = valid.reshape(-1)[pix] & inimg
                with np.errstate(invalid="ignore", over="ignore"):
                    clamp = inimg & bit & ((lo.reshape(-1)[tix] - zc).astype(np.float32) >= TAU)
                    behind = inimg & bit & ((hi.reshape(-1)[tix] - zc).astype(np.float32) < -TAU)
                dec = inimg & (~bit | clamp | behind)
                need = inimg & ~dec
                acc["lanes"] += zc.size
                acc["in_img"] += int(inimg.sum())
                acc["dec_invalid"] += int((inimg & ~bit).sum())
                acc["dec_clamp"] += int(clamp.sum())
                acc["dec_behind"] += int(behind.sum())
                S = zc.shape[0] * 64
                need_s, in_s = need.reshape(S, 64), inimg.reshape(S, 64)
                win = np.where(in_s, pix.reshape(S, 64) >> 1, -1)
                winl = np.where(need_s, win, -1)
                recs = np.where(in_s, tix.reshape(S, 64), -1)

                def distinct(a):
                    s = np.sort(a, axis=1)
                    return ((s[:, 1:] != s[:, :-1]) & (s[:, 1:] >= 0)).sum(1) + (s[:, 0] >= 0)
                acc["slots"] += S
                acc["slots_skip"] += int((~need_s.any(1)).sum())
                acc["slots_skip_in_img"] += int((~need_s.any(1) & in_s.any(1)).sum())
                acc["win_base"] += int(distinct(win).sum())
                acc["reads_base"] += S
                acc["win_left"] += int(distinct(winl).sum())
                acc["reads_left"] += int(need_s.any(1).sum())
                acc["rec"] += int(distinct(recs).sum())
        ii = max(acc["in_img"], 1)
        res[f"{T}x{T}"] = {
            "in_image_lane_frac": acc["in_img"] / acc["lanes"],
            "decided_frac_of_in_image": {"invalid": acc["dec_invalid"] / ii, "clamped": acc["dec_clamp"] / ii,
                                         "behind": acc["dec_behind"] / ii,
                                         "total": (acc["dec_invalid"] + acc["dec_clamp"] + acc["dec_behind"]) / ii},
            "slots_without_pixel_read": acc["slots_skip"] / acc["slots"],
            "slots_in_image_without_pixel_read": acc["slots_skip_in_img"] / acc["slots"],
            "distinct_windows_per_slot_baseline": acc["win_base"] / acc["reads_base"],
            "distinct_windows_per_issued_read_with_proofs": acc["win_left"] / max(acc["reads_left"], 1),
            "distinct_windows_total_ratio": acc["win_left"] / max(acc["win_base"], 1),
            "distinct_records_per_slot": acc["rec"] / acc["slots"]}
        print(T, json.dumps(res[f"{T}x{T}"]), file=sys.stderr, flush=True)
    print(json.dumps({"workload": f"C2 room walk frames 128-{127 + nfr}, 640x480, 5 mm, R 16, trunc 10",
                      "tiles": res}, indent=1))


if __name__ == "__main__":
    main()
