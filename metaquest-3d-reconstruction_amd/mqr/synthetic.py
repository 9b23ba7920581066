"""Synthetic Quest-style depth captures (there is no network and the reference ships no data).

Generates the BASELINE.json configurations:

* ``sphere``: procedural sphere r=0.5 m at the origin, cameras on a 1.5 m ring at 0.2 m height
  looking at the origin (config 0 / C1: 32 frames 640x480, 2 cm voxels).
* ``room``: a 2.56 m cube room (= 512^3 voxels at 5 mm) with three spheres and two boxes; the
  head walks a closed loop at 1.6 m with a +-60 deg yaw sweep (configs 1-4: 500+ frames, 5 mm).

Depth is ray-cast analytically at integer pixel coordinates in the Open3D camera convention,
optionally corrupted (sigma = 0.002 z Gaussian, 1 % dropout, ``default_rng(seed)``), encoded as
the Quest NDC buffer (``d = 1 - near/z`` for ``far = inf``), and can be written out as a capture
directory in the reference layout (raw files + descriptor CSV with UNITY poses).  The in-memory
``make_sequence`` goes through the same encode -> decode -> UNITY -> Open3D round trip, so its
depth / K / T are exactly what the reference's loaders would hand to the integrator.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from .depth_utils import convert_depth_to_linear, encode_linear_to_ndc
from .models import CoordinateSystem, Transforms
from scipy.spatial.transform import Rotation

NEAR = 0.1
FAR = float("inf")

SCENES = {
    "sphere": {"spheres": [((0.0, 0.0, 0.0), 0.5)], "boxes": [], "room": None},
    "room": {
        "spheres": [((0.6, 0.4, 0.7), 0.35), ((-0.7, 1.0, -0.5), 0.25), ((0.2, 1.9, -0.9), 0.2)],
        "boxes": [((-1.1, 0.0, 0.5), (-0.5, 0.75, 1.1)), ((0.5, 0.0, -1.2), (1.2, 1.2, -0.7))],
        "room": ((-1.28, 0.0, -1.28), (1.28, 2.56, 1.28)),
    },
    # C5: an 8 x 8 x 3 m hall with furniture-sized boxes and spheres
    "hall": {
        "spheres": [((1.5, 0.6, 1.0), 0.6), ((-2.0, 0.4, -1.5), 0.4), ((0.5, 2.2, -2.5), 0.3), ((-2.8, 1.2, 2.6), 0.5)],
        "boxes": [((-3.5, 0.0, 1.0), (-2.0, 0.9, 3.5)), ((2.0, 0.0, -3.5), (3.8, 2.0, -2.5)),
                  ((-0.8, 0.0, -0.6), (0.6, 0.75, 0.6)), ((2.8, 0.0, 2.0), (3.6, 1.2, 3.8))],
        "room": ((-4.0, 0.0, -4.0), (4.0, 3.0, 4.0)),
    },
}


def fov_tangents(fx, cx_o3d, fy, cy, width, height):
    """Descriptor FOV tangents (l, r, t, b) that reproduce (fx, fy, cx_o3d, cy) after the cx flip."""
    return cx_o3d / fx, (width - cx_o3d) / fx, cy / fy, (height - cy) / fy


def look_at(eye, target, up=(0.0, 1.0, 0.0)):
    """Open3D camera->world rotation: columns = camera x (right), y (down), z (forward)."""
    eye, target, up = (np.asarray(a, dtype=np.float64) for a in (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    return np.stack([r, d, f], axis=1)


def sphere_ring_poses(n, radius=1.5, height=0.2, target=(0.0, 0.0, 0.0)):
    poses = []
    for i in range(n):
        a = 2 * np.pi * i / n
        eye = np.array([radius * np.cos(a), height, radius * np.sin(a)])
        poses.append((look_at(eye, target), eye))
    return poses


def room_loop_poses(n, radius=0.5, height=1.6, sweep_deg=60.0, sweeps=4, pitch_deg=-12.0, center=(0.0, 0.0)):
    """Closed walk around the room centre looking across it; yaw sweeps +-sweep_deg."""
    poses = []
    for i in range(n):
        a = 2 * np.pi * i / n
        eye = np.array([center[0] + radius * np.cos(a), height, center[1] + radius * np.sin(a)])
        yaw = a + np.pi + np.deg2rad(sweep_deg) * np.sin(sweeps * a)
        pitch = np.deg2rad(pitch_deg)
        fwd = np.array([np.cos(yaw) * np.cos(pitch), np.sin(pitch), np.sin(yaw) * np.cos(pitch)])
        poses.append((look_at(eye, eye + fwd), eye))
    return poses


def render_depth(scene, K, R, t, height, width):
    """Analytic z-depth (float32, 0 = no hit) at integer pixel coordinates (Open3D pinhole)."""
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    v, u = np.mgrid[0:height, 0:width]
    dc = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u, dtype=np.float64)], axis=-1).reshape(-1, 3)
    d = dc @ np.asarray(R).T  # world directions (camera z component == 1 -> param == z depth)
    o = np.asarray(t, dtype=np.float64)
    best = np.full(d.shape[0], np.inf)
    for c, r in scene["spheres"]:
        oc = o - np.asarray(c)
        a = np.einsum("ij,ij->i", d, d)
        b = 2 * d @ oc
        cc = oc @ oc - r * r
        disc = b * b - 4 * a * cc
        ok = disc >= 0
        sq = np.sqrt(np.where(ok, disc, 0))
        s0 = (-b - sq) / (2 * a)
        s1 = (-b + sq) / (2 * a)
        s = np.where(s0 > 1e-6, s0, np.where(s1 > 1e-6, s1, np.inf))
        best = np.minimum(best, np.where(ok, s, np.inf))
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        for lo, hi in scene["boxes"]:
            t0 = (np.asarray(lo) - o) * inv
            t1 = (np.asarray(hi) - o) * inv
            tn = np.nanmax(np.minimum(t0, t1), axis=1)
            tf = np.nanmin(np.maximum(t0, t1), axis=1)
            hit = (tf >= tn) & (tn > 1e-6)
            best = np.minimum(best, np.where(hit, tn, np.inf))
        if scene["room"] is not None:
            lo, hi = scene["room"]
            t0 = (np.asarray(lo) - o) * inv
            t1 = (np.asarray(hi) - o) * inv
            tf = np.nanmin(np.maximum(t0, t1), axis=1)
            best = np.minimum(best, np.where(tf > 1e-6, tf, np.inf))
    z = np.where(np.isfinite(best), best, 0.0)
    return z.reshape(height, width).astype(np.float32)


def render_depth_torch(scene, K, poses, height, width, device="cuda"):
    """Batched torch version of render_depth (float64 on the GPU; synthetic-input generation only).

    Returns (N,H,W) float32 torch tensor on `device`."""
    import torch
    fx, fy, cx, cy = (float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]))
    v, u = torch.meshgrid(torch.arange(height, device=device, dtype=torch.float64),
                          torch.arange(width, device=device, dtype=torch.float64), indexing="ij")
    dc = torch.stack([(u - cx) / fx, (v - cy) / fy, torch.ones_like(u)], dim=-1).reshape(-1, 3)
    out = torch.empty((len(poses), height, width), dtype=torch.float32, device=device)
    inf = torch.tensor(float("inf"), dtype=torch.float64, device=device)
    for i, (R, t) in enumerate(poses):
        d = dc @ torch.as_tensor(np.asarray(R).T, dtype=torch.float64, device=device)
        o = torch.as_tensor(np.asarray(t), dtype=torch.float64, device=device)
        best = torch.full((d.shape[0],), float("inf"), dtype=torch.float64, device=device)
        a = (d * d).sum(1)
        for c, r in scene["spheres"]:
            oc = o - torch.as_tensor(c, dtype=torch.float64, device=device)
            b = 2 * d @ oc
            cc = oc @ oc - r * r
            disc = b * b - 4 * a * cc
            ok = disc >= 0
            sq = torch.sqrt(torch.clamp(disc, min=0))
            s0 = (-b - sq) / (2 * a)
            s1 = (-b + sq) / (2 * a)
            s = torch.where(s0 > 1e-6, s0, torch.where(s1 > 1e-6, s1, inf))
            best = torch.minimum(best, torch.where(ok, s, inf))
        inv = 1.0 / d
        for lo, hi in scene["boxes"]:
            t0 = (torch.as_tensor(lo, dtype=torch.float64, device=device) - o) * inv
            t1 = (torch.as_tensor(hi, dtype=torch.float64, device=device) - o) * inv
            tn = torch.nan_to_num(torch.minimum(t0, t1), nan=-float("inf")).amax(1)
            tf = torch.nan_to_num(torch.maximum(t0, t1), nan=float("inf")).amin(1)
            hit = (tf >= tn) & (tn > 1e-6)
            best = torch.minimum(best, torch.where(hit, tn, inf))
        if scene["room"] is not None:
            lo, hi = scene["room"]
            t0 = (torch.as_tensor(lo, dtype=torch.float64, device=device) - o) * inv
            t1 = (torch.as_tensor(hi, dtype=torch.float64, device=device) - o) * inv
            tf = torch.nan_to_num(torch.maximum(t0, t1), nan=float("inf")).amin(1)
            best = torch.minimum(best, torch.where(tf > 1e-6, tf, inf))
        out[i] = torch.where(torch.isfinite(best), best, torch.zeros_like(best)).reshape(height, width).float()
    return out


def hall_loop_poses(n, radius=2.2, height=1.6, sweep_deg=70.0, sweeps=6, pitch_deg=-15.0):
    """C5 walk: a closed loop through the hall, looking outwards and across with a yaw sweep."""
    return room_loop_poses(n, radius=radius, height=height, sweep_deg=sweep_deg, sweeps=sweeps, pitch_deg=pitch_deg)


def render_color_torch(scene, K, poses, height, width, device="cuda"):
    """(N,H,W,3) uint8 colour frames (texture() at the ray hits, black on a miss) on `device`."""
    import torch
    z = render_depth_torch(SCENES[scene] if isinstance(scene, str) else scene, K, poses, height, width, device)
    z = z.double()
    fx, fy, cx, cy = (float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]))
    v, u = torch.meshgrid(torch.arange(height, device=device, dtype=torch.float64),
                          torch.arange(width, device=device, dtype=torch.float64), indexing="ij")
    dc = torch.stack([(u - cx) / fx, (v - cy) / fy, torch.ones_like(u)], dim=-1)
    out = torch.empty((len(poses), height, width, 3), dtype=torch.uint8, device=device)
    for i, (R, t) in enumerate(poses):
        Rt = torch.as_tensor(np.asarray(R).T, dtype=torch.float64, device=device)
        pw = (dc * z[i][..., None]) @ Rt + torch.as_tensor(np.asarray(t), dtype=torch.float64, device=device)
        rgb = torch.stack([0.5 + 0.5 * torch.sin(7.0 * pw[..., 0] + 1.0), 0.5 + 0.5 * torch.sin(5.0 * pw[..., 1] + 2.0),
                           0.5 + 0.5 * torch.sin(3.0 * pw[..., 2] + 3.0)], dim=-1)
        rgb = torch.where((z[i] > 0)[..., None], rgb, torch.zeros_like(rgb))
        out[i] = torch.clamp(torch.round(rgb * 255.0), 0, 255).to(torch.uint8)
    return out


def make_sequence_fast(scene="room", poses=None, n=500, height=480, width=640, f=525.0, noise=True, seed=0,
                       near=NEAR, far=FAR, device="cuda"):
    """make_sequence for benchmark-sized inputs: GPU (torch) ray casting, same decode/pose path.

    Noise comes from a torch generator (so it differs from make_sequence's numpy stream)."""
    import torch
    cx_o3d, cy = (width - 1) / 2.0, (height - 1) / 2.0
    l, r, t, b = fov_tangents(f, cx_o3d, f, cy, width, height)
    fx, fy = width / (r + l), height / (t + b)
    cx_desc, cy_desc = width * r / (r + l), height * t / (t + b)
    K64 = np.array([[fx, 0, width - cx_desc], [0, fy, cy_desc], [0, 0, 1]])
    if poses is None:
        poses = sphere_ring_poses(n) if scene == "sphere" else room_loop_poses(n)
    z = render_depth_torch(SCENES[scene], K64, poses, height, width, device).double()
    if noise:
        g = torch.Generator(device=device).manual_seed(seed)
        noisy = z + torch.randn(z.shape, generator=g, device=device, dtype=torch.float64) * 0.002 * z
        drop = torch.rand(z.shape, generator=g, device=device) < 0.01
        z = torch.where((z > 0) & ~drop & (noisy > 0), noisy, torch.zeros_like(z))
    # encode to the Quest NDC buffer and decode exactly like the reference loader
    x, y = (-2.0 * near, -1.0) if np.isinf(far) or far < near else (-2.0 * far * near / (far - near),
                                                                        -(far + near) / (far - near))
    ndc = torch.where(z > 0, x / torch.where(z > 0, z, torch.ones_like(z)) - y, torch.ones_like(z))
    raw = torch.clamp((ndc + 1.0) * 0.5, 0.0, 1.0).float()
    ndc32 = raw * 2.0 - 1.0
    denom = ndc32 + np.float32(y)
    depth = torch.where(denom != 0, np.float32(x) / torch.where(denom != 0, denom, torch.ones_like(denom)),
                        torch.zeros_like(denom)).float()
    unity = o3d_poses_to_unity(poses)
    o3d = unity.convert_coordinate_system(CoordinateSystem.OPEN3D, is_camera=True)
    K = np.zeros((len(poses), 3, 3), np.float32)
    K[:, 0, 0], K[:, 1, 1], K[:, 2, 2] = fx, fy, 1.0
    K[:, 0, 2], K[:, 1, 2] = cx_desc, cy_desc
    K[:, 0, 2] = width - K[:, 0, 2]
    return {"depth_t": depth, "raw_t": raw, "K": K, "T_wc": o3d.extrinsics_wc, "T_cw": o3d.extrinsics_cw,
            "unity": unity, "tangents": (l, r, t, b), "near": near, "far": far, "width": width, "height": height}


def texture(points):
    """Analytic RGB texture of the procedural scenes at world points (..., 3) -> (..., 3) in [0, 1]."""
    p = np.asarray(points, np.float64)
    return np.stack([0.5 + 0.5 * np.sin(7.0 * p[..., 0] + 1.0), 0.5 + 0.5 * np.sin(5.0 * p[..., 1] + 2.0),
                     0.5 + 0.5 * np.sin(3.0 * p[..., 2] + 3.0)], axis=-1)


def render_color(scene, K, R, t, height, width):
    """uint8 RGB colour frame of `scene` from an Open3D camera (R cam->world, t eye), texture() at
    each pixel's hit point (black where nothing is hit); same pinhole model as render_depth."""
    z = render_depth(SCENES[scene] if isinstance(scene, str) else scene, K, R, t, height, width).astype(np.float64)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    v, u = np.mgrid[0:height, 0:width]
    dc = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u, dtype=np.float64)], axis=-1)
    pw = (dc * z[..., None]) @ np.asarray(R).T + np.asarray(t)
    rgb = np.where((z > 0)[..., None], texture(pw), 0.0)
    return np.clip(np.round(rgb * 255.0), 0, 255).astype(np.uint8)


def corrupt(z, rng, sigma_rel=0.002, dropout=0.01):
    z = z.astype(np.float64)
    noisy = z + rng.standard_normal(z.shape) * sigma_rel * z
    drop = rng.random(z.shape) < dropout
    return np.where((z > 0) & ~drop & (noisy > 0), noisy, 0.0).astype(np.float32)


def o3d_poses_to_unity(poses) -> Transforms:
    """Open3D camera->world poses -> the UNITY Transforms the Quest descriptor CSV stores."""
    rots = np.stack([R for R, _ in poses])
    pos = np.stack([t for _, t in poses])
    t_o3d = Transforms(CoordinateSystem.OPEN3D, pos, Rotation.from_matrix(rots).as_quat())
    return t_o3d.convert_coordinate_system(CoordinateSystem.UNITY, is_camera=True)


def make_sequence(scene="room", n=32, height=480, width=640, f=525.0, noise=True, seed=0, poses=None,
                  near=NEAR, far=FAR, side_offset=None):
    """In-memory capture as the fusion path sees it.

    Returns dict: raw (N,H,W) f32 NDC buffers, depth (N,H,W) f32 metric (decoded like the
    reference), K (N,3,3) f32 Open3D intrinsics (cx flipped), T_wc / T_cw (N,4,4) f32,
    unity (Transforms in UNITY), tangents (l, r, t, b), near, far.
    """
    sc = SCENES[scene]
    cx_o3d, cy = (width - 1) / 2.0, (height - 1) / 2.0
    l, r, t, b = fov_tangents(f, cx_o3d, f, cy, width, height)
    fx = width / (r + l)
    fy = height / (t + b)
    cx_desc = width * r / (r + l)
    cy_desc = height * t / (t + b)
    K64 = np.array([[fx, 0, width - cx_desc], [0, fy, cy_desc], [0, 0, 1]])
    if poses is None:
        poses = sphere_ring_poses(n) if scene == "sphere" else room_loop_poses(n)
    if side_offset is not None:  # stereo baseline along camera x
        poses = [(R, t + R[:, 0] * side_offset) for R, t in poses]
    rng = np.random.default_rng(seed)
    raws = np.empty((len(poses), height, width), np.float32)
    for i, (R, tt) in enumerate(poses):
        z = render_depth(sc, K64, R, tt, height, width)
        if noise:
            z = corrupt(z, rng)
        raws[i] = encode_linear_to_ndc(z, near, far)
    depth = np.stack([convert_depth_to_linear(x, near, far) for x in raws])
    unity = o3d_poses_to_unity(poses)
    o3d = unity.convert_coordinate_system(CoordinateSystem.OPEN3D, is_camera=True)
    K = np.zeros((len(poses), 3, 3), np.float32)
    K[:, 0, 0] = fx
    K[:, 1, 1] = fy
    K[:, 2, 2] = 1.0
    K[:, 0, 2] = cx_desc
    K[:, 1, 2] = cy_desc
    K[:, 0, 2] = width - K[:, 0, 2]  # compute_o3d_intrinsic_matrices' cx flip (o3d_utils.py:14-19)
    return {"raw": raws, "depth": depth, "K": K, "T_wc": o3d.extrinsics_wc, "T_cw": o3d.extrinsics_cw,
            "unity": unity, "tangents": (l, r, t, b), "near": near, "far": far, "width": width, "height": height}


def write_capture(project_dir, seq, side_value="left", t0=1_000_000, dt=33):
    """Write a sequence in the reference's capture layout (raw files + descriptor CSV)."""
    import pandas as pd
    project_dir = Path(project_dir)
    ddir = project_dir / f"{side_value}_depth"
    ddir.mkdir(parents=True, exist_ok=True)
    l, r, t, b = seq["tangents"]
    rows = []
    for i in range(seq["raw"].shape[0]):
        ts = t0 + i * dt
        seq["raw"][i].astype("<f4").tofile(ddir / f"{ts}.raw")
        p, q = seq["unity"].positions[i], seq["unity"].rotations[i]
        rows.append({"timestamp_ms": ts, "width": seq["width"], "height": seq["height"], "near_z": seq["near"],
                     "far_z": seq["far"], "fov_left_angle_tangent": l, "fov_right_angle_tangent": r,
                     "fov_top_angle_tangent": t, "fov_down_angle_tangent": b,
                     "create_pose_location_x": p[0], "create_pose_location_y": p[1], "create_pose_location_z": p[2],
                     "create_pose_rotation_x": q[0], "create_pose_rotation_y": q[1], "create_pose_rotation_z": q[2],
                     "create_pose_rotation_w": q[3]})
    pd.DataFrame(rows).to_csv(project_dir / f"{side_value}_depth_descriptors.csv", index=False)
    return project_dir
