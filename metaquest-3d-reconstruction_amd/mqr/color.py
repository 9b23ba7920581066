"""Per-vertex colour projection from colour keyframes.

The reference colours the extracted mesh with Open3D's colour-map pipeline
(processing/reconstruction/color_map_optimization/optimize_color_pose.py:24-73): the filtered
mesh goes into a RaycastingScene, every colour keyframe gets a colour-aligned depth map from
``raycast_in_color_view`` (utils/o3d_utils.py:324-341), and ``run_rigid_optimizer`` assigns vertex
colours by visibility-tested averaging (upstream ColorMapUtils.cpp) while it refines the poses.
The pose optimisation stays OUT of scope; this module is the colour assignment
with the keyframe poses as given (run_rigid_optimizer at maximum_iteration = 0):

    colors, counts = color_map(vertices, images, t_hit, K, T_wc)      # complete upstream semantics
    colors, counts = project_vertex_colors(mesh, images, K, T_wc)     # ray casts t_hit first
    colors, counts = color_vertices(vertices, images, depths, K, T_wc)  # visibility + average only

color_map adds what run_rigid_optimizer does around the averaging (upstream ColorMapUtils /
RigidOptimizer / Image.cpp, recalled -- VERIFY): the RGBD depth truncated at 3 m
(create_from_color_and_depth), depth-discontinuity masks (Sobel > 0.1, dilated by 3 px), float64
means, and the mean of the 3 nearest sampled vertices for vertices no keyframe samples.  All on the
GPU (libmqr_hip.so: color.hip; raycast.hip for the depths).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MQR_HOST, call, ptr

# Open3D RigidOptimizerOption defaults (maximum_allowable_depth, depth_threshold_for_visibility_check,
# image_boundary_margin)
MAX_DEPTH = 2.5
VISIBILITY_THRESHOLD = 0.03
MARGIN = 10
# ... depth_threshold_for_discontinuity_check, half_dilation_kernel_size_for_discontinuity_map,
# invisible_vertex_color_knn; and RGBDImage.create_from_color_and_depth's default depth_trunc
DISCONTINUITY_THRESHOLD = 0.1
HALF_DILATION = 3
KNN = 3
DEPTH_TRUNC = 3.0


def color_vertices(vertices, images, depths, K, T_wc, max_depth=MAX_DEPTH,
                   visibility_threshold=VISIBILITY_THRESHOLD, margin=MARGIN, device=0):
    """vertices (V,3) float32; images (N,H,W,3) uint8 RGB; depths (N,H,W) float32 colour-aligned
    depth; K (N,3,3), T_wc (N,4,4) world->camera.  Returns (colours (V,3) float32 in [0,1],
    counts (V,) int32 = keyframes averaged)."""
    V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
    im = np.ascontiguousarray(images, dtype=np.uint8)
    if im.ndim != 4 or im.shape[3] != 3:
        raise ValueError(f"images must be (N,H,W,3) uint8, got {im.shape}")
    N, H, W = im.shape[:3]
    d = np.ascontiguousarray(depths, dtype=np.float32).reshape(N, H, W)
    Kd = np.ascontiguousarray(K, dtype=np.float64).reshape(N, 9)
    Td = np.ascontiguousarray(T_wc, dtype=np.float64).reshape(N, 16)
    out = np.empty((len(V), 3), np.float32)
    cnt = np.empty(len(V), np.int32)
    call("mqr_color_vertices", int(device), ptr(V), len(V), MQR_HOST, ptr(im), ptr(d), MQR_HOST, N, H, W,
         ptr(Kd, _lib._f64p), ptr(Td, _lib._f64p), float(max_depth), float(visibility_threshold), int(margin),
         ptr(out), ptr(cnt), MQR_HOST)
    return out, cnt


def color_map(vertices, images, t_hit, K, T_wc, max_depth=MAX_DEPTH, visibility_threshold=VISIBILITY_THRESHOLD,
              margin=MARGIN, discontinuity_threshold=DISCONTINUITY_THRESHOLD, half_dilation=HALF_DILATION,
              depth_trunc=DEPTH_TRUNC, knn=KNN, device=0):
    """run_rigid_optimizer's vertex colours with the poses as given.  t_hit (N,H,W) float32: the
    keyframes' raycast_in_color_view depth (inf on a miss).  Returns (colours (V,3) float32,
    counts (V,) int32 = keyframes averaged; 0 where the colour comes from the knn fill).  Vertices and
    t_hit already in HBM on `device` (a mesh from this package's extraction, a cast's t_hit Tensor) are
    used in place."""
    from .geometry import device_ptr
    from ._lib import MQR_DEVICE, DeviceBuffer
    im = np.ascontiguousarray(images, dtype=np.uint8)
    if im.ndim != 4 or im.shape[3] != 3:
        raise ValueError(f"images must be (N,H,W,3) uint8, got {im.shape}")
    N, H, W = im.shape[:3]
    dv = device_ptr(vertices, device) if getattr(vertices, "dtype", None) == np.float32 else None
    if dv is not None and vertices.shape[-1:] == (3,):
        nv, vptr, vloc = int(np.prod(vertices.shape[:-1])), ctypes.c_void_p(dv[0]), MQR_DEVICE
    else:
        V = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        nv, vptr, vloc = len(V), ptr(V), MQR_HOST
    dt = device_ptr(t_hit, device) if getattr(t_hit, "dtype", None) == np.float32 else None
    keep = None
    if dt is not None and int(np.prod(t_hit.shape)) == N * H * W:  # images go up beside the resident depths
        keep = DeviceBuffer.from_array(im, int(device))
        iptr, tptr, iloc = keep.ptr, ctypes.c_void_p(dt[0]), MQR_DEVICE
    else:
        d = np.ascontiguousarray(t_hit, dtype=np.float32).reshape(N, H, W)
        iptr, tptr, iloc = ptr(im), ptr(d), MQR_HOST
    Kd = np.ascontiguousarray(K, dtype=np.float64).reshape(N, 9)
    Td = np.ascontiguousarray(T_wc, dtype=np.float64).reshape(N, 16)
    out = np.empty((nv, 3), np.float32)
    cnt = np.empty(nv, np.int32)
    call("mqr_color_map", int(device), vptr, nv, vloc, iptr, tptr, iloc, N, H, W,
         ptr(Kd, _lib._f64p), ptr(Td, _lib._f64p), float(max_depth), float(visibility_threshold), int(margin),
         float(discontinuity_threshold), int(half_dilation), float(depth_trunc), int(knn), ptr(out), ptr(cnt), MQR_HOST)
    del keep
    return out, cnt


def project_vertex_colors(mesh, images, K, T_wc, device=0, complete=True, **kw):
    """Ray-cast each keyframe's colour-aligned depth from `mesh` (raycast_in_color_view), then colour
    the vertices: color_map (complete=True) or the visibility-and-average primitive color_vertices.
    Returns (colours, counts)."""
    from .raycasting import RaycastingScene, _device_mesh, _mesh_arrays
    im = np.asarray(images)
    N, H, W = im.shape[:3]
    scene = RaycastingScene(device=device)
    if _device_mesh(mesh, None, device) is not None:  # the mesh stays in HBM from extraction to colours
        v = mesh.vertex.positions
        scene.add_triangles(mesh)
    else:
        v, t = _mesh_arrays(mesh)
        scene.add_triangles(v, t)
    depth = scene.cast_pinhole(np.asarray(K, np.float64).reshape(N, 3, 3), np.asarray(T_wc, np.float64).reshape(N, 4, 4),
                               W, H)["t_hit"]
    if complete:
        return color_map(v, im, depth, K, T_wc, device=device, **kw)
    return color_vertices(v, im, depth.numpy(), K, T_wc, device=device, **kw)
