"""``VoxelBlockGrid`` -- HBM-resident voxel-block TSDF volume on one MI355X.

Drop-in for the ``o3d.t.geometry.VoxelBlockGrid`` surface the reference uses
(scripts/processing/reconstruction/utils/o3d_utils.py:170-229, reconstruct_scene.py:90-108,
refine_fragment_poses.py:39, reconstruction_data_io.py:42-55):

    VoxelBlockGrid(attr_names=('tsdf','weight'), attr_dtypes=(f32,f32), attr_channels=((1),(1)),
                   voxel_size, block_resolution, block_count, device)
    .compute_unique_block_coordinates(depth, intrinsic, extrinsic, depth_scale, depth_max,
                                      trunc_voxel_multiplier) -> (N,3) int32 block keys
    .integrate(block_coords, depth, intrinsic, extrinsic, depth_scale, depth_max, trunc_voxel_multiplier)
    .extract_point_cloud(weight_threshold=3.0, estimated_point_number=-1)
    .extract_triangle_mesh(weight_threshold=3.0, estimated_vertex_number=-1)
    .save(path) / VoxelBlockGrid.load(path)

plus ``integrate_frames`` (the batched whole-loop entry used by ``mqr.o3d_utils.integrate``).
Every call goes through libmqr_hip.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import MQR_DEVICE, MQR_DEVICE_RESIDENT, MQR_HOST, MqrStats, call, ptr
from .geometry import Image, PointCloud, Tensor, TriangleMesh

# Open3D defaults for the keyword arguments the reference relies on.
_O3D_DEPTH_SCALE = 1000.0
_O3D_DEPTH_MAX = 3.0
_O3D_TRUNC = 8.0


def parse_device(device) -> int:
    """'CUDA:0' / 'HIP:0' / 'cuda:1' / 0 / o3d.core.Device -> HIP device index.

    The reference's default is 'CPU:0' (config/pipeline_config.yml:14); this framework always
    runs the fusion path on the GPU, so 'CPU:n' maps to HIP device 0."""
    if device is None:
        return 0
    if isinstance(device, (int, np.integer)):
        return int(device)
    s = str(device).strip()
    if hasattr(device, "get_id") and hasattr(device, "get_type"):
        s = f"{device.get_type()}:{device.get_id()}"
    s = s.replace("Device(", "").replace(")", "")
    if ":" in s:
        kind, idx = s.rsplit(":", 1)
        if kind.strip().upper().endswith("CPU"):
            return 0
        try:
            return int(idx)
        except ValueError:
            return 0
    return 0


def _depth_array(depth) -> np.ndarray:
    if isinstance(depth, Image):
        return depth.numpy()
    if hasattr(depth, "as_tensor"):
        depth = depth.as_tensor()
    if hasattr(depth, "numpy"):
        depth = depth.numpy()
    a = np.ascontiguousarray(depth, dtype=np.float32)
    if a.ndim == 3 and a.shape[2] == 1:
        a = np.ascontiguousarray(a[:, :, 0])
    if a.ndim != 2:
        raise ValueError(f"depth must be H x W, got shape {a.shape}")
    return a


def _mat(m, shape) -> np.ndarray:
    if hasattr(m, "numpy"):
        m = m.numpy()
    a = np.ascontiguousarray(m, dtype=np.float64)
    if a.shape != shape:
        raise ValueError(f"expected matrix of shape {shape}, got {a.shape}")
    return a


# Released grids kept for reuse: creating and destroying a grid (its HBM pool and hash table, its streams)
# cost ~2.6 ms per fresh volume, which the fragment path pays once per 100 frames (tools/fragment_probe.py).
# A released grid that never grew is reset (the state of a new grid, mqr_vbg_reset) and handed to the next
# VoxelBlockGrid of the same voxel size, resolution, block count and device.  Budget per process: at most
# SPARE_GRIDS kept in total, only grids whose pool is at most SPARE_MAX_BYTES (the reference's default
# 50 000-block grid at R = 16 is 1.64 GB; a large volume's HBM is not held back), and only while at least
# SPARE_MIN_FREE of the device's HBM stays free (hipMemGetInfo).  A create that fails while spares are
# held releases them and tries once more.  A 4-process fragment pool on one GPU thus holds <= 8 GiB.
SPARE_GRIDS = 1
SPARE_MAX_BYTES = 2 << 30
SPARE_MIN_FREE = 0.25
_spares = []  # [(key, handle)]
_spares_lock = threading.Lock()


def _hbm_headroom(device) -> bool:
    """At least SPARE_MIN_FREE of `device`'s HBM is free (a spare grid is kept only then)."""
    free, total = ctypes.c_int64(), ctypes.c_int64()
    if _lib._lib.mqr_device_mem_info(int(device), ctypes.byref(free), ctypes.byref(total)) != 0 or total.value <= 0:
        return False
    return free.value >= SPARE_MIN_FREE * total.value


def release_spare_grids():
    """Destroy the kept released grids (their HBM is freed)."""
    with _spares_lock:
        hs = [h for _, h in _spares]
        _spares.clear()
    for h in hs:
        _lib._lib.mqr_vbg_destroy(h)


class VoxelBlockGrid:
    def __init__(self, attr_names=("tsdf", "weight"), attr_dtypes=None, attr_channels=None, voxel_size=0.01,
                 block_resolution=16, block_count=50_000, device=None):
        names = tuple(attr_names)
        if names != ("tsdf", "weight"):
            raise NotImplementedError(f"only attr_names=('tsdf','weight') is supported (the reference's "
                                      f"o3d_utils.py:172 layout), got {names}")
        self.voxel_size = float(voxel_size)
        self.block_resolution = int(block_resolution)
        self.device = device
        self.device_id = parse_device(device)
        self._key = (self.voxel_size, self.block_resolution, int(block_count), self.device_id)
        with _spares_lock:
            i = next((j for j, (k, _) in enumerate(_spares) if k == self._key), None)
            h = _spares.pop(i)[1] if i is not None else None
        if h is None:
            h = ctypes.c_void_p()
            try:
                call("mqr_vbg_create", self.voxel_size, self.block_resolution, int(block_count), self.device_id,
                     ctypes.byref(h))
            except _lib.MqrError:
                with _spares_lock:
                    held = bool(_spares)
                if not held:
                    raise
                release_spare_grids()  # their HBM may be what the new grid lacks
                h = ctypes.c_void_p()
                call("mqr_vbg_create", self.voxel_size, self.block_resolution, int(block_count), self.device_id,
                     ctypes.byref(h))
        self._h = h

    # -- lifetime -----------------------------------------------------------------------------
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is None or not h.value or _lib._lib is None:
            return
        self._h = None
        try:  # (at interpreter exit the module's globals may already be gone: then just destroy)
            key = None if getattr(self, "_profiled", False) else getattr(self, "_key", None)
            cap = ctypes.c_int64(-1)
            # (the integrate configuration back to a new grid's default, then emptied)
            if (key is not None and SPARE_GRIDS > 0 and key[2] * key[1] ** 3 * 8 <= SPARE_MAX_BYTES
                    and _hbm_headroom(key[3])
                    and _lib._lib.mqr_vbg_capacity(h, ctypes.byref(cap)) == 0
                    and cap.value == key[2] and _lib._lib.mqr_vbg_set_variant(h, 0) == 0
                    and _lib._lib.mqr_vbg_reset(h) == 0):
                with _spares_lock:
                    if len(_spares) < SPARE_GRIDS:
                        _spares.append((key, h))
                        return
        except Exception:  # noqa: BLE001
            pass
        _lib._lib.mqr_vbg_destroy(h)

    @property
    def handle(self):
        return self._h

    def reset(self):
        """Empty the grid in place (same state as a new grid, allocations kept)."""
        call("mqr_vbg_reset", self._h)

    def export_keys(self) -> np.ndarray:
        n = self.size()
        keys = np.empty((n, 3), np.int32)
        if n:
            call("mqr_vbg_export", self._h, ptr(keys), None, None, MQR_HOST)
        return keys

    def pack_weighted(self, union_keys_dev_ptr, U, out_dev_ptr):
        """[U][R^3][2] (w*tsdf, w) float32 into device memory, zeros for absent blocks."""
        call("mqr_vbg_pack_weighted", self._h, ctypes.c_void_p(union_keys_dev_ptr), int(U),
             ctypes.c_void_p(out_dev_ptr))

    def unpack_weighted(self, union_keys_dev_ptr, U, in_dev_ptr):
        """Activate the union keys and set tsdf = sum(w*tsdf)/sum(w), weight = sum(w)."""
        call("mqr_vbg_unpack_weighted", self._h, ctypes.c_void_p(union_keys_dev_ptr), int(U),
             ctypes.c_void_p(in_dev_ptr))

    def size(self) -> int:
        n = ctypes.c_int64()
        call("mqr_vbg_size", self._h, ctypes.byref(n))
        return n.value

    def capacity(self) -> int:
        n = ctypes.c_int64()
        call("mqr_vbg_capacity", self._h, ctypes.byref(n))
        return n.value

    # -- per-frame Open3D API -------------------------------------------------------------------
    def compute_unique_block_coordinates(self, depth, intrinsic, extrinsic, depth_scale=_O3D_DEPTH_SCALE,
                                         depth_max=_O3D_DEPTH_MAX, trunc_voxel_multiplier=_O3D_TRUNC):
        d = _depth_array(depth)
        H, W = d.shape
        K = _mat(intrinsic, (3, 3))
        T = _mat(extrinsic, (4, 4))
        out = np.empty((max(4 * (H // 4) * (W // 4), 1), 3), np.int32)
        n = ctypes.c_int64()
        call("mqr_touch", self._h, ptr(d), MQR_HOST, H, W, ptr(K, _lib._f64p), ptr(T, _lib._f64p),
             float(depth_scale), float(depth_max), float(trunc_voxel_multiplier), ptr(out, _lib._i32p),
             ctypes.byref(n))
        return Tensor(out[: n.value].copy())

    def integrate(self, block_coords, depth, intrinsic, extrinsic=None, depth_scale=_O3D_DEPTH_SCALE,
                  depth_max=_O3D_DEPTH_MAX, trunc_voxel_multiplier=_O3D_TRUNC):
        keys = np.ascontiguousarray(block_coords.numpy() if hasattr(block_coords, "numpy") else block_coords,
                                    dtype=np.int32).reshape(-1, 3)
        d = _depth_array(depth)
        H, W = d.shape
        K = _mat(intrinsic, (3, 3))
        T = _mat(extrinsic, (4, 4))
        call("mqr_integrate", self._h, ptr(keys, _lib._i32p), keys.shape[0], ptr(d), MQR_HOST, H, W,
             ptr(K, _lib._f64p), ptr(T, _lib._f64p), float(depth_scale), float(depth_max),
             float(trunc_voxel_multiplier))

    # -- batched whole-sequence entry ---------------------------------------------------------------
    def integrate_frames(self, depths, intrinsics, extrinsics, frame_ok=None, depth_scale=1.0, depth_max=3.0,
                         trunc_voxel_multiplier=8.0, resident=False):
        """touch + integrate for every frame in order (== sequential per-frame calls, bit for bit).

        depths: (B,H,W) float32 host array, or an ``_lib.DeviceBuffer`` holding B*H*W floats (then
        pass ``depths=(buffer, B, H, W)``); intrinsics (B,3,3), extrinsics (B,4,4) world->camera.
        resident=True (device frames only): the caller keeps the frames allocated and unchanged until it
        synchronizes the device (MQR_DEVICE_RESIDENT, include/mqr.h), so its stream does not wait for the
        call's integrates and the next call's first touch can overlap them."""
        if isinstance(depths, tuple):
            buf, B, H, W = depths
            dptr, loc = buf.ptr, (MQR_DEVICE_RESIDENT if resident else MQR_DEVICE)
            keep = None
        else:
            keep = np.ascontiguousarray(depths, dtype=np.float32)
            B, H, W = keep.shape
            dptr, loc = ptr(keep), MQR_HOST
        K = np.ascontiguousarray(intrinsics, dtype=np.float64).reshape(B, 3, 3)
        T = np.ascontiguousarray(extrinsics, dtype=np.float64).reshape(B, 4, 4)
        ok = None if frame_ok is None else np.ascontiguousarray(frame_ok, dtype=np.uint8)
        call("mqr_integrate_frames", self._h, dptr, loc, B, H, W, ptr(K, _lib._f64p), ptr(T, _lib._f64p),
             None if ok is None else ptr(ok, _lib._u8p), float(depth_scale), float(depth_max),
             float(trunc_voxel_multiplier))
        del keep

    # -- extraction --------------------------------------------------------------------------------
    def _geom(self, fn, thr):
        """The extraction's result, left in HBM (DeviceGeom): host arrays are copied on first access."""
        from .geometry import DeviceGeom
        g = ctypes.c_void_p()
        try:
            call(fn, self._h, float(thr), ctypes.byref(g))
        except _lib.MqrError:
            if g.value:  # a failed extraction may still have handed out its result object
                _lib._lib.mqr_geom_free(g)
            raise
        try:
            return DeviceGeom(g, self.device_id)
        except Exception:
            _lib._lib.mqr_geom_free(g)
            raise

    def extract_point_cloud(self, weight_threshold=3.0, estimated_point_number=-1):
        """Open3D returns the cloud on the volume's device; so does this (positions / normals in HBM,
        copied to the host on first host access)."""
        return PointCloud.from_device(self._geom("mqr_extract_points", weight_threshold), device=self.device)

    def extract_triangle_mesh(self, weight_threshold=3.0, estimated_vertex_number=-1):
        """The mesh on the volume's device, as Open3D returns it (arrays in HBM until a host access)."""
        return TriangleMesh.from_device(self._geom("mqr_extract_mesh", weight_threshold), device=self.device)

    # -- contents ----------------------------------------------------------------------------------
    def export(self):
        """(keys (N,3) int32, tsdf (N,R,R,R) f32, weight (N,R,R,R) f32) in buffer order."""
        n = self.size()
        R = self.block_resolution
        keys = np.empty((n, 3), np.int32)
        tsdf = np.empty((n, R, R, R), np.float32)
        wgt = np.empty((n, R, R, R), np.float32)
        if n:
            call("mqr_vbg_export", self._h, ptr(keys), ptr(tsdf), ptr(wgt), MQR_HOST)
        return keys, tsdf, wgt

    def import_blocks(self, keys, tsdf, weight):
        keys = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        tsdf = np.ascontiguousarray(tsdf, dtype=np.float32)
        weight = np.ascontiguousarray(weight, dtype=np.float32)
        call("mqr_vbg_import", self._h, ptr(keys), ptr(tsdf), ptr(weight), keys.shape[0], MQR_HOST)

    def save(self, file_name):
        """npz with Open3D's VoxelBlockGrid::Save keys: voxel_size, block_resolution, key, tsdf, weight."""
        keys, tsdf, wgt = self.export()
        R = self.block_resolution
        np.savez(file_name, voxel_size=np.array([self.voxel_size], np.float32),
                 block_resolution=np.array([R], np.int64), key=keys,
                 tsdf=tsdf.reshape(-1, R, R, R, 1), weight=wgt.reshape(-1, R, R, R, 1))

    @staticmethod
    def load(file_name, device=None):
        data = np.load(file_name, allow_pickle=False)
        R = int(np.asarray(data["block_resolution"]).reshape(-1)[0])
        keys = np.asarray(data["key"], np.int32).reshape(-1, 3)
        vbg = VoxelBlockGrid(voxel_size=float(np.asarray(data["voxel_size"]).reshape(-1)[0]), block_resolution=R,
                             block_count=max(len(keys), 1), device=device)
        if len(keys):
            vbg.import_blocks(keys, np.asarray(data["tsdf"]).reshape(-1, R, R, R),
                              np.asarray(data["weight"]).reshape(-1, R, R, R))
        return vbg

    # -- profiling ---------------------------------------------------------------------------------
    def profile(self, enable=True, touch=False):
        """Per-launch timing events (stats()['integrate_ms']); touch=True also times the touch launches."""
        call("mqr_vbg_profile", self._h, (2 if touch else 1) if enable else 0)
        self._profiled = True  # (its timing state stays with it: not kept for reuse)

    def stats(self, reset=False) -> dict:
        s = MqrStats()
        call("mqr_vbg_stats", self._h, ctypes.byref(s), 1 if reset else 0)
        return {k: getattr(s, k) for k, _ in MqrStats._fields_}
