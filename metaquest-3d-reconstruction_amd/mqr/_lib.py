"""ctypes binding of libmqr_hip.so (the C ABI declared in include/mqr.h).

There is no CPU fallback: if the HIP library is missing or no MI355X is visible, the product
raises.  (The CPU restatement under oracle/ is test infrastructure only.)
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MQR_HIP_LIB", os.path.join(_HERE, "libmqr_hip.so"))

MQR_HOST = 0
MQR_DEVICE = 1
MQR_DEVICE_RESIDENT = 2  # mqr_integrate_frames: device frames kept unchanged until the caller synchronizes

_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p


class MqrStats(ctypes.Structure):
    _fields_ = [("integrate_launches", ctypes.c_int64), ("integrate_ms", ctypes.c_double),
                ("union_blocks", ctypes.c_int64), ("frame_blocks", ctypes.c_int64), ("frames", ctypes.c_int64),
                ("touch_launches", ctypes.c_int64), ("touch_ms", ctypes.c_double), ("pixels", ctypes.c_int64),
                ("table_retries", ctypes.c_int64)]


# name -> (restype, argtypes); every function returns int status
SIGNATURES = {
    "mqr_version": (ctypes.c_int, []),
    "mqr_last_error": (ctypes.c_char_p, []),
    "mqr_build_tag": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "mqr_vbg_last_kernel": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    "mqr_vbg_flips": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "mqr_vbg_last_kernel_name": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_int]),
    "mqr_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mqr_set_stream": (ctypes.c_int, [_vp]),
    "mqr_get_stream": (ctypes.c_int, [ctypes.POINTER(_vp)]),
    "mqr_device_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(_vp)]),
    "mqr_device_free": (ctypes.c_int, [ctypes.c_int, _vp]),
    "mqr_memcpy": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int]),
    "mqr_device_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "mqr_device_mem_info": (ctypes.c_int, [ctypes.c_int, _i64p, _i64p]),
    "mqr_vbg_create": (ctypes.c_int, [ctypes.c_float, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(_vp)]),
    "mqr_vbg_destroy": (ctypes.c_int, [_vp]),
    "mqr_vbg_reset": (ctypes.c_int, [_vp]),
    "mqr_vbg_size": (ctypes.c_int, [_vp, _i64p]),
    "mqr_vbg_capacity": (ctypes.c_int, [_vp, _i64p]),
    "mqr_vbg_params": (ctypes.c_int, [_vp, _f32p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "mqr_touch": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p, _f64p, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_float, _i32p, _i64p]),
    "mqr_integrate": (ctypes.c_int, [_vp, _i32p, ctypes.c_int64, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p,
                                     _f64p, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    "mqr_integrate_frames": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p,
                                            _f64p, _u8p, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    "mqr_vbg_export": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_int]),
    "mqr_vbg_import": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_int64, ctypes.c_int]),
    "mqr_vbg_pack_weighted": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp]),
    "mqr_vbg_unpack_weighted": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp]),
    "mqr_extract_points": (ctypes.c_int, [_vp, ctypes.c_float, ctypes.POINTER(_vp)]),
    "mqr_extract_mesh": (ctypes.c_int, [_vp, ctypes.c_float, ctypes.POINTER(_vp)]),
    "mqr_extract_mesh_owned": (ctypes.c_int, [_vp, ctypes.c_float, ctypes.c_int64, ctypes.POINTER(_vp)]),
    "mqr_comm_unique_id": (ctypes.c_int, [_u8p]),
    "mqr_comm_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, ctypes.POINTER(_vp)]),
    "mqr_comm_destroy": (ctypes.c_int, [_vp]),
    "mqr_reduce_rccl": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, _i64p]),
    "mqr_comm_timing": (ctypes.c_int, [_vp, _f32p]),
    "mqr_comm_counts": (ctypes.c_int, [_vp, _i64p, _i64p, _i64p]),
    "mqr_merge_local_timing": (ctypes.c_int, [_f32p, ctypes.c_int]),
    "mqr_merge_set_per_source": (ctypes.c_int, [ctypes.c_int]),
    "mqr_merge_local": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(_vp), _i64p]),
    "mqr_xchg_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                       ctypes.c_int64, ctypes.c_int, _vp, ctypes.POINTER(_vp)]),
    "mqr_xchg_counts": (ctypes.c_int, [_vp, _i64p, _i64p, _i64p, _i64p]),
    "mqr_xchg_send_segment": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int]),
    "mqr_xchg_recv_segment": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int]),
    "mqr_xchg_finish": (ctypes.c_int, [_vp, _i64p]),
    "mqr_xchg_destroy": (ctypes.c_int, [_vp]),
    "mqr_geom_counts": (ctypes.c_int, [_vp, _i64p, _i64p]),
    "mqr_geom_device_ptrs": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "mqr_geom_copy": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_int]),
    "mqr_geom_free": (ctypes.c_int, [_vp]),
    "mqr_confidence": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                      _f32p, _f32p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                      ctypes.c_double, _vp, _vp, ctypes.c_int]),
    "mqr_confidence_counts": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, _f32p, _f32p, _f32p, _u8p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_double, ctypes.c_double, _vp,
                                             ctypes.POINTER(ctypes.c_int)]),
    "mqr_confidence_stats": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _i64p]),
    "mqr_pixel_error_map": (ctypes.c_int, [ctypes.c_int, _f32p, _f32p, ctypes.c_int, ctypes.c_int, _f32p, _f32p,
                                           _f32p, _f32p, _f32p, ctypes.c_double, _f32p]),
    "mqr_write_confidence_npz": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), _vp, _vp, ctypes.c_int,
                                                ctypes.c_int, _vp, ctypes.c_int]),
    "mqr_crc32": (ctypes.c_uint32, [ctypes.c_uint32, _vp, ctypes.c_int64]),
    "mqr_write_confidence_npz_counts": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), _vp,
                                                       ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int]),
    "mqr_read_frames": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                       ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp, ctypes.c_int]),
    "mqr_read_frames_masked": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                              ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int,
                                              ctypes.c_double, ctypes.c_int, _vp, _vp, _vp, ctypes.c_int]),
    "mqr_decode_depth": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        _f64p, _f64p, _u8p, _vp, _vp, _u8p, ctypes.c_int, ctypes.c_double,
                                        ctypes.c_int, _vp, ctypes.c_int, _u8p]),
    "mqr_decode_depth_masked": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, _f64p, _f64p, _u8p, _vp, _u8p, ctypes.c_int, _vp,
                                               ctypes.c_int, _u8p]),
    "mqr_color_vertices": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p, _f64p, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int, _vp, _vp, ctypes.c_int]),
    "mqr_color_map": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p, _f64p, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_double,
                                     ctypes.c_int, _vp, _vp, ctypes.c_int]),
    "mqr_scene_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "mqr_scene_destroy": (ctypes.c_int, [_vp]),
    "mqr_scene_add_triangles": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, _vp, ctypes.c_int64, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_uint32)]),
    "mqr_scene_build": (ctypes.c_int, [_vp]),
    "mqr_scene_triangle_count": (ctypes.c_int, [_vp, _i64p]),
    "mqr_scene_cast_pinhole": (ctypes.c_int, [_vp, _f64p, _f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp,
                                              _vp, _vp, _vp, ctypes.c_int]),
    "mqr_scene_cast_rays": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int, _vp, _vp, _vp, _vp, _vp,
                                           ctypes.c_int]),
    "mqr_mesh_filter_components": (ctypes.c_int, [ctypes.c_int, _vp, _vp, ctypes.c_int64, _vp, ctypes.c_int64,
                                                  ctypes.c_int, ctypes.c_int64, ctypes.POINTER(_vp), _i64p]),
    "mqr_vbg_profile": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mqr_vbg_set_variant": (ctypes.c_int, [_vp, ctypes.c_int]),
    "mqr_check_div64": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_uint64), _f64p]),
    "mqr_check_division": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "mqr_vbg_stats": (ctypes.c_int, [_vp, ctypes.POINTER(MqrStats), ctypes.c_int]),
}

_lib = None


# mqr_read_frames status bits (include/mqr.h)
MQR_FRAME_RAW_OK, MQR_FRAME_RAW_MISSING, MQR_FRAME_RAW_OTHER = 1, 2, 4
MQR_FRAME_CONF_OK, MQR_FRAME_CONF_MISSING, MQR_FRAME_CONF_OTHER = 8, 16, 32


class MqrError(RuntimeError):
    """Raised for any non-zero status from the HIP library (Open3D raises RuntimeError too)."""

    def __init__(self, msg, code):
        super().__init__(msg)
        self.code = code


def hip_runtime_path():
    """The HIP runtime this process must use.

    libamdhip64 is bound by SONAME (libamdhip64.so.7): whichever copy is mapped first serves every
    later library that needs it.  PyTorch ships its own copy (and its own HSA runtime, loaded by
    file name), so if /opt/rocm's copy came first -- libmqr_hip.so's RUNPATH -- a later
    ``import torch`` maps a second HIP + HSA runtime and finds no device.  Mapping torch's copy first
    (when torch is installed) gives ONE runtime per process in either import order.  MQR_HIP_RUNTIME
    overrides the choice; without torch, libmqr's RUNPATH (/opt/rocm/lib) applies."""
    env = os.environ.get("MQR_HIP_RUNTIME")
    if env:
        return env
    return _torch_lib("libamdhip64.so")


def _torch_lib(name: str):
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    p = os.path.join(os.path.dirname(spec.origin), "lib", name)
    return p if os.path.exists(p) else None


_rccl_loaded = False


def preload_rccl():
    """Bring in the RCCL that torch links (when torch is installed) before libmqr resolves
    librccl.so.1 at run time: torch links it by file name, so a copy from /opt/rocm mapped first
    would be followed by a second RCCL (and ROCm SMI) instance.  It has to come in through
    ``import torch`` itself -- mapping torch's librccl.so by hand before torch's own libraries
    leaves the process with a double free at exit.  MQR_RCCL names another library instead."""
    global _rccl_loaded
    if _rccl_loaded:
        return
    if os.environ.get("MQR_RCCL"):
        ctypes.CDLL(os.environ["MQR_RCCL"], mode=ctypes.RTLD_GLOBAL)
    elif _torch_lib("librccl.so"):
        import torch  # noqa: F401
    _rccl_loaded = True


def load(path: str = LIB_PATH):
    """Load libmqr_hip.so (no compute happens here)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libmqr_hip.so not found at {path}; build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
    rt = hip_runtime_path()
    if rt:
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
    L = ctypes.CDLL(path)
    partial = os.path.abspath(path) != os.path.abspath(os.path.join(_HERE, "libmqr_hip.so"))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is None and partial:  # the A/B library (tools/_ab) carries the volume entry points only
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# Entry points that may read or write caller device buffers: before each, the thread's caller stream
# (include/mqr.h "stream ordering") is set to torch's current stream, so tensors torch is still
# writing on any stream -- the default one or a side stream under ``torch.cuda.stream(s)`` -- are
# complete before the library reads them.
ORDERED = frozenset({
    "mqr_touch", "mqr_integrate", "mqr_integrate_frames", "mqr_vbg_export", "mqr_vbg_import",
    "mqr_vbg_pack_weighted", "mqr_vbg_unpack_weighted", "mqr_xchg_create", "mqr_xchg_send_segment",
    "mqr_xchg_recv_segment", "mqr_geom_copy", "mqr_confidence", "mqr_confidence_counts", "mqr_decode_depth", "mqr_decode_depth_masked",
    "mqr_color_vertices",
    "mqr_color_map", "mqr_scene_add_triangles", "mqr_scene_cast_pinhole", "mqr_scene_cast_rays",
    "mqr_mesh_filter_components", "mqr_memcpy",
})
_tls = threading.local()


def torch_stream() -> int:
    """torch's current stream (its handle) once torch has initialised HIP in this process, else 0
    (the null stream -- nothing torch-side can be pending)."""
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return 0
    return int(torch.cuda.current_stream().cuda_stream)


def set_stream(stream: int):
    """Make `stream` (a hipStream_t handle, 0 = null stream) this thread's caller stream."""
    if getattr(_tls, "stream", None) != stream:
        rc = load().mqr_set_stream(ctypes.c_void_p(stream or None))
        if rc != 0:
            raise MqrError(f"mqr_set_stream failed ({rc})", rc)
        _tls.stream = stream


def call(name, *args):
    L = load()
    if name in ORDERED:
        set_stream(torch_stream())
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.mqr_last_error().decode(errors="replace")
        raise MqrError(f"{name} failed ({rc}): {msg}", rc)
    return rc


def build_tag(which: int) -> str:
    """Hash of the integrate (0) / confidence (1) sources compiled into the loaded library."""
    buf = ctypes.create_string_buffer(64)
    call("mqr_build_tag", int(which), buf, 64)
    return buf.value.decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    try:
        call("mqr_device_count", ctypes.byref(n))
    except MqrError:
        return 0
    return n.value


def ptr(a: np.ndarray, t=None):
    if t is None:
        return ctypes.c_void_p(a.ctypes.data)
    return a.ctypes.data_as(t)


class DeviceBuffer:
    """Raw HBM allocation owned by Python (keeps inputs resident without any framework)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device = device
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        call("mqr_device_alloc", device, max(self.nbytes, 4), ctypes.byref(p))
        self.ptr = p

    @classmethod
    def from_array(cls, a: np.ndarray, device: int = 0):
        a = np.ascontiguousarray(a)
        buf = cls(a.nbytes, device)
        call("mqr_memcpy", buf.ptr, MQR_DEVICE, ptr(a), MQR_HOST, a.nbytes, device)
        return buf

    def to_array(self, shape, dtype):
        out = np.empty(shape, dtype)
        call("mqr_memcpy", ptr(out), MQR_HOST, self.ptr, MQR_DEVICE, out.nbytes, self.device)
        return out

    def free(self):
        if self.ptr is not None and self.ptr.value:
            call("mqr_device_free", self.device, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
