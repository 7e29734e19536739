"""ctypes mirror of include/raytracer_hip.h and the loader for libraytracer_hip.so.

The shared library is the product: HIP kernels for gfx950 behind a plain C ABI.  There is
no CPU fallback -- if the library is missing or no device is present, the calls below
raise.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# RAYTRACER_HIP_LIB selects another build of the library (A/B variants under lib/ab/)
LIB_PATH = os.environ.get("RAYTRACER_HIP_LIB") or os.path.join(PKG_ROOT, "lib", "libraytracer_hip.so")

RT_ABI_VERSION = 10  # include/raytracer_hip.h
RT_COMM_ID_BYTES = 128
RT_CREATE_RCCL_GATHER = 1
RT_CREATE_SHARED_DEVICE = 2
RT_MAX_WORKERS = 64
RT_BANDS_INT32, RT_BANDS_RGB24, RT_BANDS_FRAME = 0, 1, 2
RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_NO_DEVICE = -2
RT_ERR_HIP = -3
RT_ERR_NO_SCENE = -4
RT_ERR_UNSUPPORTED = -5
RT_ERR_RCCL = -6
RT_ERR_OOM = -7
RT_MAX_RECURSION_LIMIT = 63
RT_MAX_LIGHTS = 65536

RT_KEY_W, RT_KEY_A, RT_KEY_S, RT_KEY_D, RT_KEY_SPACE, RT_KEY_SHIFT = 1, 2, 3, 4, 5, 6


class rt_vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]

    def tuple(self):
        return (self.x, self.y, self.z)


class rt_material(C.Structure):
    _fields_ = [("kd", rt_vec3), ("ka", rt_vec3), ("ks", rt_vec3), ("n", C.c_float), ("km", rt_vec3)]


class rt_sphere(C.Structure):
    _fields_ = [("center", rt_vec3), ("radius", C.c_float), ("material", rt_material)]


class rt_plane(C.Structure):
    _fields_ = [("center", rt_vec3), ("normal", rt_vec3), ("material", rt_material)]


class rt_light(C.Structure):
    _fields_ = [("position", rt_vec3), ("intensity", C.c_float)]


class rt_camera(C.Structure):
    _fields_ = [("position", rt_vec3), ("yaw", C.c_float), ("pitch", C.c_float)]


class rt_view(C.Structure):
    _fields_ = [
        ("position", rt_vec3), ("right", rt_vec3), ("up", rt_vec3), ("forward", rt_vec3),
        ("plane_width", C.c_float), ("plane_height", C.c_float), ("near_clip", C.c_float),
    ]


class rt_segment(C.Structure):
    _fields_ = [("origin", rt_vec3), ("end", rt_vec3), ("kind", C.c_int32), ("pixel", C.c_int32)]


class rt_stats(C.Structure):
    _fields_ = [
        ("frames", C.c_uint64), ("pixels", C.c_uint64), ("primary_rays", C.c_uint64),
        ("reflect_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("sphere_tests", C.c_uint64),
        ("plane_tests", C.c_uint64), ("launches", C.c_uint64), ("kernel_ms", C.c_double),
        ("last_kernel_ms", C.c_double), ("copy_ms", C.c_double), ("gather_ms", C.c_double),
        ("timed_launches", C.c_uint64), ("timed_copies", C.c_uint64), ("timed_gathers", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class rt_work(C.Structure):
    _fields_ = [
        ("primary_rays", C.c_uint64), ("reflect_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
        ("sphere_tests", C.c_uint64), ("plane_tests", C.c_uint64), ("shadow_rays_run", C.c_uint64),
        ("sphere_tests_run", C.c_uint64), ("plane_tests_run", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class rt_wire_layout(C.Structure):
    _fields_ = [
        ("fixed_bytes", C.c_uint64), ("max_bytes", C.c_uint64), ("tiles_x", C.c_int32), ("tiles_y", C.c_int32),
        ("tiles_per_frame", C.c_int32), ("n_frames", C.c_int32), ("n_tiles", C.c_int32), ("n_chunks", C.c_int32),
    ]


# (name, restype, argtypes) of every exported entry point declared in the header.
EXPORTS = [
    ("rt_abi_version", C.c_int, []),
    ("rt_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("rt_last_error", C.c_char_p, [C.c_void_p]),
    ("rt_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_create_ex", C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_destroy", None, [C.c_void_p]),
    ("rt_set_scene", C.c_int, [C.c_void_p, C.POINTER(rt_sphere), C.c_int, C.POINTER(rt_plane), C.c_int,
                               C.POINTER(rt_light), C.c_int, rt_vec3, C.c_int]),
    ("rt_set_camera", C.c_int, [C.c_void_p, C.POINTER(rt_camera)]),
    ("rt_set_view_height", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_set_counting", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_get_camera", C.c_int, [C.c_void_p, C.POINTER(rt_camera)]),
    ("rt_camera_view", C.c_int, [C.POINTER(rt_camera), C.c_int, C.c_int, C.POINTER(rt_view)]),
    ("rt_camera_on_key", C.c_int, [C.POINTER(rt_camera), C.c_int]),
    ("rt_camera_on_mouse_move", C.c_int, [C.POINTER(rt_camera), C.c_float, C.c_float]),
    ("rt_render", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_register_host", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rt_unregister_host", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rt_render_device", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    ("rt_render_bands", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                  C.c_void_p, C.POINTER(C.c_int)]),
    ("rt_scatter_bands", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                   C.c_void_p, C.c_void_p]),
    ("rt_render_bands_ex", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                     C.c_void_p, C.POINTER(C.c_int)]),
    ("rt_render_bands_batch", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                        C.c_size_t, C.c_int, C.c_void_p, C.POINTER(C.c_int)]),
    ("rt_scatter_gathered", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                      C.c_int, C.c_void_p, C.c_void_p]),
    ("rt_wire_layout_of", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(rt_wire_layout)]),
    ("rt_encode_bands", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rt_decode_gathered", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                     C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]),
    ("rt_render_bands_tiles", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_void_p, C.c_void_p]),
    ("rt_finish_wire", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                 C.c_void_p, C.c_void_p]),
    ("rt_comm_probe", C.c_int, []),
    ("rt_comm_unique_id", C.c_int, [C.c_void_p]),
    ("rt_comm_init", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_comm_allreduce_max_i64", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    ("rt_comm_gather", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
    ("rt_render_async", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_wait", C.c_int, [C.c_void_p]),
    ("rt_write_ppm", C.c_int, [C.c_char_p, C.c_void_p, C.c_int, C.c_int]),
    ("rt_debug_segments", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    ("rt_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_dispatch_order", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("rt_get_stats", C.c_int, [C.c_void_p, C.POINTER(rt_stats)]),
    ("rt_reset_stats", C.c_int, [C.c_void_p]),
    ("rt_count_work", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(rt_work)]),
]

_lib = None


class RayTracerError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libraytracer_hip error {code}: {msg}")
        self.code = code


def load_library(path: str | None = None, local: bool = False):
    """Load libraytracer_hip.so (in-tree build).  Raises if it was not built.
    local=True loads with RTLD_LOCAL (several builds side by side, tools/ab.py)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"libraytracer_hip.so not found at {p}: run __graft_entry__.build() "
            "(there is no CPU fallback)")
    lib = C.CDLL(p, mode=C.RTLD_LOCAL if local else C.RTLD_GLOBAL)
    for name, res, args in EXPORTS:
        fn = getattr(lib, name, None)
        if fn is None:
            if local:  # an older build under A/B comparison
                continue
            raise RuntimeError(f"{p} does not export {name}: stale build, run __graft_entry__.build()")
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(lib, code: int, ctx=None):
    if code != RT_OK:
        msg = lib.rt_last_error(ctx)
        raise RayTracerError(code, msg.decode() if msg else "")
    return code
