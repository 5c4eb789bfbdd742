"""ctypes mirror of include/rtm.h and the loader for the HIP library (librtm.so).

The structs are byte-for-byte the C ABI; the loader fails loudly when the
library is missing (there is no CPU fallback on the product path).
"""
from __future__ import annotations

import ctypes as C
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RTM_LIB: another build of the same library (A/B timing runs only, tools/ab_bench.py)
LIB_PATH = os.environ.get("RTM_LIB") or os.path.join(_PKG_DIR, "librtm.so")

RTM_ABI_VERSION = 11
# library versions whose public structs share this layout (an RTM_LIB A/B build may be one)
RTM_ABI_LAYOUT_COMPATIBLE = frozenset({9, 10, 11})
RTM_MAX_SPHERES = 16
RTM_MAX_PATCHES = 4
RTM_MAX_CIRCLE_PLANES = 16
RTM_MAX_CAPPED_CYLINDERS = 16
RTM_MAX_SDFS = 8
RTM_MAX_DIM = 32768

RTM_OK = 0
RTM_ERR_INVALID = -1
RTM_ERR_UNSUPPORTED = -2
RTM_ERR_HIP = -3
RTM_ERR_NO_DEVICE = -4
RTM_ERR_OOM = -5
RTM_ERR_COMM = -6

RTM_CAMERA_ORTHOGONAL = 0
RTM_CAMERA_PERSPECTIVE = 1
RTM_FACE_FRONT = 0
RTM_FACE_BACK = 1

RTM_FLAG_NO_MARCH = 0x1
RTM_FLAG_NO_SHADOW_RASTER = 0x2
RTM_FLAG_FUSED_SHADOW = 0x4

# frame output formats (ABI v6): RGBA f32 / writeColorImage bytes + alpha 255 / packed RGB8
RTM_FORMAT_RGBA32F = 0
RTM_FORMAT_RGBA8 = 1
RTM_FORMAT_RGB8 = 2
FORMAT_BYTES = {RTM_FORMAT_RGBA32F: 16, RTM_FORMAT_RGBA8: 4, RTM_FORMAT_RGB8: 3}


class rtm_sphere(C.Structure):
    _fields_ = [("id", C.c_int64), ("pos", C.c_double * 3), ("r", C.c_double),
                ("color", C.c_double * 3)]


class rtm_patch(C.Structure):
    _fields_ = [("a0", C.c_double), ("b0", C.c_double), ("a1", C.c_double), ("b1", C.c_double)]


class rtm_camera(C.Structure):
    _fields_ = [("type", C.c_int32), ("reserved", C.c_int32), ("pos", C.c_double * 3),
                ("dir", C.c_double * 3), ("up", C.c_double * 3), ("side", C.c_double * 3)]


class rtm_circle_plane(C.Structure):
    _fields_ = [("id", C.c_int64), ("pos", C.c_double * 3), ("n", C.c_double * 3), ("radius", C.c_double),
                ("color", C.c_double * 3)]


class rtm_capped_cylinder(C.Structure):
    _fields_ = [("id", C.c_int64), ("pa", C.c_double * 3), ("pb", C.c_double * 3), ("ra", C.c_double),
                ("rb", C.c_double), ("color", C.c_double * 3)]


class rtm_sdf(C.Structure):
    _fields_ = [("id", C.c_int64), ("box_center", C.c_double * 3), ("tri_anchor", C.c_double * 3),
                ("aabb_center", C.c_double * 3), ("aabb_extent", C.c_double * 3), ("color", C.c_double * 3),
                ("max_steps", C.c_int32), ("reserved", C.c_int32)]


class rtm_scene(C.Structure):
    _fields_ = [("spheres", C.POINTER(rtm_sphere)), ("patches", C.POINTER(rtm_patch)),
                ("n_spheres", C.c_int32), ("n_patches", C.c_int32),
                ("circle_planes", C.POINTER(rtm_circle_plane)),
                ("capped_cylinders", C.POINTER(rtm_capped_cylinder)),
                ("n_circle_planes", C.c_int32), ("n_capped_cylinders", C.c_int32),
                ("sdfs", C.POINTER(rtm_sdf)), ("n_sdfs", C.c_int32), ("reserved", C.c_int32)]


class rtm_stats(C.Structure):
    _fields_ = [("eye_hits", C.c_int64 * RTM_MAX_SPHERES), ("eye_hit_pixels", C.c_int64),
                ("lit_pixels", C.c_int64), ("eye_sphere_tests", C.c_int64),
                ("shadow_sphere_tests", C.c_int64), ("march_iterations", C.c_int64),
                ("march_hits", C.c_int64), ("march_in_range", C.c_int64),
                ("eye_circle_plane_pixels", C.c_int64), ("eye_capped_cylinder_pixels", C.c_int64),
                ("eye_sdf_pixels", C.c_int64), ("sdf_distance_evals", C.c_int64),
                ("eye_plane_tests", C.c_int64), ("eye_cylinder_tests", C.c_int64)]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "eye_hits"}
        d["eye_hits"] = list(self.eye_hits)
        return d


assert C.sizeof(rtm_sphere) == 64
assert C.sizeof(rtm_patch) == 32
assert C.sizeof(rtm_camera) == 104
assert C.sizeof(rtm_circle_plane) == 88
assert C.sizeof(rtm_capped_cylinder) == 96
assert C.sizeof(rtm_sdf) == 136
assert C.sizeof(rtm_scene) == 64
assert C.sizeof(rtm_stats) == 8 * (RTM_MAX_SPHERES + 13)

# (name, restype, argtypes) for every symbol include/rtm.h declares.
_P = C.c_void_p
_I32 = C.c_int32
ABI_SYMBOLS = [
    ("rtm_abi_version", C.c_int32, []),
    ("rtm_last_error", C.c_char_p, []),
    ("rtm_device_count", C.c_int32, []),
    ("rtm_ctx_create", C.c_int, [_I32, C.POINTER(_P)]),
    ("rtm_ctx_destroy", None, [_P]),
    ("rtm_ctx_stream", _P, [_P]),
    ("rtm_ctx_synchronize", C.c_int, [_P]),
    ("rtm_ctx_alloc", C.c_int, [_P, C.c_int64, C.POINTER(_P)]),
    ("rtm_ctx_free", C.c_int, [_P, _P]),
    ("rtm_ctx_copy_to_host", C.c_int, [_P, _P, _P, C.c_int64]),
    ("rtm_ctx_oob_reads", C.c_int, [_P, C.POINTER(C.c_int64)]),
    ("rtm_ctx_last_kernel_ms", C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("rtm_ctx_set_timing_capacity", C.c_int, [_P, _I32]),
    ("rtm_ctx_set_timing_stride", C.c_int, [_P, _I32]),
    ("rtm_ctx_set_lanes", C.c_int, [_P, _I32]),
    ("rtm_ctx_last_lanes", C.c_int, [_P, C.POINTER(_I32)]),
    ("rtm_ctx_set_batch", C.c_int, [_P, _I32]),
    ("rtm_ctx_last_batch", C.c_int, [_P, C.POINTER(_I32)]),
    ("rtm_ctx_kernel_ms_history", C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_float), _I32,
                                            C.POINTER(_I32)]),
    ("rtm_render", C.c_int, [C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                             _I32, _I32, _I32, _I32, C.POINTER(C.c_float)]),
    ("rtm_render_async", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                   C.POINTER(rtm_camera), _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_render_frames_async", C.c_int, [_P, _I32, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                          C.POINTER(rtm_camera), _I32, _I32, _I32, _I32, C.POINTER(_P)]),
    ("rtm_ctx_shadow_map", _P, [_P]),
    ("rtm_ctx_shadow_map_texel_bytes", C.c_int32, [_P]),
    ("rtm_ctx_shadow_map_stored_bytes", C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(_I32)]),
    ("rtm_ctx_frames_plan", C.c_int, [_P, _I32, _I32, _I32, C.POINTER(_I32), C.POINTER(_I32)]),
    ("rtm_ctx_last_eye_blocks", C.c_int, [_P, C.POINTER(_I32)]),
    ("rtm_render_multi", C.c_int, [C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                                   _I32, _I32, _I32, _I32, C.POINTER(C.c_float), _I32]),
    ("rtm_render_stats", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                   C.POINTER(rtm_camera), _I32, _I32, _I32, _I32,
                                   C.POINTER(rtm_stats)]),
    ("rtm_encode_rgb8_async", C.c_int, [_P, _P, C.c_int64, _P]),
    ("rtm_ppm_max_bytes", C.c_int64, [_I32, _I32]),
    ("rtm_write_ppm", C.c_int, [_P, _P, _I32, _I32, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]),
    ("rtm_encode_thresholds", C.c_int, [C.POINTER(C.c_float)]),
    ("rtm_render_ex", C.c_int, [C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                                _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_render_multi_ex", C.c_int, [C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                                      _I32, _I32, _I32, _I32, _I32, _P, _I32]),
    ("rtm_format_bytes", C.c_int32, [_I32]),
    ("rtm_host_register", C.c_int, [_P, C.c_int64]),
    ("rtm_host_unregister", C.c_int, [_P]),
    ("rtm_render_rows_async", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                        C.POINTER(rtm_camera), _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_group_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("rtm_group_create", C.c_int, [_I32, C.POINTER(_I32), C.POINTER(_P)]),
    ("rtm_group_create_rank", C.c_int, [_I32, _I32, _I32, C.POINTER(C.c_uint8), C.POINTER(_P)]),
    ("rtm_group_destroy", None, [_P]),
    ("rtm_group_info", C.c_int, [_P, C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I32)]),
    ("rtm_group_ctx", _P, [_P, _I32]),
    ("rtm_group_render_async", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                         C.POINTER(rtm_camera), _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_group_render_frames_async", C.c_int, [_P, _I32, C.POINTER(rtm_scene), C.POINTER(rtm_camera),
                                                C.POINTER(rtm_camera), _I32, _I32, _I32, _I32, _I32, _I32,
                                                C.POINTER(_P)]),
    ("rtm_group_render", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                                   _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_group_stream", _P, [_P]),
    ("rtm_group_synchronize", C.c_int, [_P, _I32]),
    ("rtm_group_set_root_staging", C.c_int, [_P, _I32]),
    ("rtm_group_create_loopback", C.c_int, [_I32, C.POINTER(_I32), C.POINTER(_P)]),
    ("rtm_group_set_host_direct", C.c_int, [_P, _I32]),
    ("rtm_group_set_partition", C.c_int, [_P, _I32]),
    ("rtm_group_partition", C.c_int32, [_P]),
    ("rtm_group_frames_plan", C.c_int, [_P, _I32, _I32, _I32, _I32, C.POINTER(_I32), C.POINTER(_I32)]),
    ("rtm_render_stripes_async", C.c_int, [_P, C.POINTER(rtm_scene), C.POINTER(rtm_camera), C.POINTER(rtm_camera),
                                           _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    ("rtm_stripe_rows", C.c_int32, [_I32, _I32, _I32, _I32]),
    ("rtm_viewport_create", C.c_int, [_P, _I32, _I32, _I32, C.POINTER(rtm_camera), C.POINTER(_P)]),
    ("rtm_viewport_destroy", None, [_P]),
    ("rtm_viewport_rasterize", C.c_int, [_P, C.POINTER(rtm_scene)]),
    ("rtm_viewport_process_raytracing_rays", C.c_int, [_P, C.POINTER(rtm_scene)]),
    ("rtm_viewport_process_raymarching_rays", C.c_int, [_P, C.POINTER(rtm_patch), _I32, _I32]),
    ("rtm_render_color_image", C.c_int, [C.POINTER(rtm_scene), _P, _P, C.POINTER(C.c_float)]),
    ("rtm_viewport_read_zbuffer", C.c_int, [_P, C.POINTER(C.c_double)]),
]


class RtmError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str = ""):
        super().__init__(f"{where} failed with {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load librtm.so (the HIP build).  Raises if it is missing: the product
    path has no CPU fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    # torch wheels bundle their own libamdhip64.so.7.  Loading torch first makes
    # librtm bind to that same runtime (same soname), so a process that also uses
    # torch has ONE HIP runtime; two runtimes in one process cannot both see the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{p} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP library is the only render path)")
    lib = C.CDLL(p)
    # An A/B build (RTM_LIB) may predate the newest calls: those stay unbound there (and
    # are named on stderr).  Its public struct layouts must still be this package's: only
    # the versions listed as layout-compatible are accepted.
    ab = bool(os.environ.get("RTM_LIB")) and path is None
    ver = lib.rtm_abi_version()
    if ver != RTM_ABI_VERSION and not (ab and ver in RTM_ABI_LAYOUT_COMPATIBLE):
        raise RuntimeError(f"librtm ABI version {ver} at {p}, this package needs {RTM_ABI_VERSION}"
                           + (f" (an RTM_LIB build may be one of {sorted(RTM_ABI_LAYOUT_COMPATIBLE)})" if ab else ""))
    unbound = []
    for name, res, args in ABI_SYMBOLS:
        if ab and not hasattr(lib, name):
            unbound.append(name)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if unbound:
        import sys
        sys.stderr.write(f"librtm ({p}, RTM_LIB A/B build, ABI {ver}): unbound {', '.join(unbound)}\n")
    if path is None:
        _lib = lib
    return lib


def check(lib, code: int, where: str) -> None:
    if code != RTM_OK:
        msg = lib.rtm_last_error()
        raise RtmError(code, where, msg.decode() if msg else "")
