"""ctypes binding of the C ABI in ``include/pt_abi.h`` (``lib/libpt.so``).

This is the Python-side equivalent of the ``extern "C"`` block a Rust host
would declare.  There is no fallback: if the HIP library is
missing the import of anything that renders raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpt.so")

PT_OK = 0
PT_ERR_INVALID = -1
PT_ERR_HIP = -2
PT_ERR_UNSUPPORTED = -3
PT_ERR_STATE = -4
PT_ERR_RCCL = -5
PT_ERR_SIZE = -6

PT_NODE_UNION, PT_NODE_SPHERE, PT_NODE_CUBE, PT_NODE_TORUS, PT_NODE_OCTAHEDRON, PT_NODE_PLANE = range(6)
PT_UNION_TYPE_UNION, PT_UNION_TYPE_SUBTRACTION = 0, 1
PT_OP_UNION_BEGIN, PT_OP_SHAPE, PT_OP_UNION_END = 0, 1, 2
PT_COMBINE_ASSIGN, PT_COMBINE_UNION, PT_COMBINE_SUBTRACTION = 0, 1, 2
PT_SO_SCALAR, PT_SO_VEC3, PT_SO_ONE, PT_SO_TORUS = 0, 1, 2, 3
PT_COMM_ID_BYTES = 128
PT_DISPLAY_RGBA32F, PT_DISPLAY_SRGB8 = 0, 1
PT_STAT_COUNT = 32
STAT_NAMES = (
    "samples", "segments", "march_steps", "normal_maps", "shaded", "aabb_tests", "xform_union", "xform_shape",
    "sdf_sphere", "sdf_cube", "sdf_torus", "sdf_octahedron", "comb_union", "comb_sub", "comb_assign", "rr_break",
    "wave_maps", "wave_shapes", "wave_iters", "lane_idle", "idle_shade", "idle_free",
    # wavefront kernel, wave-clock cycles (s_memtime) per phase, summed over waves
    "cyc_refill", "cyc_bounds", "cyc_map", "cyc_shade", "cyc_total",
    "culled", "wave_evals", "bounds_waves", "bounds_exact",
    "shaded_first",  # binned pipeline: hits shaded in shade pass 0
)

PT_ST_COUNT = len(STAT_NAMES)  # device counters (pt_device.h PT_ST_COUNT)

SYMBOLS = (
    "pt_compile_scene", "pt_create", "pt_resize_clear", "pt_set_program", "pt_set_data", "pt_set_tiles",
    "pt_dispatch", "pt_read_accum", "pt_accum_device_ptr", "pt_get_size", "pt_comm_get_unique_id",
    "pt_comm_init", "pt_reduce_accum", "pt_read_reduced", "pt_sync", "pt_last_dispatch_ms",
    "pt_dispatch_stats", "pt_set_option", "pt_get_option", "pt_jit_log", "pt_jit_compile", "pt_last_error",
    "pt_destroy", "pt_abi_version", "pt_device_math", "pt_check_sqrt_exhaustive", "pt_check_div_exhaustive",
    "pt_check_div_random", "pt_check_box_random", "pt_check_div_k", "pt_display", "pt_write_accum",
    "pt_compile_scene_keyed", "pt_save_rgba8", "pt_comm_size", "pt_traffic_probe", "pt_scene_kernel_source",
)
PT_MATH = {"max": 0, "min": 1, "sqrt": 2, "sqrtf": 3, "sin": 4, "cos": 5, "div": 6, "fma": 7}


class Constants(Structure):
    """== ``Constants`` UBO (path_tracer.rs:149-155)."""

    _fields_ = [("time", c_float), ("frame", c_int32), ("aspect", c_float), ("last_clear", c_int32)]


class Settings(Structure):
    """== ``Settings`` UBO (path_tracer.rs:157-163); defaults match the reference sliders."""

    _fields_ = [("debug", c_int32), ("bounces", c_int32), ("scale", c_float), ("fov", c_float), ("aabb", c_int32)]


class SceneNode(Structure):
    _fields_ = [
        ("kind", c_int32), ("parent", c_int32), ("union_type", c_int32), ("aabb", c_int32),
        ("scale", c_float), ("position", c_float * 3), ("rotation", c_float * 3), ("aabb_exaggeration", c_float),
        ("size", c_float * 3), ("material", c_float * 18),
    ]


PT_NODE_FLOATS = 29


class FloatKey(Structure):
    """pt_float_key: a Float's u128 serde hash (lo, hi); {0, 0} = anonymous."""

    _fields_ = [("lo", c_uint64), ("hi", c_uint64)]


class Op(Structure):
    _fields_ = [
        ("opcode", c_uint32), ("shape", c_uint32), ("combine", c_uint32), ("check", c_int32),
        ("scale", c_uint32), ("position", c_uint32 * 3), ("rotation", c_uint32 * 3), ("aabb_exaggeration", c_uint32),
        ("size", c_uint32 * 3), ("material", c_uint32 * 18),
    ]


class Aabb(Structure):
    _fields_ = [
        ("back", c_int32), ("so_kind", c_uint32), ("union_position", c_uint32 * 3), ("union_scale", c_uint32),
        ("shape_position", c_uint32 * 3), ("shape_scale", c_uint32), ("size", c_uint32 * 3),
        ("aabb_exaggeration", c_uint32),
    ]


assert ctypes.sizeof(Constants) == 16 and ctypes.sizeof(Settings) == 20
assert ctypes.sizeof(SceneNode) == 132 and ctypes.sizeof(Op) == 132 and ctypes.sizeof(Aabb) == 56


class NativeError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """Load ``libpt.so`` (the HIP build).  Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("PT_LIB") or LIB_PATH  # PT_LIB: an in-tree A/B variant (build.build_variant)
    if not os.path.exists(path):
        raise ImportError(f"HIP library {path} missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = ctypes.CDLL(path)
    ctx = c_void_p
    u32p = POINTER(c_uint32)
    sig = {
        "pt_compile_scene": (c_int, [POINTER(SceneNode), c_uint32, POINTER(Op), c_uint32, u32p, POINTER(Aabb), c_uint32,
                                     u32p, POINTER(c_float), c_uint32, u32p, u32p]),
        "pt_compile_scene_keyed": (c_int, [POINTER(SceneNode), c_uint32, POINTER(FloatKey), POINTER(Op), c_uint32, u32p,
                                           POINTER(Aabb), c_uint32, u32p, POINTER(c_float), c_uint32, u32p, u32p]),
        "pt_save_rgba8": (c_int, [POINTER(c_float), c_uint32, c_uint32, POINTER(c_uint8), c_size_t]),
        "pt_create": (c_int, [c_int, c_uint32, c_uint32, POINTER(ctx)]),
        "pt_resize_clear": (c_int, [ctx, c_uint32, c_uint32]),
        "pt_set_program": (c_int, [ctx, POINTER(Op), c_uint32, POINTER(Aabb), c_uint32, c_uint32]),
        "pt_set_data": (c_int, [ctx, POINTER(c_float), c_uint32]),
        "pt_set_tiles": (c_int, [ctx, c_uint32, c_uint32]),
        "pt_dispatch": (c_int, [ctx, POINTER(Constants), POINTER(Settings), c_uint32]),
        "pt_read_accum": (c_int, [ctx, POINTER(c_float), c_size_t]),
        "pt_accum_device_ptr": (c_int, [ctx, POINTER(c_void_p), POINTER(c_size_t)]),
        "pt_get_size": (c_int, [ctx, u32p, u32p]),
        "pt_comm_get_unique_id": (c_int, [POINTER(c_uint8)]),
        "pt_comm_init": (c_int, [ctx, c_uint32, c_uint32, POINTER(c_uint8)]),
        "pt_comm_size": (c_int, [ctx, u32p]),
        "pt_reduce_accum": (c_int, [ctx, c_int]),
        "pt_read_reduced": (c_int, [ctx, POINTER(c_float), c_size_t]),
        "pt_sync": (c_int, [ctx]),
        "pt_last_dispatch_ms": (c_int, [ctx, POINTER(c_float)]),
        "pt_dispatch_stats": (c_int, [ctx, POINTER(Constants), POINTER(Settings), c_uint32, POINTER(c_uint64)]),
        "pt_set_option": (c_int, [ctx, c_char_p, c_int]),
        "pt_get_option": (c_int, [ctx, c_char_p, POINTER(ctypes.c_double)]),
        "pt_jit_log": (c_char_p, [ctx]),
        "pt_jit_compile": (c_int, [POINTER(Op), c_uint32, POINTER(Aabb), c_uint32, POINTER(c_float), c_uint32, c_char_p,
                                   c_size_t, POINTER(c_size_t)]),
        "pt_scene_kernel_source": (c_int, [POINTER(Op), c_uint32, POINTER(Aabb), c_uint32, POINTER(c_float), c_uint32,
                                           c_int, c_char_p, c_size_t, POINTER(c_size_t)]),
        "pt_last_error": (c_char_p, [ctx]),
        "pt_destroy": (None, [ctx]),
        "pt_abi_version": (c_int, []),
        "pt_device_math": (c_int, [c_int, c_int, POINTER(c_float), POINTER(c_float), POINTER(c_float), c_uint32]),
        "pt_check_sqrt_exhaustive": (c_int, [c_int, POINTER(c_uint64), POINTER(c_uint32)]),
        "pt_check_div_exhaustive": (c_int, [c_int, c_uint32, c_uint32, c_uint32, c_uint32, POINTER(c_uint64),
                                            POINTER(c_uint64)]),
        "pt_check_div_random": (c_int, [c_int, c_uint32, c_uint32, POINTER(c_uint64), POINTER(c_uint64)]),
        "pt_check_box_random": (c_int, [c_int, c_uint32, c_uint32, c_int, POINTER(c_uint64)]),
        "pt_check_div_k": (c_int, [c_int, c_float, c_uint32, c_uint32, POINTER(c_uint64), POINTER(c_uint64)]),
        "pt_traffic_probe": (c_int, [c_int, c_uint32, POINTER(c_float), POINTER(c_uint64)]),
        "pt_display": (c_int, [c_void_p, c_int, c_void_p, c_size_t]),
        "pt_write_accum": (c_int, [c_void_p, POINTER(c_float), c_size_t]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("PT_LIB") and not hasattr(L, name):
            continue  # an older A/B variant may predate a self-test entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(fn: str, rc: int, ctx=None) -> None:
    if rc != PT_OK:
        msg = ""
        if ctx is not None:
            raw = lib().pt_last_error(ctx)
            msg = raw.decode() if raw else ""
        raise NativeError(fn, rc, msg)
