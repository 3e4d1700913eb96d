"""ctypes wrapper of the CPU oracle (oracle/libpt_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  The oracle is a
C restatement of the reference GLSL path (see pt_oracle.h for file:line
citations and the parity status: "parity unpinned" at the GLSL/driver
boundary, pinned for slot topology and integer RNG).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, Structure, c_float, c_int, c_int32, c_uint8, c_uint32, c_uint64, c_void_p
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpt_oracle.so")

UNION, SPHERE, CUBE, TORUS, OCTAHEDRON, PLANE = range(6)


class Node(Structure):
    _fields_ = [("kind", c_int32), ("parent", c_int32), ("union_type", c_int32), ("aabb", c_int32),
                ("scale", c_float), ("pos", c_float * 3), ("rot", c_float * 3), ("aabb_ex", c_float),
                ("size", c_float * 3), ("mat", c_float * 18)]


class Constants(Structure):
    _fields_ = [("time", c_float), ("frame", c_int32), ("aspect", c_float), ("last_clear", c_int32)]


class Settings(Structure):
    _fields_ = [("debug", c_int32), ("bounces", c_int32), ("scale", c_float), ("fov", c_float), ("aabb", c_int32)]


COUNTER_NAMES = ("samples", "segments", "march_steps", "normal_maps", "shaded", "aabb_tests", "xform_union",
                 "xform_shape", "sdf_union", "sdf_sphere", "sdf_cube", "sdf_torus", "sdf_octahedron", "sdf_plane",
                 "comb_union", "comb_sub", "comb_assign", "rr_break")


class Counters(Structure):
    _fields_ = [(n, c_uint64) for n in COUNTER_NAMES]


_lib = None


def build_native(out_dir: str) -> str:
    """The oracle compiled for the host it runs on (-march=native; the
    shipped build targets x86-64-v3 so it loads on any box).  Same semantics:
    -ffp-contract=off keeps every rounding step, and the explicit fmaf calls
    are fused either way.  Used by bench.py's cpu_baseline leg."""
    out = os.path.join(out_dir, "libpt_oracle_native.so")
    subprocess.run(["gcc", "-O3", "-march=native", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                    "-pthread", "-o", out, os.path.join(HERE, "pt_oracle.c"), "-lm"], check=True)
    return out


def use_library(path: str) -> None:
    """Load the oracle from ``path`` (before its first use in the process)."""
    global LIB_PATH, _lib
    if _lib is not None:
        raise RuntimeError("oracle library already loaded")
    LIB_PATH = path


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.pto_scene_build.argtypes = [POINTER(Node), c_int, POINTER(vp)]
        L.pto_scene_build.restype = c_int
        L.pto_scene_build_keyed.argtypes = [POINTER(Node), c_int, POINTER(c_uint64), POINTER(vp)]
        L.pto_scene_build_keyed.restype = c_int
        L.pto_scene_free.argtypes = [vp]
        L.pto_scene_n_data.argtypes = [vp]
        L.pto_scene_n_check.argtypes = [vp]
        L.pto_scene_get_data.argtypes = [vp, POINTER(c_float)]
        L.pto_scene_set_data.argtypes = [vp, POINTER(c_float), c_int]
        L.pto_scene_node_slots.argtypes = [vp, c_int, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]
        L.pto_wang_hash.argtypes = [POINTER(c_uint32)]
        L.pto_wang_hash.restype = c_uint32
        L.pto_random01.argtypes = [POINTER(c_uint32)]
        L.pto_random01.restype = c_float
        L.pto_gen_rng.argtypes = [c_int32] * 5
        L.pto_gen_rng.restype = c_uint32
        L.pto_sin.argtypes = [c_float]
        L.pto_sin.restype = c_float
        L.pto_cos.argtypes = [c_float]
        L.pto_cos.restype = c_float
        L.pto_map.argtypes = [vp, POINTER(c_float), POINTER(c_uint8), POINTER(c_int32)]
        L.pto_map.restype = c_float
        L.pto_bounds.argtypes = [vp, POINTER(c_float), POINTER(c_float), POINTER(c_uint8), POINTER(c_float)]
        L.pto_render.argtypes = [vp, POINTER(c_float), c_int, c_int, POINTER(Constants), POINTER(Settings), c_int,
                                 c_int, c_int, c_int, c_int, POINTER(Counters)]
        L.pto_display.argtypes = [POINTER(c_float), c_int, c_int, c_int, vp]
        L.pto_display.restype = None
        L.pto_pow_pos.argtypes = [c_float, c_float]
        L.pto_pow_pos.restype = c_float
        _lib = L
    return _lib


def rows_to_nodes(rows: Sequence[dict]) -> ctypes.Array:
    arr = (Node * max(1, len(rows)))()
    for i, r in enumerate(rows):
        n = arr[i]
        n.kind, n.parent, n.union_type, n.aabb = r["kind"], r["parent"], r["union_type"], r["aabb"]
        n.scale, n.aabb_ex = r["scale"], r["aabb_exaggeration"]
        for k in range(3):
            n.pos[k], n.rot[k], n.size[k] = r["position"][k], r["rotation"][k], r["size"][k]
        for k in range(18):
            n.mat[k] = r["material"][k]
    return arr


class OracleScene:
    """The editor tree compiled by the oracle's own restatement of
    SDFEditor::compile (slot allocation independent of the product)."""

    def __init__(self, rows: Sequence[dict]):
        self._L = lib()
        self._nodes = rows_to_nodes(rows)
        self.n_nodes = len(rows)
        h = ctypes.c_void_p()
        # the Floats' u128 hashes (rows' "keys", 29 per node): shared hashes
        # share a slot, as DataArray::get_index does
        self._keys = None
        if any(r.get("keys") for r in rows):
            self._keys = (c_uint64 * (2 * 29 * max(1, len(rows))))()
            for i, r in enumerate(rows):
                for k, key in enumerate(r.get("keys") or []):
                    self._keys[2 * (i * 29 + k)] = key & 0xFFFFFFFFFFFFFFFF
                    self._keys[2 * (i * 29 + k) + 1] = (key >> 64) & 0xFFFFFFFFFFFFFFFF
        rc = self._L.pto_scene_build_keyed(self._nodes, len(rows), self._keys, ctypes.byref(h))
        if rc != 0:
            raise ValueError(f"pto_scene_build rc={rc}")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.pto_scene_free(self._h)
            self._h = None

    @property
    def n_check(self) -> int:
        return self._L.pto_scene_n_check(self._h)

    def data(self) -> np.ndarray:
        n = self._L.pto_scene_n_data(self._h)
        out = np.zeros(n, np.float32)
        self._L.pto_scene_get_data(self._h, out.ctypes.data_as(POINTER(c_float)))
        return out

    def set_data(self, data: np.ndarray) -> None:
        d = np.ascontiguousarray(data, np.float32)
        if self._L.pto_scene_set_data(self._h, d.ctypes.data_as(POINTER(c_float)), d.size) != 0:
            raise ValueError("data size mismatch")

    def node_slots(self, i: int):
        slots = (c_int32 * 29)()
        chk, bidx = c_int32(), c_int32()
        self._L.pto_scene_node_slots(self._h, i, slots, ctypes.byref(chk), ctypes.byref(bidx))
        return list(slots), chk.value, bidx.value

    def map(self, p, check: Optional[Sequence[int]] = None):
        pc = (c_float * 3)(*p)
        ck = (c_uint8 * max(1, self.n_check))(*(check if check is not None else [1] * self.n_check))
        m = c_int32()
        d = self._L.pto_map(self._h, pc, ck, ctypes.byref(m))
        return float(d), m.value

    def bounds(self, ro, rd):
        ck = (c_uint8 * max(1, self.n_check))()
        dbg = (c_float * 3)()
        self._L.pto_bounds(self._h, (c_float * 3)(*ro), (c_float * 3)(*rd), ck, dbg)
        return list(ck), list(dbg)

    def render(self, width: int, height: int, constants: Constants, settings: Settings, spp: int,
               image: Optional[np.ndarray] = None, rank: int = 0, nranks: int = 1, row_stride: int = 1,
               threads: int = 0, counters: bool = False):
        if image is None:
            image = np.zeros((height, width, 4), np.float32)
        assert image.dtype == np.float32 and image.flags.c_contiguous and image.shape == (height, width, 4)
        if threads <= 0:
            threads = os.cpu_count() or 1
        ct = Counters() if counters else None
        self._L.pto_render(self._h, image.ctypes.data_as(POINTER(c_float)), width, height, ctypes.byref(constants),
                           ctypes.byref(settings), spp, rank, nranks, row_stride, threads,
                           ctypes.byref(ct) if ct is not None else None)
        if counters:
            return image, {n: int(getattr(ct, n)) for n in COUNTER_NAMES}
        return image


def wang_hash(seed: int) -> int:
    s = c_uint32(seed)
    return int(lib().pto_wang_hash(ctypes.byref(s)))


def random01_seq(seed: int, n: int) -> List[float]:
    s = c_uint32(seed)
    return [float(lib().pto_random01(ctypes.byref(s))) for _ in range(n)]


def gen_rng(x, y, frame, w, h) -> int:
    return int(lib().pto_gen_rng(x, y, frame, w, h))


def sin(x: float) -> float:
    return float(lib().pto_sin(x))


def cos(x: float) -> float:
    return float(lib().pto_cos(x))


def display(image: np.ndarray, srgb8: bool = False) -> np.ndarray:
    """The display pass restated (pto_display): fs_main RGBA32F per texel, or
    the sRGB swapchain's 8-bit RGBA in screen order."""
    img = np.ascontiguousarray(image, np.float32)
    h, w = img.shape[:2]
    out = np.empty((h, w, 4), np.uint8 if srgb8 else np.float32)
    lib().pto_display(img.ctypes.data_as(POINTER(c_float)), w, h, 1 if srgb8 else 0, out.ctypes.data_as(c_void_p))
    return out


def pow_pos(x: float, y: float) -> float:
    return float(lib().pto_pow_pos(x, y))
