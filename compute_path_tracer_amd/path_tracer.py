"""Host mirror of the reference's ``PathTracer`` (src/path_tracer/path_tracer.rs).

Same public surface -- ``new``/``remake_pipeline``/``update``/``compute_pass``,
the ``Constants``/``Settings`` blocks with the reference defaults, the
``changed`` flag -- but the wgpu pipeline, UBOs and storage texture are
replaced by one native context (``include/pt_abi.h``) driving the HIP kernel.
``render(spp)`` is the batched form: it is exactly ``spp`` repetitions of
``update()`` + ``compute_pass()`` with no reset in between, executed as one
launch that keeps the accumulation texel in registers.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N
from .sdf_editor import Program


def default_settings() -> N.Settings:
    """defaults_and_sliders_gui!(Settings, ...) (path_tracer.rs:157-163)."""
    return N.Settings(debug=1, bounces=8, scale=1.0, fov=1.0, aabb=0)


class PathTracer:
    def __init__(self, width: int, height: int, program: Optional[Program] = None, data: Optional[np.ndarray] = None,
                 device: int = 0, settings: Optional[N.Settings] = None, options: Optional[dict] = None):
        """PathTracer::new (path_tracer.rs:28-60) + the storage texture it binds
        (StorageTexturePackage::new, structs.rs:113-160).  ``width``/``height``
        are the window size; the image is window * settings.scale."""
        self._L = N.lib()
        self.window = (int(width), int(height))
        self.constants = N.Constants(time=0.0, frame=0, aspect=0.0, last_clear=0)
        self.settings = settings if settings is not None else default_settings()
        self.changed = False
        self.device = device
        self.size = self._scaled_size()
        ctx = ctypes.c_void_p()
        N.check("pt_create", self._L.pt_create(device, self.size[0], self.size[1], ctypes.byref(ctx)))
        self._ctx = ctx
        for k, v in (options or {}).items():
            self.set_option(k, v)
        if program is not None:
            self.remake_pipeline(program)
            self.set_data(program.data if data is None else data)

    # -- lifecycle -----------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._L.pt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, fn: str, rc: int) -> None:
        N.check(fn, rc, self._ctx)

    def _scaled_size(self):
        s = np.float32(self.settings.scale)
        return (int(np.float32(self.window[0]) * s), int(np.float32(self.window[1]) * s))

    # -- reference surface ---------------------------------------------------
    def remake_pipeline(self, program: Program) -> None:
        """path_tracer.rs:62-76: a topology change (queue_compile)."""
        self._chk("pt_set_program", self._L.pt_set_program(self._ctx, program.ops, program.n_ops, program.aabbs,
                                                            program.n_aabb, program.n_check))

    def set_data(self, data: np.ndarray) -> None:
        """DataArray::update (primitives.rs:131-151): value-only upload."""
        arr = np.ascontiguousarray(data, dtype=np.float32)
        self._chk("pt_set_data", self._L.pt_set_data(self._ctx, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                      arr.size))

    def update(self, resized: bool = False, reset: bool = False, time: float = 0.0,
               window: Optional[tuple] = None) -> None:
        """path_tracer.rs:97-118: reset on resize/settings change/Space, then
        advance frame and last_clear."""
        if window is not None:
            self.window = (int(window[0]), int(window[1]))
        if resized or self.changed or reset:
            self.size = self._scaled_size()
            self._chk("pt_resize_clear", self._L.pt_resize_clear(self._ctx, self.size[0], self.size[1]))
            self.constants.last_clear = 0
        self.constants.time = float(time)
        self.constants.aspect = float(np.float32(self.window[0]) / np.float32(self.window[1]))  # setup.rs:84-86
        self.constants.frame += 1
        self.constants.last_clear += 1
        self.changed = False

    def compute_pass(self) -> None:
        """path_tracer.rs:128-146: one frame (1 spp) with the current blocks."""
        self._chk("pt_dispatch", self._L.pt_dispatch(self._ctx, ctypes.byref(self.constants),
                                                      ctypes.byref(self.settings), 1))

    # -- batched / multi-GPU ----------------------------------------------
    def render(self, spp: int) -> None:
        """``spp`` x (update(); compute_pass()) without resets, one dispatch."""
        if spp <= 0:
            return
        if self.changed:
            self.update()
            self.constants.frame -= 1
            self.constants.last_clear -= 1
        c = N.Constants(time=self.constants.time, frame=self.constants.frame + 1,
                        aspect=float(np.float32(self.window[0]) / np.float32(self.window[1])),
                        last_clear=self.constants.last_clear + 1)
        self.constants.aspect = c.aspect
        self._chk("pt_dispatch", self._L.pt_dispatch(self._ctx, ctypes.byref(c), ctypes.byref(self.settings), spp))
        self.constants.frame += spp
        self.constants.last_clear += spp

    def dispatch(self, constants: N.Constants, spp: int) -> None:
        """Raw pt_dispatch with explicit constants (frame j = frame + j)."""
        self._chk("pt_dispatch", self._L.pt_dispatch(self._ctx, ctypes.byref(constants), ctypes.byref(self.settings),
                                                      spp))

    def stats(self, constants: N.Constants, spp: int) -> dict:
        buf = (ctypes.c_uint64 * N.PT_STAT_COUNT)()
        self._chk("pt_dispatch_stats", self._L.pt_dispatch_stats(self._ctx, ctypes.byref(constants),
                                                                  ctypes.byref(self.settings), spp, buf))
        return dict(zip(N.STAT_NAMES, (int(v) for v in buf)))

    def tap_stats(self) -> dict:
        """The share of the last stats() run done by the shade pass's normal
        taps (shade_taps on; zeros otherwise)."""
        return {name: int(self.get_option(f"tap_stat_{k}")) for k, name in enumerate(N.STAT_NAMES)
                if k < N.PT_ST_COUNT}

    KERNELS = {"auto": 0, "simple": 1, "wave": 2, "jit": 2, "binned": 3}

    def set_option(self, key: str, value) -> None:
        if key == "kernel" and isinstance(value, str):
            value = self.KERNELS[value]
        self._chk("pt_set_option", self._L.pt_set_option(self._ctx, key.encode(), int(value)))

    def get_option(self, key: str) -> float:
        v = ctypes.c_double()
        self._chk("pt_get_option", self._L.pt_get_option(self._ctx, key.encode(), ctypes.byref(v)))
        return float(v.value)

    def jit_log(self) -> str:
        raw = self._L.pt_jit_log(self._ctx)
        return raw.decode() if raw else ""

    def set_tiles(self, rank: int, nranks: int) -> None:
        self._chk("pt_set_tiles", self._L.pt_set_tiles(self._ctx, rank, nranks))

    def clear(self) -> None:
        self._chk("pt_resize_clear", self._L.pt_resize_clear(self._ctx, self.size[0], self.size[1]))
        self.constants.last_clear = 0

    def sync(self) -> None:
        self._chk("pt_sync", self._L.pt_sync(self._ctx))

    def last_dispatch_ms(self) -> float:
        ms = ctypes.c_float()
        self._chk("pt_last_dispatch_ms", self._L.pt_last_dispatch_ms(self._ctx, ctypes.byref(ms)))
        return float(ms.value)

    def read_image(self) -> np.ndarray:
        """The accumulation image as float32 [height][width][4], row 0 = y 0."""
        w, h = self.size
        out = np.empty((h, w, 4), dtype=np.float32)
        self._chk("pt_read_accum", self._L.pt_read_accum(self._ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                          out.nbytes))
        return out

    def write_image(self, img: np.ndarray) -> None:
        """Replace the accumulation image (pt_write_accum): float32 [h][w][4]."""
        w, h = self.size
        a = np.ascontiguousarray(img, np.float32)
        if a.shape != (h, w, 4):
            raise ValueError(f"image must be ({h}, {w}, 4), got {a.shape}")
        self._chk("pt_write_accum", self._L.pt_write_accum(self._ctx, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                            a.nbytes))

    def display(self, srgb8: bool = False) -> np.ndarray:
        """The display pass (RenderTexturePipeline::render_pass,
        render_texture_shader.wgsl:23-94) on the device.  srgb8=False: fs_main's
        RGBA32F per texel [height][width][4], row 0 = bottom.  srgb8=True: the
        sRGB swapchain's 8-bit RGBA [height][width][4], row 0 = top of screen."""
        w, h = self.size
        out = np.empty((h, w, 4), dtype=np.uint8 if srgb8 else np.float32)
        fmt = N.PT_DISPLAY_SRGB8 if srgb8 else N.PT_DISPLAY_RGBA32F
        self._chk("pt_display", self._L.pt_display(self._ctx, fmt, out.ctypes.data_as(ctypes.c_void_p), out.nbytes))
        return out

    # -- RCCL ------------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * N.PT_COMM_ID_BYTES)()
        N.check("pt_comm_get_unique_id", N.lib().pt_comm_get_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        buf = (ctypes.c_uint8 * N.PT_COMM_ID_BYTES).from_buffer_copy(uid)
        self._chk("pt_comm_init", self._L.pt_comm_init(self._ctx, nranks, rank, buf))

    def comm_size(self) -> int:
        """Ranks of the context's RCCL communicator (ncclCommCount)."""
        n = ctypes.c_uint32()
        self._chk("pt_comm_size", self._L.pt_comm_size(self._ctx, ctypes.byref(n)))
        return int(n.value)

    def reduce(self, root: int = 0) -> None:
        self._chk("pt_reduce_accum", self._L.pt_reduce_accum(self._ctx, root))

    def save_image(self) -> np.ndarray:
        """State::save_image (state.rs:237-303) without the PNG encoder: the
        blocking readback plus the 8-bit gamma transform (row 0 = top)."""
        return save_image_rgba8(self.read_image())

    def read_reduced(self) -> np.ndarray:
        w, h = self.size
        out = np.empty((h, w, 4), dtype=np.float32)
        self._chk("pt_read_reduced", self._L.pt_read_reduced(self._ctx, out.ctypes.data_as(
            ctypes.POINTER(ctypes.c_float)), out.nbytes))
        return out


def save_image_rgba8(img: np.ndarray) -> np.ndarray:
    """State::save_image pixel transform (state.rs:277-289) on the host, in
    the library (pt_save_rgba8): (v.powf(1.0 / 2.2) * 255.0) as u8 with
    Rust's f32 1.0 / 2.2 and libm powf, alpha * 255, `as u8` saturating (NaN
    -> 0), rows flipped (row 0 = top)."""
    a = np.ascontiguousarray(img, np.float32)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError(f"image must be (h, w, 4), got {a.shape}")
    h, w = a.shape[:2]
    out = np.empty((h, w, 4), np.uint8)
    N.check("pt_save_rgba8", N.lib().pt_save_rgba8(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), w, h,
                                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.nbytes))
    return out


def save_png(img: np.ndarray, path: str) -> None:
    from PIL import Image

    Image.fromarray(save_image_rgba8(img), mode="RGBA").save(path)
