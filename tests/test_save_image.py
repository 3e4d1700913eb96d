"""State::save_image's pixel transform (src/state.rs:277-289), SURVEY 8(f)
row 2: byte-exact against an independent restatement.  No GPU.

Restatement: Rust's `1.0 / 2.2` in f32 (both literals f32: RN(1 / RN(2.2)),
0x3EE8BA2E), f32::powf = the platform libm powf (glibc here, called through
ctypes one value at a time), `* 255.0` in f32, `as u8` saturating (NaN -> 0,
<= 0 -> 0, >= 255 -> 255, else truncation), output row y = input row
height - 1 - y.  Parity vs a real Rust build is unpinned (no cargo here);
the Rust semantics above are the language's documented ones."""
import ctypes
import math

import numpy as np

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd.path_tracer import save_image_rgba8

_m = ctypes.CDLL("libm.so.6")
_m.powf.restype = ctypes.c_float
_m.powf.argtypes = [ctypes.c_float, ctypes.c_float]
GAMMA = np.float32(1.0) / np.float32(2.2)


def _as_u8(v: np.float32) -> int:
    v = float(v)
    if math.isnan(v) or v <= 0.0:
        return 0
    if v >= 255.0:
        return 255
    return int(v)


def _restated(img: np.ndarray) -> np.ndarray:
    h, w, _ = img.shape
    out = np.zeros((h, w, 4), np.uint8)
    for y in range(h):
        for x in range(w):
            px = img[h - 1 - y, x]
            for k in range(3):
                out[y, x, k] = _as_u8(np.float32(_m.powf(float(px[k]), float(GAMMA))) * np.float32(255.0))
            out[y, x, 3] = _as_u8(px[3] * np.float32(255.0))
    return out


def _special_values() -> np.ndarray:
    """NaNs, signed zeros and infinities, negatives, subnormals, values > 1,
    and every byte boundary (x with x^(1/2.2) * 255 = k) +- 40 ulps."""
    f = np.float32
    vals = [f(np.nan), -f(np.nan), f(0.0), f(-0.0), f(np.inf), f(-np.inf), f(-1e-3), f(-2.0), f(1e-45), f(1e-40),
            f(1.0), f(1.0000001), f(1.5), f(2.0), f(1e30), np.nextafter(f(1.0), f(0.0)), f(3.4e38)]
    ks = np.arange(0, 257, dtype=np.float64)
    xs = (ks / 255.0) ** 2.2
    bits = xs.astype(np.float32).view(np.int32)
    around = (bits[:, None] + np.arange(-40, 41)[None, :]).astype(np.int32).ravel()
    around = around[around >= 0].view(np.float32)
    return np.concatenate([np.array(vals, np.float32), around])


def test_gamma_constant_is_rusts_f32_division():
    assert GAMMA.view(np.uint32) == 0x3EE8BA2E
    assert np.float32(1.0 / 2.2).view(np.uint32) == 0x3EE8BA2F  # the one-ulp-off double rounding


def test_save_transform_byte_exact_on_special_and_boundary_values():
    v = _special_values()
    n = (v.size + 3) // 4 * 4
    v = np.concatenate([v, np.zeros(n - v.size, np.float32)])
    img = v.reshape(-1, 1, 4)  # one texel per row: rows flip
    got = save_image_rgba8(img)
    want = _restated(img)
    assert got.dtype == np.uint8 and got.shape == want.shape
    bad = np.argwhere(got != want)
    assert bad.size == 0, [(tuple(i), float(img[img.shape[0] - 1 - i[0], i[1], i[2]])) for i in bad[:5]]


def test_save_transform_random_image_with_row_flip():
    rng = np.random.default_rng(5)
    img = (rng.random((37, 53, 4), dtype=np.float32) * np.float32(1.3)).astype(np.float32)
    img[3, 4, 1] = np.nan
    img[0, 0, 3] = 1.0
    got = save_image_rgba8(img)
    assert np.array_equal(got, _restated(img))
    assert got[36, 0, 3] == 255 and got[33, 4, 1] == 0  # row 0 of the input is the PNG's last row


def test_save_transform_threads_and_errors():
    """Tall images take the threaded path (row blocks): the same bytes."""
    rng = np.random.default_rng(6)
    img = rng.random((1024, 3, 4), dtype=np.float32)
    got = save_image_rgba8(img)
    assert np.array_equal(got[::97], _restated(img)[::97])
    out = (ctypes.c_uint8 * 4)()
    one = np.zeros(4, np.float32)
    assert N.lib().pt_save_rgba8(one.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 1, 1, out, 3) == N.PT_ERR_SIZE
    assert N.lib().pt_save_rgba8(None, 1, 1, out, 4) == N.PT_ERR_INVALID
    assert N.lib().pt_save_rgba8(None, 0, 0, None, 0) == N.PT_OK
