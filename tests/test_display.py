"""Display pass (render_texture_shader.wgsl:23-94).

CPU: the oracle's restatement against float64 evaluations of the WGSL
formulas (pow within one f32 ulp, the contract's bound).  GPU: pt_display
bit-exact against the oracle for both formats, special values included."""
import math

import numpy as np
import pytest

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.path_tracer import PathTracer
from compute_path_tracer_amd.sdf_editor import CompData
from oracle import oracle as O

SPECIAL = [0.0, -0.0, 1e-30, 0.0031308, 0.00313, 0.0032, 0.5, 1.0, 2.0, 10.0, 1e6, np.inf, -np.inf, np.nan, -1.0]


def _image(seed=0, h=37, w=29):
    rng = np.random.default_rng(seed)
    img = rng.exponential(0.6, (h, w, 4)).astype(np.float32)
    flat = img.reshape(-1)
    flat[:len(SPECIAL)] = np.array(SPECIAL, np.float32)
    return img


def _ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    return np.abs(ai - bi)


def test_pow_within_one_ulp_of_true_pow():
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(0.0031308, 1.0, 20000), np.geomspace(1e-30, 1e30, 2000)]).astype(np.float32)
    y = np.float32(1.0 / 2.4)
    got = np.array([O.pow_pos(float(x), float(y)) for x in xs], np.float32)
    want = np.array([math.pow(float(x), float(y)) for x in xs], np.float32)  # RN of the (near-)exact value
    assert _ulp_diff(got, want).max() <= 1


def _wgsl_f64(x):
    """fs_main's channel transform in float64 (no f32 rounding at all)."""
    x = np.asarray(x, np.float64)
    n, d = x * (2.51 * x + 0.03), x * (2.43 * x + 0.59) + 0.14
    with np.errstate(all="ignore"):
        a = np.clip(np.nan_to_num(n / d, nan=0.0), 0.0, 1.0)
    return np.where(a < 0.0031308, a * 12.92, np.power(a, 1 / 2.4) * 1.055 - 0.055)


def test_oracle_display_matches_float64_formula():
    img = _image()
    got = O.display(img)[..., :3].astype(np.float64)
    want = _wgsl_f64(img[..., :3])
    finite = np.isfinite(img[..., :3])
    assert np.abs(got - want)[finite].max() < 2e-6
    assert np.all(O.display(img)[..., 3] == 1.0)


def test_oracle_srgb8_is_screen_order_and_double_encoded():
    img = _image(1)
    fs = O.display(img)
    s8 = O.display(img, srgb8=True)
    h = img.shape[0]
    c = np.clip(fs[..., :3].astype(np.float64), 0, 1)
    enc = np.where(c < 0.0031308, c * 12.92, np.power(c, 1 / 2.4) * 1.055 - 0.055)
    want = np.rint(enc * 255.0)
    diff = np.abs(s8[::-1][..., :3].astype(np.int32) - want.astype(np.int32))  # screen row 0 = texel row h-1
    assert diff.max() <= 1 and (diff == 0).mean() > 0.99
    assert np.all(s8[..., 3] == 255)
    assert np.array_equal(s8[0], O.display(img[h - 1:h], srgb8=True)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("srgb8", [False, True])
def test_gpu_display_bit_exact(gpu, srgb8):
    ed = scenes.c2_sphere_box_torus()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=4, scale=1.0, fov=1.0, aabb=0)
    w, h = 61, 37
    pt = PathTracer(w, h, prog, settings=st)
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=float(np.float32(w) / np.float32(h)), last_clear=1), 3)
    img = pt.read_image()
    img.reshape(-1)[:len(SPECIAL)] = np.array(SPECIAL, np.float32)  # special values through the device path too
    q = PathTracer(w, h, prog, settings=st)
    q.write_image(img)
    assert np.array_equal(q.read_image().view(np.uint32), img.view(np.uint32))
    got = q.display(srgb8=srgb8)
    want = O.display(img, srgb8=srgb8)
    same = got.view(np.uint32 if not srgb8 else np.uint8) == want.view(np.uint32 if not srgb8 else np.uint8)
    assert same.all(), np.argwhere(~same)[:5]
    ms = q.get_option("display_ms")
    assert ms > 0.0
    pt.close()
    q.close()
