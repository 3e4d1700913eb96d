"""Device arithmetic against the semantics contract."""
import ctypes
import math

import numpy as np
import pytest

import pyref
from compute_path_tracer_amd import _native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def dev(op, a, b=None):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), np.float32)
    out = np.empty_like(a)
    fp = ctypes.POINTER(ctypes.c_float)
    rc = N.lib().pt_device_math(0, N.PT_MATH[op], a.ctypes.data_as(fp), b.ctypes.data_as(fp), out.ctypes.data_as(fp),
                                a.size)
    assert rc == N.PT_OK
    return out


SPECIAL = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38, 0.5, -2.5],
                   np.float32)


@pytest.mark.parametrize("op", ["max", "min"])
def test_min_max_are_ieee_maxnum_minnum(gpu, op):
    a, b = np.meshgrid(SPECIAL, SPECIAL)
    a, b = a.ravel(), b.ravel()
    got = dev(op, a, b)
    f = pyref.gmax if op == "max" else pyref.gmin
    want = np.array([f(x, y) for x, y in zip(a, b)], np.float32)
    nan = np.isnan(got) & np.isnan(want)
    assert np.array_equal(got.view(np.uint32)[~nan], want.view(np.uint32)[~nan])
    assert np.array_equal(np.isnan(got), np.isnan(want))


def test_sqrt_fast_path_equals_ieee_sqrt_for_all_inputs(gpu):
    bad, first = ctypes.c_uint64(), ctypes.c_uint32()
    assert N.lib().pt_check_sqrt_exhaustive(0, ctypes.byref(bad), ctypes.byref(first)) == N.PT_OK
    assert bad.value == 0, hex(first.value)


def test_sqrt_and_div_correctly_rounded(gpu):
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(0, 1e4, 100000), rng.uniform(0, 1e-30, 1000), SPECIAL]).astype(np.float32)
    y = np.concatenate([rng.uniform(-10, 10, 100000), rng.uniform(1e-3, 1, 1000), SPECIAL[::-1]]).astype(np.float32)
    with np.errstate(all="ignore"):
        for op, want in (("sqrt", np.sqrt(x)), ("sqrtf", np.sqrt(x)), ("div", x / y)):
            got = dev(op, x, y)
            ok = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
            assert ok.all(), (op, x[~ok][:4], y[~ok][:4])


def test_sincos_matches_oracle(gpu):
    x = np.concatenate([np.linspace(-50, 50, 20001), [0.0, -0.0, 6.2831855, 16777216.0, 2e7]]).astype(np.float32)
    s, c = dev("sin", x), dev("cos", x)
    for i in range(0, x.size, 97):
        assert np.float32(O.sin(float(x[i]))).view(np.uint32) == s[i:i + 1].view(np.uint32)[0] or \
            (math.isnan(s[i]) and math.isnan(O.sin(float(x[i]))))
        assert np.float32(O.cos(float(x[i]))).view(np.uint32) == c[i:i + 1].view(np.uint32)[0] or \
            (math.isnan(c[i]) and math.isnan(O.cos(float(x[i]))))


def test_fma_is_fused(gpu):
    a = np.float32(1.0000001)
    got = dev("fma", np.array([a], np.float32), np.array([a], np.float32))[0]
    assert got == pyref.fmaf(a, a, np.float32(1.0))


def test_div_rcp_equals_ieee_div_for_all_significand_pairs(gpu):
    """bounds()' reciprocal division against IEEE division for all 2^46 pairs
    of significands (a, b in [1, 2)); with no under/overflow -- what the
    bounds() guards ensure -- power-of-two scaling and sign symmetry carry the
    result to every guarded operand."""
    bad, first = ctypes.c_uint64(), ctypes.c_uint64()
    assert N.lib().pt_check_div_exhaustive(0, 0, 1 << 23, 0, 1 << 23, ctypes.byref(bad), ctypes.byref(first)) == N.PT_OK
    assert bad.value == 0, hex(first.value)


@pytest.mark.parametrize("seed", [1, 2])
def test_div_rcp_on_guarded_operands(gpu, seed):
    """The composed claim on 2^28 random guarded operands per seed: slab
    differences a = x - o of guarded coordinates (zeros included) over guarded
    divisors."""
    bad, first = ctypes.c_uint64(), ctypes.c_uint64()
    assert N.lib().pt_check_div_random(0, seed, 1 << 28, ctypes.byref(bad), ctypes.byref(first)) == N.PT_OK
    assert bad.value == 0, hex(first.value)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5, 6, 7])
def test_margin_decided_slab_test(gpu, mode):
    """bounds()' slab test from reciprocal products (modes
    2-5: one fma per slab, 3.18, 4-5 with far origins and near boxes; 6-7:
    the margin in units of the last place, 3.19): every
    pair the margin decides agrees with the IEEE slab test; the undecided ones
    (ray through a box edge, odd modes) agree after the exact fallback."""
    counts = (ctypes.c_uint64 * 4)()
    n = 1 << 24
    assert N.lib().pt_check_box_random(0, 7 + mode, n, mode, counts) == N.PT_OK
    decided_bad, exact_bad, undecided, skipped = list(counts)
    print(f"mode {mode}: undecided {undecided} of {n}, skipped {skipped}")
    assert decided_bad == 0 and exact_bad == 0
    assert skipped < n // 4
    if mode % 2 == 1:
        assert undecided > 0  # the near-ties reach the fallback


@pytest.mark.parametrize("b", [1.0 / 0.9, 1.0 / 1.1, 0.9, 1.1, 1.0, 3.0, 0.3, 0.0625, 16.0, -1.25,
                               1.9999998807907104, 1.0000001192092896])
def test_div_k_every_numerator(gpu, b):
    """pt_div_k (the baked kernels' division by a scale constant) equals the
    IEEE a / b for all 2^32 numerator patterns: the guarded Markstein range,
    the v_div_fixup specials and the wave fallback."""
    # na is a multiple of 256 below 2^32: two calls cover every pattern,
    # the last 256 (negative NaNs through v_div_fixup) included
    for a0, na in ((0, 0xFFFFFF00), (0xFFFFFF00, 256)):
        bad, first = ctypes.c_uint64(), ctypes.c_uint64()
        assert N.lib().pt_check_div_k(0, ctypes.c_float(b), a0, na, ctypes.byref(bad), ctypes.byref(first)) == N.PT_OK
        assert bad.value == 0, (hex(a0), hex(first.value))
