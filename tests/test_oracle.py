"""The CPU oracle against the committed fixtures and the independent Python
restatement (tests/pyref.py).  No GPU."""
import hashlib
import json
import math
import os

import numpy as np
import pytest

import pyref
from compute_path_tracer_amd import scenes
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_rng_known_answers():
    kat = json.load(open(os.path.join(GOLD, "rng_kat.json")))
    for seed, seq in kat["wang_hash"].items():
        s = int(seed)
        for v in seq:
            s2 = O.wang_hash(s)
            assert s2 == v == pyref.wang_hash(s)
            s = s2
    for g in kat["gen_rng"]:
        assert O.gen_rng(g["x"], g["y"], g["frame"], g["w"], g["h"]) == g["seed"]
    for r in kat["random01"]:
        bits = [int(np.float32(v).view(np.uint32)) for v in O.random01_seq(r["seed"], len(r["bits"]))]
        assert bits == r["bits"]


def test_random01_range_and_exactness():
    # float(u)/2^32 rounds to exactly 1.0 for u >= 2^32 - 128 (rng.glsl:11-14)
    s = 0xFFFFFFFF
    assert O.random01_seq(0, 1)[0] == np.float32(O.wang_hash(0)) / np.float32(4294967296.0)
    assert pyref.Rng(s).f01() >= 0.0


def test_sincos_contract():
    xs = np.concatenate([np.linspace(-7.0, 7.0, 2001, dtype=np.float32),
                         np.float32([0.0, -0.0, 1e-30, 3.14159265, 6.2831855, 1000.5, -12345.67, 16777216.0])])
    for x in xs:
        s, c = pyref.sincos(x)
        assert np.float32(O.sin(float(x))).view(np.uint32) == np.float32(s).view(np.uint32)
        assert np.float32(O.cos(float(x))).view(np.uint32) == np.float32(c).view(np.uint32)
        if abs(x) < 8.0:
            assert abs(float(s) - math.sin(float(x))) < 4e-7
            assert abs(float(c) - math.cos(float(x))) < 4e-7
    assert math.isnan(O.sin(float("inf"))) and math.isnan(O.cos(float("nan")))


@pytest.mark.parametrize("name", sorted(json.load(open(os.path.join(GOLD, "oracle_images.json")))))
def test_oracle_golden_images(name):
    meta = json.load(open(os.path.join(GOLD, "oracle_images.json")))[name]
    rows = scenes.SCENES[meta["scene"]]().rows()
    w, h = meta["w"], meta["h"]
    a = float(np.float32(w) / np.float32(h))
    img = O.OracleScene(rows).render(w, h, O.Constants(0.0, meta["frame"], a, meta["last_clear"]),
                                     O.Settings(meta["debug"], meta["bounces"], 1.0, 1.0, 0), meta["spp"])
    gold = np.load(os.path.join(GOLD, name + ".npy"), allow_pickle=False)
    assert hashlib.sha256(gold.tobytes()).hexdigest() == meta["sha256"]
    assert np.array_equal(img.view(np.uint32), gold.view(np.uint32))


def test_oracle_matches_python_restatement_live():
    rows = scenes.c2_sphere_box_torus().rows()
    a = float(np.float32(6) / np.float32(5))
    img = O.OracleScene(rows).render(6, 5, O.Constants(0.0, 7, a, 3), O.Settings(0, 3, 1.0, 1.0, 0), 2)
    py = pyref.render(rows, 6, 5, 7, 3, a, 3, 2)
    assert np.array_equal(img.view(np.uint32), py.view(np.uint32))


def test_empty_scene_renders_black():
    img = O.OracleScene(scenes.empty().rows()).render(16, 8, O.Constants(0.0, 1, 2.0, 1), O.Settings(0, 4, 1, 1, 0), 3)
    assert np.all(img[..., :3] == 0) and np.all(img[..., 3] == 1)


def test_accumulation_identity():
    """A_n = mix(A_{n-1}, c_n, 1/(n+1)) starting from 0: the image after n
    one-frame dispatches equals one n-frame dispatch, and equals the running
    mix of the individual frames (test_compute.glsl:242-245)."""
    rows = scenes.c1_default().rows()
    osc = O.OracleScene(rows)
    st = O.Settings(0, 1, 1.0, 1.0, 0)
    w = h = 16
    batched = osc.render(w, h, O.Constants(0.0, 1, 1.0, 1), st, 4)
    step = np.zeros((h, w, 4), np.float32)
    for k in range(4):
        osc.render(w, h, O.Constants(0.0, 1 + k, 1.0, 1 + k), st, 1, image=step)
    assert np.array_equal(batched.view(np.uint32), step.view(np.uint32))
    # the same from the per-frame colours: last_clear = 0 makes mix(A, c, 1) = c
    acc = np.zeros((h, w, 3), np.float32)
    for k in range(4):
        c = osc.render(w, h, O.Constants(0.0, 1 + k, 1.0, 0), st, 1)[..., :3]
        wgt = np.float32(1.0) / np.float32(k + 2)
        acc = acc * (np.float32(1.0) - wgt) + c * wgt
    assert np.array_equal(acc.view(np.uint32), batched[..., :3].view(np.uint32))
    assert batched[..., 3].min() == 1.0


def test_sdf_and_bounds_values():
    ed = scenes.c1_default()
    osc = O.OracleScene(ed.rows())
    d, m = osc.map((0.0, 0.0, -3.0))
    assert d == np.float32(2.0) and m >= 0  # unit sphere at the origin
    d, _ = osc.map((0.0, 0.0, 0.0))
    assert d == -1.0
    check, dbg = osc.bounds((0.0, 0.0, -3.0), (0.0, 0.0, 1.0))
    assert check[0] == 1 and np.isclose(dbg[0], 0.1)
    check, dbg = osc.bounds((0.0, 0.0, -3.0), (0.0, 1.0, 0.0))
    assert check[0] == 0 and dbg[0] == 0.0
    # a culled shape is skipped: map with check false returns MAXHIT
    d, m = osc.map((0.0, 0.0, -3.0), check=[0])
    assert d == 10000.0 and m == -1


def test_tile_partition_covers_image():
    rows = scenes.c2_sphere_box_torus().rows()
    osc = O.OracleScene(rows)
    st = O.Settings(0, 2, 1.0, 1.0, 0)
    c = O.Constants(0.0, 1, 1.5, 1)
    full = osc.render(20, 13, c, st, 1)
    acc = np.zeros_like(full)
    for r in range(3):
        acc += osc.render(20, 13, c, st, 1, rank=r, nranks=3)
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32))
