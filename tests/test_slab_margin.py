"""CPU check of the decision rules behind bounds()' fast slab tests
(DESIGN.md 3.14 and 3.19), in numpy float32 (IEEE, correctly rounded, no
contraction): the slab values from reciprocal products t' = RN(RN(b - o) * y),
y = RN(1/d), decide `tnear < tfar && tfar > 0` exactly like the reference's
RN(RN(b - o) / d) (aabb.glsl:21-33) whenever the margin says so.

The device runs the same rules (pt_path.h ray_box_approx / ray_box_ulp) and
pt_selftest.hip checks them there; this restatement pins the arithmetic
argument itself on the host, including the ulp margin's slack (> 8 steps
suffices, the kernels use 16)."""
import numpy as np
import pytest

F = np.float32


def _coord_ok(x):
    u = x.view(np.uint32) & np.uint32(0x7FFFFFFF)
    return (u == 0) | ((u - np.uint32(0x2D800000)) <= np.uint32(0x5D000000 - 0x2D800000))


def _dir_ok(d):
    u = d.view(np.uint32) & np.uint32(0x7FFFFFFF)
    return (u - np.uint32(0x35800000)) <= np.uint32(0x5D000000 - 0x35800000)


def _pairs(n, edge, rng):
    """Random guarded (ray, box) pairs around a point p = o + d t on the ray;
    `edge` puts the entry and exit faces through p (the near-ties)."""
    o = (rng.integers(-32768, 32768, (n, 3)).astype(F) * F(4.0 / 32768.0)).astype(F)
    d = rng.standard_normal((n, 3)).astype(F)
    d = np.where(np.abs(d) < F(2.0 ** -20), F(1.0), d).astype(F)
    t = (F(0.5) + rng.random(n).astype(F) * F(16.0)).astype(F)
    p = (o + d * t[:, None]).astype(F)
    r1 = (F(0.01) + rng.random((n, 3)).astype(F) * F(2.0)).astype(F)
    r2 = (F(0.01) + rng.random((n, 3)).astype(F) * F(2.0)).astype(F)
    bmin, bmax = (p - r1).astype(F), (p + r2).astype(F)
    if edge:
        a1 = rng.integers(0, 3, n)
        a2 = (a1 + 1 + rng.integers(0, 2, n)) % 3
        i = np.arange(n)
        u1 = rng.integers(-4, 5, n).astype(np.int64)
        u2 = rng.integers(-4, 5, n).astype(np.int64)
        j1 = (p[i, a1].view(np.uint32).astype(np.int64) + u1).astype(np.uint32).view(F)
        j2 = (p[i, a2].view(np.uint32).astype(np.int64) + u2).astype(np.uint32).view(F)
        pos1, pos2 = d[i, a1] > 0, d[i, a2] > 0
        bmin[i[pos1], a1[pos1]] = j1[pos1]
        bmax[i[~pos1], a1[~pos1]] = j1[~pos1]
        bmax[i[pos2], a2[pos2]] = j2[pos2]
        bmin[i[~pos2], a2[~pos2]] = j2[~pos2]
    ok = (_coord_ok(o) & _dir_ok(d) & _coord_ok(bmin) & _coord_ok(bmax)).all(axis=1)
    return o[ok], d[ok], bmin[ok], bmax[ok]


def _ends(t0, t1):
    lo, hi = np.minimum(t0, t1), np.maximum(t0, t1)
    return lo.max(axis=1), hi.min(axis=1)


@pytest.mark.parametrize("edge", [False, True])
def test_margins_decide_like_the_ieee_slab_test(edge):
    rng = np.random.default_rng(20261017 + int(edge))
    o, d, bmin, bmax = _pairs(1 << 21, edge, rng)
    with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
        tn, tf = _ends((bmin - o) / d, (bmax - o) / d)  # the reference: RN(RN(b - o) / d)
        y = (F(1.0) / d).astype(F)
        tn2, tf2 = _ends(((bmin - o) * y).astype(F), ((bmax - o) * y).astype(F))
    want = (tn < tf) & (tf > 0)
    got = (tn2 < tf2) & (tf2 > 0)
    # 3.14: the float margin
    gap = np.abs(tf2 - tn2) - (np.abs(tn2) + np.abs(tf2)) * F(2.0 ** -20)
    dec = gap > 0
    assert not (dec & (got != want)).any()
    # 3.19: the ulp margin, at the kernels' 16 and at the proof's 8
    sad = np.abs(tf2.view(np.uint32).astype(np.int64) - tn2.view(np.uint32).astype(np.int64))
    for margin in (16, 8):
        dec_u = sad > margin
        assert not (dec_u & (got != want)).any(), margin
    # (and the margins are not vacuous: undecided by them, the approximate
    # answer alone is wrong for some near-ties)
    if edge:
        assert (got != want).any()
    und = float(np.mean(~(sad > 16)))
    print(f"edge={edge}: {len(o)} pairs, undecided {und:.4f} (ulp) vs {float(np.mean(~dec)):.4f} (float margin)")
    if edge:
        assert und > 0.3  # the near-ties reach the exact fallback
    else:
        assert und < 1e-3
