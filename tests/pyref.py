"""Second, independent restatement of the reference path in pure Python with
numpy float32 scalars (test infrastructure).  Used on tiny images to
cross-check the C oracle (oracle/pt_oracle.c) bit for bit; the two were
written separately from the same GLSL (test_compute.glsl, rng.glsl,
funcs.glsl, shapes.glsl, aabb.glsl) and generator (src/sdf_editor/*).

float32 semantics: numpy float32 scalar + - * / and sqrt are IEEE correctly
rounded; fmaf (needed only by the sin/cos contract) is computed exactly with
fractions and rounded once to float32.
"""
from __future__ import annotations

import math
from fractions import Fraction
from typing import List, Sequence

import numpy as np

F = np.float32
U32 = 0xFFFFFFFF


def _rn32(q: Fraction) -> np.float32:
    """Round an exact rational to the nearest float32 (ties to even)."""
    if q == 0:
        return F(0.0)
    sign = -1 if q < 0 else 1
    a = abs(q)
    e = math.floor(math.log2(a.numerator) - math.log2(a.denominator))
    while Fraction(2) ** e > a:
        e -= 1
    while Fraction(2) ** (e + 1) <= a:
        e += 1
    e = max(e, -126)
    scale = Fraction(2) ** (e - 23)
    m = a / scale
    fl = m.numerator // m.denominator
    rem = m - fl
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and fl % 2 == 1):
        fl += 1
    return F(sign * float(fl * scale))


def fmaf(a, b, c) -> np.float32:
    return _rn32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def gmin(x, y):
    """IEEE-754 minNum with -0 < +0 (SPIR-V FMin on AMD hardware)."""
    x, y = F(x), F(y)
    if np.isnan(x):
        return y
    if np.isnan(y):
        return x
    if x == 0 and y == 0:
        return F(-0.0) if (np.signbit(x) or np.signbit(y)) else F(0.0)
    return y if y < x else x


def gmax(x, y):
    """IEEE-754 maxNum with -0 < +0 (SPIR-V FMax on AMD hardware)."""
    x, y = F(x), F(y)
    if np.isnan(x):
        return y
    if np.isnan(y):
        return x
    if x == 0 and y == 0:
        return F(-0.0) if (np.signbit(x) and np.signbit(y)) else F(0.0)
    return y if x < y else x


# ---------------------------------------------------------------- rng.glsl
def wang_hash(s: int) -> int:
    s = ((s ^ 61) ^ (s >> 16)) & U32
    s = (s * 9) & U32
    s = s ^ (s >> 4)
    s = (s * 0x27D4EB2D) & U32
    s = s ^ (s >> 15)
    return s


class Rng:
    def __init__(self, seed: int):
        self.s = seed & U32

    def f01(self) -> np.float32:
        self.s = wang_hash(self.s)
        return F(self.s) / F(4294967296.0)


def gen_rng(x, y, frame, w, h) -> int:
    a = int(F(F(F(x) * F(0.5)) + F(0.5)) * F(w))
    b = int(F(F(F(y) * F(0.5)) + F(0.5)) * F(h))
    return ((a * 1973 + b * 9277 + (frame & U32) * 26699) & U32) | 1


# ------------------------------------------------------- sin/cos contract
def _sinp(r):
    s = r * r
    p = fmaf(s, F(-1.9515295891e-4), F(8.3321608736e-3))
    p = fmaf(s, p, F(-1.6666654611e-1))
    return fmaf(r * s, p, r)


def _cosp(r):
    s = r * r
    p = fmaf(s, F(2.443315711809948e-5), F(-1.388731625493765e-3))
    p = fmaf(s, p, F(4.166664568298827e-2))
    t = fmaf(s, p, F(-0.5))
    return fmaf(s, t, F(1.0))


def sincos(x):
    x = F(x)
    if not abs(x) <= F(16777216.0):
        return F(np.nan), F(np.nan)
    k = F(np.rint(x * F(0.63661977236758134)))
    r = fmaf(-k, F(1.5703125), x)
    r = fmaf(-k, F(4.837512969970703125e-4), r)
    r = fmaf(-k, F(7.549789954891882e-8), r)
    q = int(k) & 3
    sp, cp = _sinp(r), _cosp(r)
    return [(sp, cp), (cp, -sp), (-sp, -cp), (-cp, sp)][q]


# ------------------------------------------------------------ vectors
def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def length(a):
    return F(np.sqrt(dot(a, a)))


def normalize(a):
    l = length(a)
    return [a[0] / l, a[1] / l, a[2] / l]


# ------------------------------------------------------------ scene
class Scene:
    """Tree + slot allocation (SDFEditor::compile restated)."""

    def __init__(self, rows: Sequence[dict]):
        self.rows = rows
        n = len(rows)
        self.cu = [[] for _ in range(n)]
        self.cs = [[] for _ in range(n)]
        self.top = []
        for i, r in enumerate(rows):
            if r["parent"] == -1:
                self.top.append(i)
            elif r["kind"] == 0:
                self.cu[r["parent"]].append(i)
            else:
                self.cs[r["parent"]].append(i)
        self.data: List[np.float32] = [F(6969.69)]
        self.slot = [dict() for _ in range(n)]
        self.check = [-1] * n
        self.bidx = [-1] * n
        idx = [0]

        def alloc(v):
            self.data.append(F(v))
            return len(self.data) - 1

        def tr(i):
            r = rows[i]
            s = self.slot[i]
            s["scale"] = alloc(r["scale"])
            s["pos"] = [alloc(v) for v in r["position"]]
            s["rot"] = [alloc(v) for v in r["rotation"]]
            s["ex"] = alloc(r["aabb_exaggeration"])

        def comp(u):
            tr(u)
            for c in self.cu[u]:
                comp(c)
            for c in self.cs[u]:
                tr(c)
                nsz = {1: 1, 2: 3, 3: 2, 4: 1}[rows[c]["kind"]]
                self.slot[c]["size"] = [alloc(rows[c]["size"][k]) for k in range(nsz)]
                self.slot[c]["mat"] = [alloc(v) for v in rows[c]["material"]]
                self.check[c] = idx[0] if rows[c]["aabb"] else -1
                idx[0] += 1

        for u in self.top:
            comp(u)
        self.n_check = max(1, idx[0])
        self.bounds_list = []
        b = 0
        for u in self.top:
            for c in self.cs[u]:
                self.bidx[c] = b
                self.bounds_list.append((c, u, b))
                b += 1

    def d(self, i):
        return self.data[i]

    def xform(self, i, p):
        s = self.slot[i]
        inv = F(1.0) / self.d(s["scale"])
        q = [p[0] * inv, p[1] * inv, p[2] * inv]
        m = [self.d(s["pos"][k]) * inv for k in range(3)]
        q = [q[0] - m[0], q[1] - m[1], q[2] - m[2]]
        rx, ry, rz = (self.d(s["rot"][k]) for k in range(3))
        sx, cx = sincos(rx)
        sy, cy = sincos(ry)
        sz, cz = sincos(rz)
        z0 = F(0.0)
        o1 = F(1.0)
        # column-major constructors; result row r = c0[r]*v.x + c1[r]*v.y + c2[r]*v.z
        for cols in (((o1, z0, z0), (z0, cx, -sx), (z0, sx, cx)),
                     ((cy, z0, sy), (z0, o1, z0), (-sy, z0, cy)),
                     ((cz, -sz, z0), (sz, cz, z0), (z0, z0, o1))):
            q = [cols[0][r] * q[0] + cols[1][r] * q[1] + cols[2][r] * q[2] for r in range(3)]
        return q

    def sdf(self, i, p):
        k = self.rows[i]["kind"]
        sz = [self.d(j) for j in self.slot[i]["size"]]
        if k == 1:
            return length(p) - sz[0]
        if k == 2:
            q = [F(abs(p[j])) - sz[j] for j in range(3)]
            m = [gmax(v, F(0.0)) for v in q]
            return length(m) + gmin(gmax(q[0], gmax(q[1], q[2])), F(0.0))
        if k == 3:
            qx = F(np.sqrt(p[0] * p[0] + p[2] * p[2])) - sz[0]
            return F(np.sqrt(qx * qx + p[1] * p[1])) - sz[1]
        s = sz[0]
        a = [F(abs(v)) for v in p]
        m = a[0] + a[1] + a[2] - s
        if F(3.0) * a[0] < m:
            q = a
        elif F(3.0) * a[1] < m:
            q = [a[1], a[2], a[0]]
        elif F(3.0) * a[2] < m:
            q = [a[2], a[0], a[1]]
        else:
            return m * F(0.57735027)
        kk = gmin(gmax(F(0.5) * (q[2] - q[1] + s), F(0.0)), s)
        return length([q[0], q[1] - s + kk, q[2] - kk])

    @staticmethod
    def comb(t, a, b):
        if t == 0:
            return a if a[0] < b[0] else b
        n = (-a[0], a[1])
        depth = gmax(n[0], b[0])
        return n if depth == n[0] else b

    def map_union(self, u, pp, check, ref, tin):
        uk = (F(10000.0), -1)
        p = self.xform(u, pp)
        for c in self.cu[u]:
            uk = self.map_union(c, p, check, uk, self.rows[u]["union_type"])
        for i, c in enumerate(self.cs[u]):
            if self.check[c] >= 0 and not check[self.check[c]]:
                continue
            q = self.xform(c, p)
            h = (self.sdf(c, q) / (F(1.0) / self.d(self.slot[c]["scale"])), c)
            uk = h if i == 0 else self.comb(self.rows[u]["union_type"], uk, h)
        uk = (uk[0] / (F(1.0) / self.d(self.slot[u]["scale"])), uk[1])
        return self.comb(tin, ref, uk)

    def map(self, p, check):
        st = (F(10000.0), -1)
        for u in self.top:
            st = self.map_union(u, p, check, st, 0)
        return st

    def bounds(self, ro, rd):
        check = [False] * self.n_check
        dbg = F(0.0)
        for c, u, b in self.bounds_list:
            if not self.rows[c]["aabb"]:
                continue
            sc, uc = self.slot[c], self.slot[u]
            ctr = [self.d(uc["pos"][k]) + self.d(sc["pos"][k]) for k in range(3)]
            kind = self.rows[c]["kind"]
            sz = [self.d(j) for j in sc["size"]]
            so = {1: [sz[0]] * 3, 4: [sz[0]] * 3, 2: sz}.get(kind)
            if kind == 3:
                so = [sz[0] + sz[1], sz[1], sz[0] + sz[1]]
            s2 = self.d(uc["scale"]) * self.d(sc["scale"])
            ex = self.d(sc["ex"])
            hs = [(so[k] * s2) * ex for k in range(3)]
            t1, t2 = [], []
            for k in range(3):
                tmin = ((ctr[k] - hs[k]) - ro[k]) / rd[k]
                tmax = ((ctr[k] + hs[k]) - ro[k]) / rd[k]
                t1.append(gmin(tmin, tmax))
                t2.append(gmax(tmin, tmax))
            tn = gmax(gmax(t1[0], t1[1]), t1[2])
            tf = gmin(gmin(t2[0], t2[1]), t2[2])
            if tn < tf and tf > F(0.0):
                check[b] = True
                dbg = dbg + F(0.1)
        return check, dbg

    def mat(self, m):
        if m < 0:
            return dict(col=[F(0)] * 3, br=F(0), light=[F(0)] * 3, spec=F(0), sc=[F(0)] * 3, rough=F(0))
        s = [self.d(j) for j in self.slot[m]["mat"]]
        return dict(col=s[0:3], br=s[3], light=s[4:7], spec=s[7], sc=s[8:11], rough=s[11])


def cast_ray(sc, ro, rd, check):
    t = F(0.0)
    mat = -1
    for _ in range(80):
        p = [ro[k] + rd[k] * t for k in range(3)]
        d, m = sc.map(p, check)
        mat = m
        t = t + d
        if F(abs(d)) < F(0.001):
            break
        if t > F(100.0):
            return t, -1
    return t, mat


def calc_normal(sc, p, check):
    e = F(0.0001)
    v = []
    for a in range(3):
        ep = [F(0.0)] * 3
        en = [F(-0.0)] * 3
        ep[a] = e
        en[a] = -e
        dp = sc.map([p[k] + ep[k] for k in range(3)], check)[0]
        dn = sc.map([p[k] + en[k] for k in range(3)], check)[0]
        v.append(dp - dn)
    return normalize(v)


PI2 = F(2.0) * F(3.14159265359)


def path_trace(sc, ro, rd, rng, bounces, debug):
    ret = [F(0)] * 3
    thr = [F(1)] * 3
    i = 0
    while i <= bounces:
        check, _ = sc.bounds(ro, rd)
        t, m = cast_ray(sc, ro, rd, check)
        if t > F(100.0):
            break
        hp = [ro[k] + rd[k] * t for k in range(3)]
        n = calc_normal(sc, hp, check)
        ro = [hp[k] + n[k] * F(0.03) for k in range(3)]
        mt = sc.mat(m)
        do_spec = rng.f01() < mt["spec"]
        prob = gmax(mt["spec"] if do_spec else F(1.0) - mt["spec"], F(0.0001))
        z = rng.f01() * F(2.0) - F(1.0)
        a = rng.f01() * PI2
        r = F(np.sqrt(F(1.0) - z * z))
        sa, ca = sincos(a)
        diffuse = normalize([n[0] + r * ca, n[1] + r * sa, n[2] + z])
        if do_spec:
            kk = F(2.0) * dot(n, rd)
            sr = [rd[k] - kk * n[k] for k in range(3)]
            al = mt["rough"] * mt["rough"]
            rd = normalize([sr[k] * (F(1.0) - al) + diffuse[k] * al for k in range(3)])
        else:
            rd = diffuse
        nl = normalize(mt["light"])
        fs = F(1.0) if do_spec else F(0.0)
        for k in range(3):
            ret[k] = ret[k] + (nl[k] * mt["br"]) * thr[k]
            thr[k] = thr[k] * (mt["col"][k] * (F(1.0) - fs) + mt["sc"][k] * fs)
            thr[k] = thr[k] / prob
        p = gmax(thr[0], gmax(thr[1], thr[2]))
        if rng.f01() > p:
            break
        ip = F(1.0) / p
        thr = [thr[k] * ip for k in range(3)]
        i += 1
    if debug == 3:
        v = F(i) / F(bounces)
        return [v, v, v]
    return ret


def render(rows, w, h, frame, last_clear, aspect, bounces, spp, debug=0, fov=1.0, image=None):
    sc = Scene(rows)
    img = np.zeros((h, w, 4), np.float32) if image is None else image
    with np.errstate(all="ignore"):
        for y in range(h):
            for x in range(w):
                for j in range(spp):
                    rng = Rng(gen_rng(x, y, frame + j, w, h))
                    jx = rng.f01() - F(0.5)
                    jy = rng.f01() - F(0.5)
                    ux = ((F(x) + jx) / F(w)) * F(2.0) - F(1.0)
                    uy = ((F(y) + jy) / F(h)) * F(2.0) - F(1.0)
                    ux = ux * F(aspect)
                    rd = normalize([ux, uy, F(fov)])
                    ro = [F(0.0), F(0.0), F(-3.0)]
                    if debug in (0, 3):
                        col = path_trace(sc, ro, rd, rng, bounces, debug)
                    elif debug == 1:
                        check, dbg = sc.bounds(ro, rd)
                        t, m = cast_ray(sc, ro, rd, check)
                        if t > F(100.0):
                            col = [dbg] * 3
                        else:
                            hp = [ro[k] + rd[k] * t for k in range(3)]
                            nn = normalize(calc_normal(sc, hp, check))
                            col = [(nn[k] * F(0.5) + F(0.5)) * F(0.2) + dbg for k in range(3)]
                    elif debug == 2:
                        check, _ = sc.bounds(ro, rd)
                        t, m = cast_ray(sc, ro, rd, check)
                        col = sc.mat(m)["col"]
                    else:
                        col = [F(0.0)] * 3
                    px = img[y, x]
                    if debug != 0:
                        px[:3] = col
                    else:
                        wgt = F(1.0) / F(last_clear + j + 1)
                        for k in range(3):
                            px[k] = F(px[k]) * (F(1.0) - wgt) + F(col[k]) * wgt
                    px[3] = F(1.0)
    return img
