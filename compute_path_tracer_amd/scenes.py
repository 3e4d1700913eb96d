"""Synthetic scenes for BASELINE.json's configurations.

All scenes are built through the editor mirror (:mod:`.sdf_editor`) so they
exercise the same compile path a user scene takes.  Values are deterministic.

* ``c1_default`` -- the editor's default scene (sdf_editor.rs:26-27: one Union
  holding one unit Sphere, AABB on, exaggeration 1.3) with brightness 1 so the
  image is not black (the default Material has brightness 0).
* ``c2_sphere_box_torus`` -- (sphere U box) - torus expressed in the
  reference's union semantics: header union A (Subtraction) = [torus, sphere]
  -> sphere - torus; header union B (Subtraction) = [torus, box] -> box -
  torus; the header level always unions, giving (sphere U box) - torus.  Plus
  one emissive sphere.  The torus is a build extension (absent upstream).
* ``c3_graph32`` -- a flat 32-node graph: 4 header unions x 7 shapes.  Union 0
  is the Cornell-like room of the reference's saved scene assets/maps/test.json
  (floor, roof, emissive light box, tilted back wall, two side walls; values
  copied, light colour (0,0,0) of non-emitters replaced by the live editor's
  default (1,1,1) because the current Mat normalises it), plus the two
  rough-specular octahedra of that file in union 1; the rest is drawn from a
  fixed PRNG (seed 42): spheres/cubes, sizes in [0.2, 0.75], rotations in
  [-pi, pi]; unions 1-3 mix Union/Subtraction and carry their own transforms.
  AABB culling is on for 24 of the 28 shapes.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np

from .sdf_editor import SDFEditor, Shape, Shapes, Union, UnionType


def _mat(shape: Shape, col=(1, 1, 1), brightness=0.0, light=(1, 1, 1), spec=0.0, spec_col=(1, 1, 1), rough=0.0):
    m = shape.material
    m.color.set(col)
    m.brightness.set(brightness)
    m.light_col.set(light)
    m.specular_chance.set(spec)
    m.specular_color.set(spec_col)
    m.roughness.set(rough)


def _shape(kind: str, pos=(0, 0, 0), rot=(0, 0, 0), scale=1.0, size: Sequence[float] = (1.0,), aabb=True, name="Shape",
           ex=1.3) -> Shape:
    s = Shape(kind)
    s.name = name
    s.transform.position.set(pos)
    s.transform.rotation.set(rot)
    s.transform.scale.set(scale)
    s.transform.aabb = aabb
    s.transform.aabb_exaggeration.set(ex)
    for p, v in zip(s.current_shape.params, size):
        p.set(v)
    return s


def _union(name: str, union_type=UnionType.UNION, pos=(0, 0, 0), rot=(0, 0, 0), scale=1.0) -> Union:
    u = Union(union_type)
    u.name = name
    u.transform.position.set(pos)
    u.transform.rotation.set(rot)
    u.transform.scale.set(scale)
    return u


def empty() -> SDFEditor:
    """PLACEHOLDER_MAP (state.rs:20-36): no unions; every pixel misses."""
    return SDFEditor([])


def c1_default() -> SDFEditor:
    ed = SDFEditor()  # Union + Sphere(1.0), defaults everywhere
    _mat(ed.header_unions[0].children_shapes[0], brightness=1.0)
    return ed


def c2_sphere_box_torus() -> SDFEditor:
    torus_rot = (1.2, 0.3, 0.0)

    def torus():
        t = _shape(Shapes.TORUS, pos=(0.0, 0.0, 0.2), rot=torus_rot, size=(1.05, 0.32), name="torus")
        _mat(t, col=(0.15, 0.35, 0.95), spec=0.2, rough=0.4)
        return t

    a = _union("sphere-torus", UnionType.SUBTRACTION)
    a.children_shapes.append(torus())
    sph = _shape(Shapes.SPHERE, pos=(-0.75, 0.0, 0.3), size=(0.95,), name="sphere")
    _mat(sph, col=(0.9, 0.25, 0.2))
    a.children_shapes.append(sph)

    b = _union("box-torus", UnionType.SUBTRACTION)
    b.children_shapes.append(torus())
    box = _shape(Shapes.CUBE, pos=(0.8, -0.1, 0.2), rot=(0.3, 0.6, 0.1), size=(0.7, 0.7, 0.7), name="box")
    _mat(box, col=(0.85, 0.85, 0.8), spec=0.5, spec_col=(1.0, 0.9, 0.7), rough=0.25)
    b.children_shapes.append(box)

    light = _union("light")
    ls = _shape(Shapes.SPHERE, pos=(0.0, 3.2, -0.5), size=(1.2,), name="light")
    _mat(ls, col=(1, 1, 1), brightness=4.0)
    light.children_shapes.append(ls)
    floor = _shape(Shapes.CUBE, pos=(0.0, -2.0, 1.0), size=(6.0, 0.5, 6.0), name="floor")
    _mat(floor, col=(0.6, 0.6, 0.6), spec=0.1, rough=0.6)
    light.children_shapes.append(floor)
    return SDFEditor([a, b, light])


# assets/maps/test.json (deprecated node-editor save of the reference)
_ROOM = [
    ("floor", (11.63, 1.0, 12.26), (0.0, -2.32, 0.0), (0.0, 0.0, 0.0),
     dict(col=(0.0, 0.6313726, 1.0), spec=0.75, spec_col=(0.50980395, 0.53333336, 1.0), rough=0.2)),
    ("roof", (11.63, 1.0, 12.26), (0.0, 3.25, 0.0), (0.0, 0.0, 0.0),
     dict(col=(0.0, 0.2509804, 1.0), spec=0.0, spec_col=(0.0, 0.0, 0.0), rough=0.0)),
    ("light", (1.0, 1.0, 2.0), (0.0, 3.23, 1.85), (0.0, 0.0, 0.0),
     dict(col=(0.0, 0.0, 0.0), brightness=1.2, light=(1.0, 1.0, 1.0), spec=0.0, spec_col=(0.0, 0.0, 0.0))),
    ("4", (11.63, 1.0, 12.26), (0.0, 3.25, 3.75), (1.4, 0.0, 0.0),
     dict(col=(1.0, 0.0, 0.0), spec=0.0, spec_col=(0.0, 0.0, 0.0))),
    ("7", (1.0, 1.15, 7.2), (3.0, 0.0, 2.1), (0.0, -0.22, 0.0),
     dict(col=(0.0, 0.0, 0.0), spec=0.5, spec_col=(1.0, 1.0, 1.0))),
    ("8", (1.0, 1.15, 7.2), (-3.0, 0.0, 2.1), (0.0, 0.22, 0.0),
     dict(col=(0.0, 0.0, 0.0), spec=0.5, spec_col=(1.0, 1.0, 1.0))),
]
_OCTA = [
    ("5", 1.0, (0.0, -0.06, 1.8), (1.61, 2.82, 1.87)),
    ("6", 1.0, (-0.05, -0.2, 1.8), (1.7, 1.8, 2.68)),
]


def c3_graph32(seed: int = 42) -> SDFEditor:
    rng = np.random.default_rng(seed)
    room = _union("room")
    for name, size, pos, rot, mat in _ROOM:
        s = _shape(Shapes.CUBE, pos=pos, rot=rot, size=size, name=name, aabb=name not in ("floor", "roof"))
        _mat(s, **mat)
        room.children_shapes.append(s)
    # 7th room piece: a small emissive panel on the left wall
    panel = _shape(Shapes.CUBE, pos=(-1.9, 1.2, 3.0), rot=(0.0, 0.22, 0.0), size=(0.05, 0.4, 0.8), name="panel")
    _mat(panel, col=(1, 1, 1), brightness=2.5, light=(1.0, 0.85, 0.6))
    room.children_shapes.append(panel)

    specs = [
        ("objects-a", UnionType.UNION, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), 1.0),
        ("objects-b", UnionType.SUBTRACTION, (0.6, 0.4, 0.8), (0.0, 0.5, 0.0), 0.9),
        ("objects-c", UnionType.UNION, (-0.4, -0.3, 0.5), (0.2, -0.3, 0.1), 1.1),
    ]
    unions = [room]
    for ui, (name, ut, upos, urot, usc) in enumerate(specs):
        u = _union(name, ut, pos=upos, rot=urot, scale=usc)
        first = 0
        if ui == 0:
            for oname, sz, opos, orot in _OCTA:
                o = _shape(Shapes.OCTAHEDRON, pos=opos, rot=orot, size=(sz * 0.6,), name=oname)
                _mat(o, col=(0.0, 0.0, 0.0), spec=1.0, spec_col=(1.0, 1.0, 1.0), rough=0.555)
                u.children_shapes.append(o)
            first = 2
        for k in range(first, 7):
            kind = Shapes.SPHERE if rng.random() < 0.5 else Shapes.CUBE
            pos = (rng.uniform(-2.4, 2.4), rng.uniform(-1.2, 1.8), rng.uniform(-0.5, 4.0))
            rot = tuple(rng.uniform(-math.pi, math.pi, 3))
            if kind == Shapes.SPHERE:
                size = (rng.uniform(0.2, 0.75),)
            else:
                size = tuple(rng.uniform(0.2, 0.75, 3))
            # subtraction unions cut with their later members: keep those small
            if ut == UnionType.SUBTRACTION and k > 0:
                size = tuple(0.6 * v for v in size)
            aabb = not (ui == 2 and k in (5, 6))
            s = _shape(kind, pos=pos, rot=rot, size=size, aabb=aabb, name=f"{name}-{k}")
            col = tuple(rng.uniform(0.1, 0.95, 3))
            emissive = rng.random() < 0.12
            spec = float(rng.choice([0.0, 0.0, 0.3, 0.8]))
            _mat(s, col=col, brightness=3.0 if emissive else 0.0, spec=spec,
                 spec_col=tuple(rng.uniform(0.6, 1.0, 3)), rough=float(rng.uniform(0.0, 0.6)))
            u.children_shapes.append(s)
        unions.append(u)
    return SDFEditor(unions)


def nested_demo() -> SDFEditor:
    """Nested unions: exercises the compiler quirks of SURVEY.md A.9 (i)-(ii)
    (child-union results discarded by the index-0 assignment; map/bounds
    check[] index mismatch)."""
    outer = _union("outer", UnionType.UNION, pos=(0.1, 0.0, 0.3), rot=(0.0, 0.3, 0.0), scale=0.9)
    inner = _union("inner", UnionType.SUBTRACTION, pos=(0.3, 0.2, 0.0), scale=1.2)
    a = _shape(Shapes.CUBE, pos=(0.0, 0.0, 0.0), size=(0.6, 0.6, 0.6), rot=(0.4, 0.1, 0.2))
    _mat(a, col=(0.8, 0.3, 0.3))
    b = _shape(Shapes.SPHERE, pos=(0.2, 0.2, -0.2), size=(0.5,))
    _mat(b, col=(0.3, 0.8, 0.3))
    inner.children_shapes += [a, b]
    deeper = _union("deeper", UnionType.UNION, pos=(-0.5, 0.0, 0.0))
    c = _shape(Shapes.OCTAHEDRON, pos=(0.0, 0.5, 0.0), size=(0.5,), rot=(0.3, 0.2, 0.1))
    _mat(c, col=(0.3, 0.3, 0.9), spec=0.6, rough=0.2)
    deeper.children_shapes.append(c)
    inner.children_unions.append(deeper)
    outer.children_unions.append(inner)
    # emitters with aabb off: under quirk (ii) an aabb-guarded shape of a nested
    # graph reads a check[] entry bounds() never sets, and would stay dark
    d = _shape(Shapes.SPHERE, pos=(-0.9, -0.2, 0.4), size=(0.45,), aabb=False)
    _mat(d, col=(0.9, 0.9, 0.2), brightness=2.0)
    e = _shape(Shapes.CUBE, pos=(0.9, -0.4, 0.0), size=(0.3, 0.5, 0.3), aabb=False)
    _mat(e, col=(0.5, 0.5, 0.5), spec=0.4)
    outer.children_shapes += [d, e]
    top2 = _union("lamp")
    l = _shape(Shapes.SPHERE, pos=(0.0, 2.5, 0.0), size=(0.8,), aabb=False)
    _mat(l, brightness=3.0)
    top2.children_shapes.append(l)
    return SDFEditor([outer, top2])


def wide_graph(seed: int = 7, unions: int = 12, per_union: int = 8) -> SDFEditor:
    """c3's room plus `unions` x `per_union` small random shapes, all with
    AABBs: more than 64 check[] entries (exercises the high mask words)."""
    rng = np.random.default_rng(seed)
    ed = c3_graph32()
    for ui in range(unions):
        u = _union(f"cloud-{ui}", pos=(rng.uniform(-0.5, 0.5), rng.uniform(-0.3, 0.3), rng.uniform(0.0, 1.0)))
        for k in range(per_union):
            kind = Shapes.SPHERE if rng.random() < 0.6 else Shapes.CUBE
            size = (rng.uniform(0.05, 0.2),) if kind == Shapes.SPHERE else tuple(rng.uniform(0.05, 0.2, 3))
            s = _shape(kind, pos=(rng.uniform(-2.2, 2.2), rng.uniform(-1.0, 1.6), rng.uniform(0.0, 4.0)),
                       rot=tuple(rng.uniform(-1.0, 1.0, 3)), size=size, name=f"cloud-{ui}-{k}")
            _mat(s, col=tuple(rng.uniform(0.2, 0.9, 3)), brightness=2.0 if rng.random() < 0.1 else 0.0,
                 spec=float(rng.choice([0.0, 0.5])), rough=0.3)
            u.children_shapes.append(s)
        ed.header_unions.append(u)
    return ed


def cull_stress(seed: int = 11) -> SDFEditor:
    """c3's room plus clustered unions of every shape kind under scaled and
    rotated union/shape transforms: the distance-bound culling of the scene
    kernels drops shapes near its threshold.  Three unions
    carry values that switch the rule off (a negative cube size, a 1e-7 shape
    scale) or keep it on with a negative sphere radius."""
    rng = np.random.default_rng(seed)
    ed = c3_graph32()
    kinds = (Shapes.SPHERE, Shapes.CUBE, Shapes.TORUS, Shapes.OCTAHEDRON)
    for ui in range(6):
        u = _union(f"cluster-{ui}", pos=(rng.uniform(-1.2, 1.2), rng.uniform(-0.6, 0.9), rng.uniform(0.5, 3.0)),
                   rot=tuple(rng.uniform(-0.8, 0.8, 3)), scale=float(rng.uniform(0.6, 1.4)))
        for k in range(6):
            kind = kinds[(ui + k) % 4]
            if kind == Shapes.CUBE:
                size = tuple(rng.uniform(0.05, 0.3, 3))
            elif kind == Shapes.TORUS:
                size = (float(rng.uniform(0.1, 0.3)), float(rng.uniform(0.02, 0.1)))
            else:
                size = (float(rng.uniform(0.05, 0.3)),)
            sc = float(rng.uniform(0.5, 1.6))
            if ui == 3 and k == 2:
                size = (0.2, -0.1, 0.2)  # degenerate cube: no bound, the union's rule is off
                kind = Shapes.CUBE
            if ui == 4 and k == 4:
                sc = 1e-7  # 1/s beyond the bound's range: no bound, the union's rule is off
            if ui == 5 and k == 1:
                kind, size = Shapes.SPHERE, (-0.15,)  # negative radius: still bounded (R = r)
            s = _shape(kind, pos=tuple(rng.uniform(-0.5, 0.5, 3)), rot=tuple(rng.uniform(-math.pi, math.pi, 3)),
                       scale=sc, size=size, aabb=bool(rng.random() < 0.7), name=f"cluster-{ui}-{k}")
            _mat(s, col=tuple(rng.uniform(0.2, 0.9, 3)), brightness=2.0 if rng.random() < 0.15 else 0.0,
                 spec=float(rng.choice([0.0, 0.5])), rough=0.3)
            u.children_shapes.append(s)
        ed.header_unions.append(u)
    return ed


def tiny_union() -> SDFEditor:
    """Open space towards a distant backdrop, with two specks behind the
    camera: header unions of scale 1e-3 and 2e-3 whose shapes are ~1 unit in
    their own frame.  A union returns MAXHIT * s (= 10,
    20 world units) when none of its shapes combines, so rays through open
    space (parent distance > 10) check that the scene kernels' distance-bound
    culling of a union's first (assign) shape keeps the reference's value
    (containers.rs:244-252: u = shape overwrites MAXHIT)."""
    a = _union("anchor")
    lamp = _shape(Shapes.SPHERE, pos=(0.0, -0.2, 2.0), size=(0.6,), name="lamp")
    _mat(lamp, col=(0.9, 0.8, 0.7), brightness=2.0)
    box = _shape(Shapes.CUBE, pos=(1.2, 0.4, 3.0), rot=(0.3, 0.5, 0.0), size=(0.3, 0.3, 0.3), name="box")
    _mat(box, col=(0.3, 0.6, 0.9), spec=0.5, rough=0.2)
    wall = _shape(Shapes.CUBE, pos=(0.0, 0.0, 40.0), size=(80.0, 80.0, 1.0), aabb=False, name="backdrop")
    _mat(wall, col=(0.7, 0.7, 0.7), brightness=0.5)
    a.children_shapes += [lamp, box, wall]
    # behind the camera: farther than the running distance while rays cross
    # the open space towards the backdrop, so their shapes are dropped
    sp = _union("speck-a", pos=(0.4, 0.3, -20.0), rot=(0.2, 0.1, 0.4), scale=1e-3)
    for k, (kind, pos, size, aabb) in enumerate([(Shapes.SPHERE, (0, 0, 0), (1.0,), False),
                                                 (Shapes.CUBE, (1.5, 0, 0), (0.8, 0.8, 0.8), False),
                                                 (Shapes.SPHERE, (0, 1.5, 0), (0.5,), True)]):
        s = _shape(kind, pos=pos, size=size, aabb=aabb, name=f"speck-a-{k}")
        _mat(s, col=(0.8, 0.2, 0.2), brightness=5.0)
        sp.children_shapes.append(s)
    sb = _union("speck-b", pos=(-0.5, 0.2, -25.0), scale=2e-3)
    s = _shape(Shapes.CUBE, size=(1.0, 1.0, 1.0), aabb=False, name="speck-b-0")
    _mat(s, col=(0.2, 0.8, 0.2))
    sb.children_shapes.append(s)
    return SDFEditor([a, sp, sb])


def far_box() -> SDFEditor:
    """c2 plus a sphere 1e20 units away with its AABB on: one box coordinate
    outside the reciprocal-division guard, so every ray of
    the scene takes bounds()'s IEEE-division path (scene kernels: the baked
    'false' branch and the table kernel's fast_bounds = 0)."""
    ed = c2_sphere_box_torus()
    u = _union("far")
    s = _shape(Shapes.SPHERE, pos=(1e20, 0.0, 0.0), size=(1.0,), name="far")
    _mat(s, col=(0.5, 0.5, 0.5))
    u.children_shapes.append(s)
    ed.header_unions.append(u)
    return ed


_DEPRECATED_KINDS = {"Sphere": Shapes.SPHERE, "Cube": Shapes.CUBE, "OctahedronExact": Shapes.OCTAHEDRON}


def deprecated_map(nodes) -> SDFEditor:
    """A map saved by the reference's deprecated node editor
    (assets/maps/*.json: a list of serde `Node`s,
    assets/depricated/node_editor_package.rs:204-218 + its `Material`) as
    a current editor scene.  One header union holds the nodes in file order.
    Each node keeps its shape (OctahedronExact -> Octahedron), scale, size,
    position and rotation.  Material fields are copied one for one
    (light_strength -> Brightness).  A light colour of (0, 0, 0) becomes
    the live editor's default (1, 1, 1): the current Mat normalises the
    light colour, and zero would make every hit NaN.  AABB culling is on,
    with the editor's default exaggeration.  `nodes`: the parsed JSON list,
    or a path to the file."""
    if isinstance(nodes, str):
        import json

        with open(nodes) as f:
            nodes = json.load(f)
    u = _union("map")
    for n in nodes:
        kind = _DEPRECATED_KINDS[n["shape"]]
        m = n["material"]
        light = tuple(m["light"])
        s = _shape(kind, pos=tuple(n["position"]), rot=tuple(n["rotation"]), scale=n["scale"],
                   size=tuple(n["size"]), name=n["title"])
        _mat(s, col=tuple(m["color"]), brightness=m["light_strength"],
             light=light if any(v != 0.0 for v in light) else (1.0, 1.0, 1.0), spec=m["spec"],
             spec_col=tuple(m["spec_col"]), rough=m["roughness"])
        mat = s.material
        mat.ior.set(m["ior"])
        mat.refract_chance.set(m["refraction_chance"])
        mat.refract_roughness.set(m["refraction_roughness"])
        mat.refract_color.set(tuple(m["refraction_color"]))
        u.children_shapes.append(s)
    return SDFEditor([u])


def c3_no_aabb() -> SDFEditor:
    """c3 with every Transform.aabb off (profiling aid: no per-lane culling)."""
    ed = c3_graph32()
    for u in ed.header_unions:
        for sh in u.children_shapes:
            sh.transform.aabb = False
    return ed


SCENES = {
    "empty": empty,
    "c1": c1_default,
    "c2": c2_sphere_box_torus,
    "c3": c3_graph32,
    "nested": nested_demo,
    "c3_noaabb": c3_no_aabb,
    "wide": wide_graph,
    "cull": cull_stress,
    "tiny": tiny_union,
    "farbox": far_box,
}

# BASELINE.json configs -> (scene, width, height, spp, bounces)
CONFIGS = {
    "c1": ("c1", 256, 256, 1, 1),
    "c2": ("c2", 1920, 1080, 64, 4),
    "c3": ("c3", 1920, 1080, 256, 8),
    "c4": ("c3", 3840, 2160, 256, 8),
    "c5": ("c3", 1920, 1080, 1024, 16),
}
