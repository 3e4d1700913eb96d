"""Host mirror of the reference's SDF editor node graph and its compiler.

Mirrors ``src/sdf_editor`` of zachdedoo13/compute_path_tracer (snapshot
2024-10-08): the same node types (``Union``, ``Shape``, ``Transform``,
``Material``, ``Float``, ``V3``), the same defaults, the same serde JSON
layout for save/load (``sdf_editor.rs:131-167``) and the same compile/update
split (``RecUpdate``, ``primitives.rs:160-190``).  What changes is the compile
target: instead of GLSL text spliced into the compute shader
(``SDFEditor::compile``, ``sdf_editor.rs:186-246``) the tree is compiled by the
native ``pt_compile_scene`` into an op list + ``data[]`` with the reference's
exact slot numbering, which :class:`compute_path_tracer_amd.path_tracer.PathTracer`
uploads through the C ABI.  The egui UI code is out of scope.
"""
from __future__ import annotations

import ctypes
import json
import secrets
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _native as N

F32_MAX = float(np.finfo(np.float32).max)

# speeds, primitives.rs:193-196
S1 = 0.001
S2 = 0.01
S3 = 0.1


def gen_hash() -> int:
    """primitives.rs:12-17: a random u128 identifying a Float's data[] slot."""
    return secrets.randbits(128) ^ secrets.randbits(128)


class Float:
    """primitives.rs:203-267."""

    def __init__(self, name: str, speed: float, val: float, rng: Tuple[float, float] = (-F32_MAX, F32_MAX),
                 hash_: Optional[int] = None):
        self.val = float(np.float32(val))
        self.range = (float(rng[0]), float(rng[1]))
        self.speed = float(speed)
        self.name = name
        self.hash = gen_hash() if hash_ is None else int(hash_)

    @classmethod
    def new(cls, name, speed, val, rng):
        return cls(name, speed, val, rng)

    @classmethod
    def inv(cls, name, speed, val):
        return cls(name, speed, val, (-F32_MAX, F32_MAX))

    @classmethod
    def percent(cls, name, speed, val):
        return cls(name, speed, val, (0.0, 1.0))

    def set(self, v: float) -> None:
        lo, hi = self.range
        self.val = float(np.float32(min(max(v, lo), hi)))

    def compile(self, comp_data: "CompData") -> int:
        return comp_data.data_array.get_index(self.val, self.hash)

    def refresh(self, comp_data: "CompData") -> None:
        comp_data.data_array.refresh(self.hash, self.val)

    def rehash(self) -> None:
        self.hash = gen_hash()

    def to_json(self):
        return {"val": self.val, "range": {"start": self.range[0], "end": self.range[1]}, "speed": self.speed,
                "name": self.name, "hash": self.hash}

    @classmethod
    def from_json(cls, d):
        r = d.get("range", {"start": -F32_MAX, "end": F32_MAX})
        return cls(d["name"], d["speed"], d["val"], (r["start"], r["end"]), d["hash"])

    def floats(self):
        yield self


class V3:
    """primitives.rs:269-331."""

    def __init__(self, x: Float, y: Float, z: Float, name: str):
        self.x, self.y, self.z, self.name = x, y, z, name

    @classmethod
    def xyz(cls, name, speed, val):
        return cls(Float.inv("X", speed, val), Float.inv("Y", speed, val), Float.inv("Z", speed, val), name)

    @classmethod
    def rgb(cls, name):
        return cls(Float.inv("R", 1.0, 1.0), Float.inv("G", 1.0, 1.0), Float.inv("B", 1.0, 1.0), name)

    def vals(self) -> List[float]:
        return [self.x.val, self.y.val, self.z.val]

    def set(self, v) -> None:
        self.x.set(v[0]); self.y.set(v[1]); self.z.set(v[2])

    def floats(self):
        yield self.x
        yield self.y
        yield self.z

    def rehash(self):
        for f in self.floats():
            f.rehash()

    def to_json(self):
        return {"x": self.x.to_json(), "y": self.y.to_json(), "z": self.z.to_json(), "name": self.name}

    @classmethod
    def from_json(cls, d):
        return cls(Float.from_json(d["x"]), Float.from_json(d["y"]), Float.from_json(d["z"]), d["name"])


class Transform:
    """data_structures.rs:10-111."""

    def __init__(self):
        self.position = V3.xyz("Position", S2, 0.0)
        self.rotation = V3.xyz("Rotation", S1, 0.0)
        self.scale = Float.new("Scale", S1, 1.0, (0.0, F32_MAX))
        self.aabb_exaggeration = Float.new("AABB_exaggeration", S2, 1.3, (0.0, 10.0))
        self.aabb = True

    def floats(self):
        # Transform::compile order: scale, position, rotation, aabb_exaggeration
        yield self.scale
        yield from self.position.floats()
        yield from self.rotation.floats()
        yield self.aabb_exaggeration

    def rehash(self):
        for f in self.floats():
            f.rehash()

    def refresh(self, comp_data):
        """data_structures.rs:98-103 (position, rotation, scale, exaggeration:
        with shared hashes the last write wins, so the order matters)."""
        for f in (*self.position.floats(), *self.rotation.floats(), self.scale, self.aabb_exaggeration):
            f.refresh(comp_data)

    def to_json(self):
        return {"position": self.position.to_json(), "rotation": self.rotation.to_json(),
                "scale": self.scale.to_json(), "aabb_exaggeration": self.aabb_exaggeration.to_json(),
                "aabb": self.aabb}

    @classmethod
    def from_json(cls, d):
        t = cls()
        t.position = V3.from_json(d["position"])
        t.rotation = V3.from_json(d["rotation"])
        t.scale = Float.from_json(d["scale"])
        t.aabb_exaggeration = Float.from_json(d["aabb_exaggeration"])
        t.aabb = bool(d["aabb"])
        return t


MATERIAL_FIELDS = ("color", "brightness", "light_col", "specular_chance", "specular_color", "roughness", "ior",
                   "refract_chance", "refract_roughness", "refract_color")


class Material:
    """data_structures.rs:115-221 (Mat order of test_compute.glsl:45-59)."""

    def __init__(self):
        self.color = V3.rgb("Surface Color")
        self.brightness = Float.new("Brightness", S2, 0.0, (0.0, F32_MAX))
        self.light_col = V3.rgb("Light Color")
        self.specular_chance = Float.percent("Spec chance", S1, 0.0)
        self.specular_color = V3.rgb("Spec color")
        self.roughness = Float.new("Roughness", S1, 0.0, (0.0, F32_MAX))
        self.ior = Float.inv("IOR", S1, 0.0)
        self.refract_chance = Float.percent("Refract chance", S1, 0.0)
        self.refract_roughness = Float.inv("Refract roughness", S1, 0.0)
        self.refract_color = V3.rgb("Refract color")

    def floats(self):
        for name in MATERIAL_FIELDS:
            yield from getattr(self, name).floats()

    def values(self) -> List[float]:
        return [f.val for f in self.floats()]

    def rehash(self):
        for f in self.floats():
            f.rehash()

    def to_json(self):
        return {name: getattr(self, name).to_json() for name in MATERIAL_FIELDS}

    @classmethod
    def from_json(cls, d):
        m = cls()
        for name in MATERIAL_FIELDS:
            v = d[name]
            setattr(m, name, V3.from_json(v) if "x" in v else Float.from_json(v))
        return m


class Shapes:
    """containers.rs:259-319 (Sphere, Cube, Plane) + Torus/Octahedron extensions."""

    SPHERE, CUBE, PLANE, TORUS, OCTAHEDRON = "Sphere", "Cube", "Plane", "Torus", "Octahedron"
    KIND = {SPHERE: N.PT_NODE_SPHERE, CUBE: N.PT_NODE_CUBE, PLANE: N.PT_NODE_PLANE, TORUS: N.PT_NODE_TORUS,
            OCTAHEDRON: N.PT_NODE_OCTAHEDRON}

    def __init__(self, kind: str = SPHERE, params: Optional[List[Float]] = None):
        self.kind = kind
        if params is None:
            if kind == self.SPHERE:
                params = [Float.inv("Size", S2, 1.0)]
            elif kind == self.CUBE:
                params = list(V3.xyz("Size", S2, 1.0).floats())
            elif kind == self.TORUS:
                params = [Float.inv("Major radius", S2, 1.0), Float.inv("Minor radius", S2, 0.25)]
            elif kind == self.OCTAHEDRON:
                params = [Float.inv("Size", S2, 1.0)]
            else:
                params = []
        self.params = params

    def floats(self):
        yield from self.params

    def rehash(self):
        for f in self.params:
            f.rehash()

    def to_json(self):
        if self.kind == self.PLANE:
            return "Plane"
        if self.kind == self.CUBE:
            x, y, z = self.params
            return {"Cube": {"x": x.to_json(), "y": y.to_json(), "z": z.to_json(), "name": "Size"}}
        if self.kind == self.TORUS:
            return {"Torus": [p.to_json() for p in self.params]}
        return {self.kind: self.params[0].to_json()}

    @classmethod
    def from_json(cls, d):
        if d == "Plane":
            return cls(cls.PLANE, [])
        (kind, v), = d.items()
        if kind == cls.CUBE:
            return cls(kind, list(V3.from_json(v).floats()))
        if kind == cls.TORUS:
            return cls(kind, [Float.from_json(p) for p in v])
        return cls(kind, [Float.from_json(v)])


class Shape:
    """containers.rs:322-476."""

    def __init__(self, kind: str = Shapes.SPHERE):
        self.transform = Transform()
        self.material = Material()
        self.current_shape = Shapes(kind)
        self.name = "Shape"

    def floats(self):
        # Shape::compile order: transform, shape settings, material
        yield from self.transform.floats()
        yield from self.current_shape.floats()
        yield from self.material.floats()

    def rehash(self):
        self.transform.rehash(); self.material.rehash(); self.current_shape.rehash()

    def refresh(self, comp_data):
        """containers.rs:466-470: transform, material, then the shape's size."""
        self.transform.refresh(comp_data)
        for f in (*self.material.floats(), *self.current_shape.floats()):
            f.refresh(comp_data)

    def to_json(self):
        return {"transform": self.transform.to_json(), "material": self.material.to_json(),
                "current_shape": self.current_shape.to_json(), "name": self.name}

    @classmethod
    def from_json(cls, d):
        s = cls()
        s.transform = Transform.from_json(d["transform"])
        s.material = Material.from_json(d["material"])
        s.current_shape = Shapes.from_json(d["current_shape"])
        s.name = d["name"]
        return s


class UnionType:
    UNION = "Union"
    SUBTRACTION = "Subtraction"


class Union:
    """containers.rs:8-203."""

    def __init__(self, union_type: str = UnionType.UNION):
        self.name = "Union"
        self.transform = Transform()
        self.union_type = union_type
        self.children_unions: List[Union] = []
        self.children_shapes: List[Shape] = []

    def refresh(self, comp_data):
        """containers.rs:204-212: transform, shapes, then child unions."""
        self.transform.refresh(comp_data)
        for s in self.children_shapes:
            s.refresh(comp_data)
        for u in self.children_unions:
            u.refresh(comp_data)

    def to_json(self):
        return {"name": self.name, "transform": self.transform.to_json(), "union_type": self.union_type,
                "children_unions": [u.to_json() for u in self.children_unions],
                "children_shapes": [s.to_json() for s in self.children_shapes]}

    @classmethod
    def from_json(cls, d):
        u = cls(d["union_type"])
        u.name = d["name"]
        u.transform = Transform.from_json(d["transform"])
        u.children_unions = [Union.from_json(c) for c in d["children_unions"]]
        u.children_shapes = [Shape.from_json(c) for c in d["children_shapes"]]
        return u


class DataArray:
    """primitives.rs:59-157 without the wgpu buffer (the C ABI owns the device copy)."""

    def __init__(self):
        self.data: List[float] = [6969.69]
        self.seen: Dict[int, int] = {}

    def get_index(self, val: float, hash_: int) -> int:
        if hash_ in self.seen:
            return self.seen[hash_]
        self.data.append(float(np.float32(val)))
        self.seen[hash_] = len(self.data) - 1
        return self.seen[hash_]

    def refresh(self, hash_: int, val: float) -> None:
        if hash_ not in self.seen:
            raise KeyError("Float hash not compiled (primitives.rs:154 panics here)")
        self.data[self.seen[hash_]] = float(np.float32(val))

    def as_array(self) -> np.ndarray:
        return np.asarray(self.data, dtype=np.float32)


class RecUpdate:
    """primitives.rs:160-190."""

    def __init__(self, compile_: bool = True, update: bool = True):
        self.queue_compile = compile_
        self.queue_update = update

    def reset(self):
        self.queue_compile = self.queue_update = False

    def update(self):
        self.queue_update = True

    def compile(self):
        self.queue_compile = True

    def both(self):
        self.queue_compile = self.queue_update = True


class CompData:
    """primitives.rs:21-57."""

    def __init__(self):
        self.data_array = DataArray()
        self.rec_update = RecUpdate(True, True)
        self.aabb_index = 0

    def reset_data_array(self):
        self.data_array.data = [6969.69]
        self.data_array.seen.clear()


@dataclass
class Program:
    """What SDFEditor::compile now produces: the map()/bounds() program."""

    ops: ctypes.Array
    aabbs: ctypes.Array
    n_ops: int
    n_aabb: int
    n_check: int
    data: np.ndarray = field(default_factory=lambda: np.zeros(1, np.float32))

    def op_dicts(self) -> List[dict]:
        out = []
        for i in range(self.n_ops):
            o = self.ops[i]
            out.append({"opcode": o.opcode, "shape": o.shape, "combine": o.combine, "check": o.check,
                        "scale": o.scale, "position": list(o.position), "rotation": list(o.rotation),
                        "aabb_exaggeration": o.aabb_exaggeration, "size": list(o.size),
                        "material": list(o.material)})
        return out

    def aabb_dicts(self) -> List[dict]:
        out = []
        for i in range(self.n_aabb):
            a = self.aabbs[i]
            out.append({"back": a.back, "so_kind": a.so_kind, "union_position": list(a.union_position),
                        "union_scale": a.union_scale, "shape_position": list(a.shape_position),
                        "shape_scale": a.shape_scale, "size": list(a.size),
                        "aabb_exaggeration": a.aabb_exaggeration})
        return out


def node_keys(t: Transform, size: List[Float], material: Optional[Material]) -> List[int]:
    """The node's Float hashes in pt_float_key order (PT_NODE_FLOATS): scale,
    position xyz, rotation xyz, exaggeration, size[3], material[18]; 0 where
    the node has no such Float."""
    keys = [f.hash for f in t.floats()]
    keys += [f.hash for f in size] + [0] * (3 - len(size))
    keys += [f.hash for f in material.floats()] if material is not None else [0] * 18
    return keys


def keys_to_ctypes(rows: List[dict]):
    """Rows' "keys" as a pt_float_key array (None when no row carries keys)."""
    if not any(r.get("keys") for r in rows):
        return None
    arr = (N.FloatKey * (max(1, len(rows)) * N.PT_NODE_FLOATS))()
    for i, r in enumerate(rows):
        for k, h in enumerate(r.get("keys") or []):
            arr[i * N.PT_NODE_FLOATS + k].lo = h & 0xFFFFFFFFFFFFFFFF
            arr[i * N.PT_NODE_FLOATS + k].hi = (h >> 64) & 0xFFFFFFFFFFFFFFFF
    return arr


def flatten(header_unions: List[Union]) -> Tuple[List[dict], List[object]]:
    """Pre-order flattening: each node's parent precedes it; a union's child
    unions precede its shapes (the order Union::compile visits them)."""
    rows: List[dict] = []
    objs: List[object] = []

    def visit(u: Union, parent: int):
        idx = len(rows)
        t = u.transform
        rows.append({"kind": N.PT_NODE_UNION, "parent": parent,
                     "union_type": N.PT_UNION_TYPE_SUBTRACTION if u.union_type == UnionType.SUBTRACTION
                     else N.PT_UNION_TYPE_UNION, "aabb": int(t.aabb), "scale": t.scale.val,
                     "position": t.position.vals(), "rotation": t.rotation.vals(),
                     "aabb_exaggeration": t.aabb_exaggeration.val, "size": [0.0, 0.0, 0.0],
                     "material": [0.0] * 18, "keys": node_keys(t, [], None)})
        objs.append(u)
        for c in u.children_unions:
            visit(c, idx)
        for s in u.children_shapes:
            st = s.transform
            sz = [p.val for p in s.current_shape.params] + [0.0] * (3 - len(s.current_shape.params))
            rows.append({"kind": Shapes.KIND[s.current_shape.kind], "parent": idx, "union_type": 0,
                         "aabb": int(st.aabb), "scale": st.scale.val, "position": st.position.vals(),
                         "rotation": st.rotation.vals(), "aabb_exaggeration": st.aabb_exaggeration.val,
                         "size": sz, "material": s.material.values(),
                         "keys": node_keys(st, s.current_shape.params, s.material)})
            objs.append(s)

    for u in header_unions:
        visit(u, -1)
    return rows, objs


def nodes_to_ctypes(rows: List[dict]) -> ctypes.Array:
    arr = (N.SceneNode * max(1, len(rows)))()
    for i, r in enumerate(rows):
        n = arr[i]
        n.kind, n.parent, n.union_type, n.aabb = r["kind"], r["parent"], r["union_type"], r["aabb"]
        n.scale = r["scale"]
        n.aabb_exaggeration = r["aabb_exaggeration"]
        for k in range(3):
            n.position[k] = r["position"][k]
            n.rotation[k] = r["rotation"][k]
            n.size[k] = r["size"][k]
        for k in range(18):
            n.material[k] = r["material"][k]
    return arr


def compile_rows(rows: List[dict]) -> Program:
    """Native pt_compile_scene_keyed on flattened rows (two-call pattern):
    Floats sharing a hash share a data[] slot (DataArray::get_index)."""
    L = N.lib()
    nodes = nodes_to_ctypes(rows)
    keys = keys_to_ctypes(rows)
    n_ops, n_aabb, n_data, n_check = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    rc = L.pt_compile_scene_keyed(nodes, len(rows), keys, None, 0, ctypes.byref(n_ops), None, 0, ctypes.byref(n_aabb),
                                  None, 0, ctypes.byref(n_data), ctypes.byref(n_check))
    N.check("pt_compile_scene_keyed", rc)
    ops = (N.Op * max(1, n_ops.value))()
    aabbs = (N.Aabb * max(1, n_aabb.value))()
    data = np.zeros(n_data.value, dtype=np.float32)
    rc = L.pt_compile_scene_keyed(nodes, len(rows), keys, ops, n_ops.value, ctypes.byref(n_ops), aabbs, n_aabb.value,
                                  ctypes.byref(n_aabb), data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                  n_data.value, ctypes.byref(n_data), ctypes.byref(n_check))
    N.check("pt_compile_scene_keyed", rc)
    return Program(ops, aabbs, n_ops.value, n_aabb.value, n_check.value, data)


class SDFEditor:
    """sdf_editor.rs:13-253: the tree, its JSON save/load and its compiler."""

    def __init__(self, header_unions: Optional[List[Union]] = None):
        if header_unions is None:  # SDFEditor::new, sdf_editor.rs:20-33
            header_unions = [Union()]
            header_unions[0].children_shapes.append(Shape())
        self.header_unions = header_unions
        self.save_name = ""

    # -- compiler ---------------------------------------------------------
    def compile(self, comp_data: CompData) -> Program:
        """SDFEditor::compile: reset data[], allocate slots, emit the program.

        The slot of every Float is registered in comp_data.data_array.seen so
        later value edits go through refresh without a recompile."""
        comp_data.reset_data_array()
        rows, objs = flatten(self.header_unions)
        prog = compile_rows(rows)
        # register Float -> slot exactly as Float::compile would have
        shape_ops = [o for o in prog.op_dicts() if o["opcode"] == N.PT_OP_SHAPE]
        union_ops = [o for o in prog.op_dicts() if o["opcode"] == N.PT_OP_UNION_BEGIN]
        data = comp_data.data_array
        data.data = [float(x) for x in prog.data]
        ui = si = 0
        for obj in objs:
            if isinstance(obj, Union):
                op = union_ops[ui]; ui += 1
            else:
                op = shape_ops[si]; si += 1
            slots = [op["scale"], *op["position"], *op["rotation"], op["aabb_exaggeration"]]
            fl = list(obj.transform.floats())
            if isinstance(obj, Shape):
                nsz = len(obj.current_shape.params)
                slots += op["size"][:nsz] + op["material"]
                fl += list(obj.current_shape.floats()) + list(obj.material.floats())
            for f, sl in zip(fl, slots):
                data.seen[f.hash] = sl
        comp_data.aabb_index = prog.n_check if prog.n_check > 1 or shape_ops else 0
        return prog

    def data_update(self, comp_data: CompData) -> None:
        """sdf_editor.rs:248-252: value-only refresh of data[]."""
        for u in self.header_unions:
            u.refresh(comp_data)

    def update(self, path_tracer, comp_data: CompData) -> None:
        """SDFEditor::update (sdf_editor.rs:35-47) + SDFEditorPackage::update (:272-283)."""
        changed = comp_data.rec_update.queue_compile or comp_data.rec_update.queue_update
        if comp_data.rec_update.queue_compile:
            prog = self.compile(comp_data)
            path_tracer.remake_pipeline(prog)
        if comp_data.rec_update.queue_update:
            self.data_update(comp_data)
        comp_data.rec_update.reset()
        if changed:
            path_tracer.changed = True
            path_tracer.set_data(comp_data.data_array.as_array())

    # -- serde JSON (sdf_editor.rs:131-167) ----------------------------
    def to_json(self) -> dict:
        return {"header_unions": [u.to_json() for u in self.header_unions], "save_name": self.save_name}

    def dumps(self) -> str:
        return json.dumps(self.to_json(), indent=2)

    @classmethod
    def from_json(cls, d: dict) -> "SDFEditor":
        ed = cls([Union.from_json(u) for u in d["header_unions"]])
        ed.save_name = d.get("save_name", "")
        return ed

    @classmethod
    def loads(cls, s: str) -> "SDFEditor":
        return cls.from_json(json.loads(s))

    def rows(self) -> List[dict]:
        return flatten(self.header_unions)[0]
