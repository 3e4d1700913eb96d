"""The scene compiler (pt_compile_scene) and the editor mirror.  No GPU."""
import ctypes
import json
import os

import numpy as np
import pytest

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.sdf_editor import (CompData, SDFEditor, Shape, Shapes, Union, UnionType, compile_rows,
                                                nodes_to_ctypes)
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _captured_scene() -> SDFEditor:
    """The tree behind shader_out/test_compute.glsl: header union "BOX"
    (Subtraction, two cubes, aabb off) and "stuffs" (Union: sphere, cube,
    sphere, sphere, cube, aabb on)."""
    box = Union(UnionType.SUBTRACTION)
    box.name = "BOX"
    for _ in range(2):
        s = Shape(Shapes.CUBE)
        s.transform.aabb = False
        box.children_shapes.append(s)
    stuffs = Union(UnionType.UNION)
    stuffs.name = "stuffs"
    for k in (Shapes.SPHERE, Shapes.CUBE, Shapes.SPHERE, Shapes.SPHERE, Shapes.CUBE):
        stuffs.children_shapes.append(Shape(k))
    return SDFEditor([box, stuffs])


def test_topology_matches_captured_compiler_output():
    fx = json.load(open(os.path.join(GOLD, "shader_out_topology.json")))
    prog = _captured_scene().compile(CompData())
    assert prog.n_check == fx["n_check"] == 7
    assert len(prog.data) == 214  # data[0..213]
    ops = prog.op_dicts()
    i = 0
    comb = {"assign": N.PT_COMBINE_ASSIGN, "opUnion": N.PT_COMBINE_UNION, "opSubtraction": N.PT_COMBINE_SUBTRACTION}
    for u in fx["unions"]:
        b = ops[i]
        assert b["opcode"] == N.PT_OP_UNION_BEGIN
        assert b["scale"] == u["scale"] == u["scale_again"] and b["position"] == u["position"]
        assert b["rotation"] == u["rotation"]
        i += 1
        for s in u["shapes"]:
            o = ops[i]
            assert o["opcode"] == N.PT_OP_SHAPE
            assert o["shape"] == (N.PT_NODE_CUBE if s["kind"] == "Cube" else N.PT_NODE_SPHERE)
            assert o["scale"] == s["scale"] == s["scale_again"] == s["finalise_scale"]
            assert o["position"] == s["position"] and o["rotation"] == s["rotation"]
            nsz = len(s["size"])
            assert o["size"][:nsz] == s["size"]
            assert o["material"] == s["material"]
            assert o["check"] == (-1 if s["check"] is None else s["check"])
            assert o["combine"] == comb[s["combine"]]
            i += 1
        e = ops[i]
        assert e["opcode"] == N.PT_OP_UNION_END and e["combine"] == comb[u["combine"]]
        i += 1
    assert i == prog.n_ops
    boxes = {a["back"]: a for a in prog.aabb_dicts()}
    for b in fx["bounds"]:
        if not b["enabled"]:
            assert b["back"] not in boxes
            continue
        a = boxes[b["back"]]
        assert a["union_position"] == b["union_position"] and a["shape_position"] == b["shape_position"]
        assert a["union_scale"] == b["union_scale"] and a["shape_scale"] == b["shape_scale"]
        assert a["aabb_exaggeration"] == b["aabb_exaggeration"]
        so = b["size"]
        assert a["size"][:len(so)] == so
        assert a["so_kind"] == (N.PT_SO_SCALAR if len(so) == 1 else N.PT_SO_VEC3)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "nested", "empty"])
def test_product_compiler_matches_oracle_restatement(name):
    ed = scenes.SCENES[name]()
    rows = ed.rows()
    prog = ed.compile(CompData())
    osc = O.OracleScene(rows)
    assert np.array_equal(prog.data.view(np.uint32), osc.data().view(np.uint32))
    assert prog.n_check == osc.n_check
    shapes = [o for o in prog.op_dicts() if o["opcode"] == N.PT_OP_SHAPE]
    si = 0
    for i, r in enumerate(rows):
        slots, chk, bidx = osc.node_slots(i)
        if r["kind"] == N.PT_NODE_UNION:
            continue
        o = shapes[si]
        si += 1
        assert [o["scale"], *o["position"], *o["rotation"], o["aabb_exaggeration"]] == slots[:8]
        nsz = {1: 1, 2: 3, 3: 2, 4: 1}[r["kind"]]
        assert o["size"][:nsz] == slots[8:8 + nsz]
        assert o["material"] == slots[11:29]
        assert o["check"] == chk
    boxes = prog.aabb_dicts()
    assert sorted(a["back"] for a in boxes) == sorted(
        osc.node_slots(i)[2] for i, r in enumerate(rows) if r["kind"] != 0 and r["aabb"] and osc.node_slots(i)[2] >= 0)


def test_nested_quirks():
    """child unions combine first and the index-0 shape
    overwrites them; map() check[] indices run DFS over all shapes while
    bounds() only numbers the header unions' direct shapes."""
    prog = scenes.nested_demo().compile(CompData())
    ops = prog.op_dicts()
    # outer: BEGIN, inner BEGIN, deeper BEGIN, c, END, a, b, END, d(assign!), e, END
    seq = [(o["opcode"], o["combine"]) for o in ops]
    assert seq[:11] == [(0, 0), (0, 0), (0, 0), (1, 0), (2, 2), (1, 0), (1, 2), (2, 1), (1, 0), (1, 1), (2, 1)]
    checks = [o["check"] for o in ops if o["opcode"] == N.PT_OP_SHAPE]
    assert checks == [0, 1, 2, -1, -1, -1]  # d, e (aabb off), lamp (aabb off)
    assert sorted(a["back"] for a in prog.aabb_dicts()) == []  # d/e/lamp are the only bounds() shapes


def test_compile_errors_and_two_call_pattern():
    L = N.lib()
    ed = SDFEditor([Union()])
    ed.header_unions[0].children_shapes.append(Shape(Shapes.PLANE))
    with pytest.raises(N.NativeError) as e:
        ed.compile(CompData())
    assert e.value.code == N.PT_ERR_UNSUPPORTED
    rows = scenes.c2_sphere_box_torus().rows()
    bad = [dict(r) for r in rows]
    bad[1]["parent"] = 5  # parent after child
    with pytest.raises(N.NativeError):
        compile_rows(bad)
    top_shape = [dict(rows[1], parent=-1)]
    with pytest.raises(N.NativeError):
        compile_rows(top_shape)
    nodes = nodes_to_ctypes(rows)
    n_ops, n_aabb, n_data, n_check = (ctypes.c_uint32() for _ in range(4))
    small = (N.Op * 1)()
    rc = L.pt_compile_scene(nodes, len(rows), small, 1, ctypes.byref(n_ops), None, 0, ctypes.byref(n_aabb), None, 0,
                            ctypes.byref(n_data), ctypes.byref(n_check))
    assert rc == N.PT_ERR_SIZE and n_ops.value == 12 and n_data.value == 193 and n_check.value == 6


def test_editor_json_round_trip_and_refresh():
    ed = scenes.c3_graph32()
    cd = CompData()
    prog = ed.compile(cd)
    s = ed.dumps()
    ed2 = SDFEditor.loads(s)
    assert ed2.dumps() == s
    cd2 = CompData()
    prog2 = ed2.compile(cd2)
    assert np.array_equal(prog.data, prog2.data)
    # value-only edit: refresh writes the same slot the compiler allocated
    u = ed.header_unions[1]
    f = u.children_shapes[3].transform.position.y
    slot = cd.data_array.seen[f.hash]
    f.set(0.125)
    ed.data_update(cd)
    assert cd.data_array.data[slot] == np.float32(0.125)
    # the recompiled program allocates identical slots with the new value
    prog3 = ed.compile(CompData())
    assert np.array_equal(prog3.data, cd.data_array.as_array())


def test_default_editor_scene():
    """SDFEditor::new (sdf_editor.rs:20-33): one union + unit sphere, 36 floats."""
    ed = SDFEditor()
    prog = ed.compile(CompData())
    assert len(prog.data) == 36 and prog.data[0] == np.float32(6969.69)
    assert prog.n_ops == 3 and prog.n_aabb == 1 and prog.n_check == 1
    assert prog.data[8] == np.float32(1.3)  # aabb_exaggeration default


GOLDEN_MAP = os.path.join(os.path.dirname(__file__), "golden", "maps_test.json")


def test_deprecated_map_loads_and_pins_c3_room():
    """assets/maps/test.json (the deprecated node-editor save, committed as a
    data fixture) loads into the current editor; c3's room copies its values."""
    from compute_path_tracer_amd.scenes import deprecated_map

    ed = deprecated_map(GOLDEN_MAP)
    (u,) = ed.header_unions
    assert [s.name for s in u.children_shapes] == ["floor", "roof", "light", "4", "5", "6", "7", "8"]
    assert [s.current_shape.kind for s in u.children_shapes].count("Octahedron") == 2
    prog = ed.compile(CompData())
    assert prog.n_aabb == 8 and prog.n_check == 8
    room = {s.name: s for s in scenes.c3_graph32().header_unions[0].children_shapes}
    for s in u.children_shapes:
        if s.name not in room:
            continue
        r = room[s.name]
        for get in (lambda x: x.transform.position.vals(), lambda x: x.transform.rotation.vals(),
                    lambda x: [p.val for p in x.current_shape.params], lambda x: x.material.color.vals(),
                    lambda x: x.material.light_col.vals(), lambda x: [x.material.brightness.val],
                    lambda x: [x.material.specular_chance.val], lambda x: x.material.specular_color.vals()):
            assert get(s) == get(r), s.name


SHARED = os.path.join(GOLD, "shared_hashes.json")
MAT_ORDER = ("color", "brightness", "light_col", "specular_chance", "specular_color", "roughness", "ior",
             "refract_chance", "refract_roughness", "refract_color")


def _v3(d):
    return [d["x"], d["y"], d["z"]]


def _size_floats(cs):
    (kind, v), = cs.items()
    return _v3(v) if kind == "Cube" else (v if kind == "Torus" else [v])


def _mat_floats(m):
    out = []
    for k in MAT_ORDER:
        out += _v3(m[k]) if "x" in m[k] else [m[k]]
    return out


class _RefData:
    """DataArray restated from primitives.rs:117-129,153-156 on the JSON."""

    def __init__(self):
        self.data, self.seen = [np.float32(6969.69)], {}

    def get_index(self, f):
        if f["hash"] not in self.seen:
            self.data.append(np.float32(f["val"]))
            self.seen[f["hash"]] = len(self.data) - 1
        return self.seen[f["hash"]]

    def refresh(self, f):
        self.data[self.seen[f["hash"]]] = np.float32(f["val"])


def _ref_compile(d):
    """Slots per node in the reference's Float::compile call order
    (sdf_editor.rs:186-246 -> containers.rs:143-179,404-440 ->
    data_structures.rs:45-55 (scale, position, scale again, rotation,
    exaggeration), :178-194), as the 29-slot rows pto_scene_node_slots
    reports (a union's size/material slots -1)."""
    D, rows = _RefData(), []

    def transform(t):
        s = [D.get_index(t["scale"])] + [D.get_index(f) for f in _v3(t["position"])]
        D.get_index(t["scale"])
        s += [D.get_index(f) for f in _v3(t["rotation"])] + [D.get_index(t["aabb_exaggeration"])]
        return s

    def union(u):
        rows.append(transform(u["transform"]) + [-1] * 21)
        for c in u["children_unions"]:
            union(c)
        for sh in u["children_shapes"]:
            s = transform(sh["transform"])
            sz = [D.get_index(f) for f in _size_floats(sh["current_shape"])]
            s += sz + [-1] * (3 - len(sz)) + [D.get_index(f) for f in _mat_floats(sh["material"])]
            rows.append(s)

    for u in d["header_unions"]:
        union(u)
    for u in d["header_unions"]:  # aabb_compile re-reads seen hashes only (containers.rs:181-202)
        for sh in u["children_shapes"]:
            assert all(f["hash"] in D.seen for f in _v3(sh["transform"]["position"]) + [sh["transform"]["scale"]])
    return D, rows


def _ref_refresh(d, D):
    """SDFEditor::data_update (sdf_editor.rs:248-252): Union::refresh
    (transform, shapes, child unions), Shape::refresh (transform, material,
    size), Transform::refresh (position, rotation, scale, exaggeration)."""
    def transform(t):
        for f in _v3(t["position"]) + _v3(t["rotation"]) + [t["scale"], t["aabb_exaggeration"]]:
            D.refresh(f)

    def union(u):
        transform(u["transform"])
        for sh in u["children_shapes"]:
            transform(sh["transform"])
            for f in _mat_floats(sh["material"]) + _size_floats(sh["current_shape"]):
                D.refresh(f)
        for c in u["children_unions"]:
            union(c)

    for u in d["header_unions"]:
        union(u)


def test_shared_hashes_share_slots_like_get_index():
    """Floats that share a hash share one data[] slot holding the first
    value (primitives.rs:117-129): product compiler and oracle both match the
    restatement of the reference's compile order on the fixture."""
    d = json.load(open(SHARED))
    D, ref_rows = _ref_compile(d)
    ed = SDFEditor.from_json(d)
    cd = CompData()
    prog = ed.compile(cd)
    assert len(prog.data) == len(D.data) < len(scenes.c2_sphere_box_torus().compile(CompData()).data) + 29 + 1
    assert np.array_equal(prog.data.view(np.uint32), np.array(D.data, np.float32).view(np.uint32))
    rows = ed.rows()
    osc = O.OracleScene(rows)
    assert np.array_equal(osc.data().view(np.uint32), prog.data.view(np.uint32))
    ops = [o for o in prog.op_dicts() if o["opcode"] != N.PT_OP_UNION_END]
    assert len(ops) == len(rows) == len(ref_rows)
    for i, (o, r) in enumerate(zip(ops, ref_rows)):
        got = [o["scale"], *o["position"], *o["rotation"], o["aabb_exaggeration"]]
        assert got == r[:8], i
        assert osc.node_slots(i)[0][:8] == r[:8], i
        if o["opcode"] == N.PT_OP_SHAPE:
            nsz = 3 - r[8:11].count(-1)
            assert o["size"][:nsz] == r[8:8 + nsz] and o["material"] == r[11:29], i
            assert osc.node_slots(i)[0][8:8 + nsz] == r[8:8 + nsz] and osc.node_slots(i)[0][11:29] == r[11:29]
    # the clone shares every slot with the box; the clone's own position value is dropped
    box, clone = ops[2], ops[3]
    assert {k: v for k, v in box.items() if k != "check"} == {k: v for k, v in clone.items() if k != "check"}
    assert (box["check"], clone["check"]) == (1, 2)  # Transform::aabb_check counts every shape
    assert prog.data[box["position"][0]] == np.float32(0.8)
    assert box["rotation"][0] == box["rotation"][2] != box["rotation"][1]
    sphere = ops[1]
    assert box["material"][8:11] == sphere["material"][0:3]
    # the Python DataArray registers the same slots (refresh targets)
    for i, r in enumerate(ref_rows):
        assert all(cd.data_array.data[s] == D.data[s] for s in r if s >= 0)


def test_shared_hashes_refresh_writes_like_the_reference():
    """A value-only refresh with shared hashes: every Float writes its slot
    in the reference's refresh order, so the last writer wins (the clone's
    -1.6 replaces the box's 0.8)."""
    d = json.load(open(SHARED))
    ed = SDFEditor.from_json(d)
    cd = CompData()
    ed.compile(cd)
    ed.header_unions[0].children_shapes[0].material.color.set((0.3, 0.6, 0.9))  # shared with the box's spec colour
    ed.header_unions[0].children_shapes[1].transform.rotation.x.set(0.45)  # shared with its rotation z
    ed.data_update(cd)
    d2 = ed.to_json()
    D, _ = _ref_compile(d)
    _ref_refresh(d2, D)
    assert np.array_equal(cd.data_array.as_array().view(np.uint32), np.array(D.data, np.float32).view(np.uint32))
    prog = ed.compile(CompData())
    box = [o for o in prog.op_dicts() if o["opcode"] == N.PT_OP_SHAPE][1]
    assert cd.data_array.data[box["position"][0]] == np.float32(-1.6)
    # rotation z's Float still holds its own (stale) value: its refresh runs
    # after x's and writes it back over the shared slot
    assert cd.data_array.data[box["rotation"][0]] == np.float32(ed.header_unions[0].children_shapes[1]
                                                                 .transform.rotation.z.val)


def test_keyed_compile_without_keys_is_the_plain_compile():
    rows = scenes.c3_graph32().rows()
    for r in rows:
        r.pop("keys")
    a = compile_rows(rows)
    b = scenes.c3_graph32().compile(CompData())
    assert np.array_equal(a.data, b.data) and a.op_dicts() == b.op_dicts()
