// pt_scene.cpp -- the SDFEditor scene compiler, re-targeted from GLSL text to
// an op list (pt_op) + bounds list (pt_aabb) + the data[] parameter buffer.
//
// Mirrors, statement for statement, what the reference code generator emits:
//   SDFEditor::compile          src/sdf_editor/sdf_editor.rs:186-246
//   Union::compile              src/sdf_editor/containers.rs:143-179
//   Union::aabb_compile         src/sdf_editor/containers.rs:181-202
//   UnionType::compile          src/sdf_editor/containers.rs:244-252
//   Shape::compile/aabb_compile src/sdf_editor/containers.rs:404-463
//   Transform::compile/aabb_*   src/sdf_editor/data_structures.rs:45-96
//   Material::compile           src/sdf_editor/data_structures.rs:178-194
//   DataArray::get_index        src/sdf_editor/primitives.rs:117-129
// Slot numbering is identical to the reference (tests/golden/shader_out_topology
// pins it against the captured compiler output), so a Rust host keeps its
// CompData/DataArray unchanged.  Host code only.
#include <cstring>
#include <map>
#include <utility>
#include <vector>

#include "../../include/pt_abi.h"

namespace {

struct Tree {
    const pt_scene_node *n;
    uint32_t count;
    std::vector<std::vector<uint32_t>> child_unions, child_shapes;
    std::vector<uint32_t> top;
};

// Float positions inside a node's key block (pt_abi.h PT_NODE_FLOATS)
enum { KF_SCALE = 0, KF_POS = 1, KF_ROT = 4, KF_EX = 7, KF_SIZE = 8, KF_MAT = 11 };

struct Emit {
    std::vector<float> data;
    std::vector<pt_op> ops;
    std::vector<pt_aabb> aabbs;
    uint32_t aabb_index = 0;
    const pt_float_key *keys = nullptr;  // [node][PT_NODE_FLOATS], or none
    std::map<std::pair<uint64_t, uint64_t>, uint32_t> seen;
    // DataArray::get_index (primitives.rs:117-129): a Float whose hash was
    // seen before reuses that slot (its value stays the first one's); a new
    // hash -- or an anonymous Float, key {0, 0} -- appends a slot
    uint32_t slot(float v, uint32_t node, uint32_t k) {
        if (keys) {
            const pt_float_key &key = keys[size_t(node) * PT_NODE_FLOATS + k];
            if (key.lo | key.hi) {
                auto it = seen.find({key.lo, key.hi});
                if (it != seen.end()) return it->second;
                seen.emplace(std::make_pair(key.lo, key.hi), uint32_t(data.size()));
            }
        }
        data.push_back(v);
        return uint32_t(data.size() - 1);
    }
};

struct Slots {
    uint32_t scale, pos[3], rot[3], ex;
};

uint32_t size_count(int32_t kind) {
    switch (kind) {
        case PT_NODE_SPHERE: return 1;
        case PT_NODE_CUBE: return 3;
        case PT_NODE_TORUS: return 2;
        case PT_NODE_OCTAHEDRON: return 1;
        default: return 0;
    }
}

// Transform::compile (data_structures.rs:45-55): scale, position.xyz, scale
// again (get_index of a seen hash: no new slot), rotation.xyz, aabb_exaggeration
Slots transform(Emit &e, const pt_scene_node &n, uint32_t node) {
    Slots s;
    s.scale = e.slot(n.scale, node, KF_SCALE);
    for (uint32_t i = 0; i < 3; ++i) s.pos[i] = e.slot(n.position[i], node, KF_POS + i);
    for (uint32_t i = 0; i < 3; ++i) s.rot[i] = e.slot(n.rotation[i], node, KF_ROT + i);
    s.ex = e.slot(n.aabb_exaggeration, node, KF_EX);
    return s;
}

void fill(pt_op &op, const Slots &s) {
    op.scale = s.scale;
    for (int i = 0; i < 3; ++i) {
        op.position[i] = s.pos[i];
        op.rotation[i] = s.rot[i];
    }
    op.aabb_exaggeration = s.ex;
}

uint32_t combine_of(int32_t union_type, uint32_t index) {
    if (index == 0) return PT_COMBINE_ASSIGN;
    return union_type == PT_UNION_TYPE_SUBTRACTION ? PT_COMBINE_SUBTRACTION : PT_COMBINE_UNION;
}

// Union::compile(reference, depth, union_type): child unions combine with this
// union's type at index 1, shapes with this union's type at their own index.
void compile_union(const Tree &t, Emit &e, uint32_t u, int32_t type_in, std::vector<Slots> &slots_of,
                   std::vector<size_t> &op_of) {
    const pt_scene_node &un = t.n[u];
    pt_op begin;
    std::memset(&begin, 0, sizeof begin);
    begin.opcode = PT_OP_UNION_BEGIN;
    begin.check = -1;
    Slots us = transform(e, un, u);
    slots_of[u] = us;
    fill(begin, us);
    e.ops.push_back(begin);
    for (uint32_t c : t.child_unions[u]) compile_union(t, e, c, un.union_type, slots_of, op_of);
    uint32_t index = 0;
    for (uint32_t c : t.child_shapes[u]) {
        const pt_scene_node &sn = t.n[c];
        pt_op op;
        std::memset(&op, 0, sizeof op);
        op.opcode = PT_OP_SHAPE;
        op.shape = uint32_t(sn.kind);
        Slots ss = transform(e, sn, c);
        slots_of[c] = ss;
        fill(op, ss);
        uint32_t nsz = size_count(sn.kind);
        for (uint32_t k = 0; k < nsz; ++k) op.size[k] = e.slot(sn.size[k], c, KF_SIZE + k);
        for (uint32_t k = nsz; k < 3; ++k) op.size[k] = op.size[nsz ? nsz - 1 : 0];
        for (uint32_t k = 0; k < 18; ++k) op.material[k] = e.slot(sn.material[k], c, KF_MAT + k);
        // Transform::aabb_check: the index advances for every shape, aabb or not
        op.check = sn.aabb ? int32_t(e.aabb_index) : -1;
        e.aabb_index++;
        op.combine = combine_of(un.union_type, index++);
        op_of[c] = e.ops.size();
        e.ops.push_back(op);
    }
    pt_op end = begin;
    end.opcode = PT_OP_UNION_END;
    end.combine = combine_of(type_in, 1);
    e.ops.push_back(end);
}

}  // namespace

extern "C" int pt_compile_scene_keyed(const pt_scene_node *nodes, uint32_t n_nodes, const pt_float_key *keys,
                                      pt_op *ops, uint32_t ops_cap, uint32_t *n_ops, pt_aabb *aabbs, uint32_t aabb_cap,
                                      uint32_t *n_aabb, float *data, uint32_t data_cap, uint32_t *n_data,
                                      uint32_t *n_check) {
    if (n_nodes > 0 && !nodes) return PT_ERR_INVALID;
    Tree t;
    t.n = nodes;
    t.count = n_nodes;
    t.child_unions.resize(n_nodes);
    t.child_shapes.resize(n_nodes);
    bool plane = false;
    for (uint32_t i = 0; i < n_nodes; ++i) {
        const pt_scene_node &n = nodes[i];
        if (n.kind < PT_NODE_UNION || n.kind > PT_NODE_PLANE) return PT_ERR_INVALID;
        if (n.kind == PT_NODE_PLANE) plane = true;
        if (n.kind == PT_NODE_UNION && n.union_type != PT_UNION_TYPE_UNION &&
            n.union_type != PT_UNION_TYPE_SUBTRACTION)
            return PT_ERR_INVALID;
        if (n.parent == -1) {
            if (n.kind != PT_NODE_UNION) return PT_ERR_INVALID;  // header_unions holds unions
            t.top.push_back(i);
        } else {
            if (n.parent < 0 || uint32_t(n.parent) >= i || nodes[n.parent].kind != PT_NODE_UNION)
                return PT_ERR_INVALID;
            if (n.kind == PT_NODE_UNION) t.child_unions[n.parent].push_back(i);
            else t.child_shapes[n.parent].push_back(i);
        }
    }
    if (plane) return PT_ERR_UNSUPPORTED;  // Shapes::Plane emits NotImplemented(...) upstream

    Emit e;
    e.keys = keys;
    e.data.push_back(6969.69f);  // CompData::reset_data_array (primitives.rs:53-56)
    std::vector<Slots> slots_of(n_nodes);
    std::vector<size_t> op_of(n_nodes, 0);
    for (uint32_t u : t.top) compile_union(t, e, u, PT_UNION_TYPE_UNION, slots_of, op_of);
    uint32_t c = e.aabb_index > 0 ? e.aabb_index : 1;  // sdf_editor.rs:213

    // bounds(): direct shapes of the header unions only, with a fresh counter
    // (sdf_editor.rs:214-221, containers.rs:181-202, 442-463).
    uint32_t back = 0;
    for (uint32_t u : t.top) {
        for (uint32_t s : t.child_shapes[u]) {
            const pt_scene_node &sn = nodes[s];
            if (sn.aabb) {
                pt_aabb a;
                std::memset(&a, 0, sizeof a);
                a.back = int32_t(back);
                const Slots &us = slots_of[u], &ss = slots_of[s];
                for (int i = 0; i < 3; ++i) {
                    a.union_position[i] = us.pos[i];
                    a.shape_position[i] = ss.pos[i];
                }
                a.union_scale = us.scale;
                a.shape_scale = ss.scale;
                a.aabb_exaggeration = ss.ex;
                for (int i = 0; i < 3; ++i) a.size[i] = e.ops[op_of[s]].size[i];  // vec3(size) / size
                switch (sn.kind) {
                    case PT_NODE_SPHERE:
                    case PT_NODE_OCTAHEDRON: a.so_kind = PT_SO_SCALAR; break;
                    case PT_NODE_CUBE: a.so_kind = PT_SO_VEC3; break;
                    case PT_NODE_TORUS: a.so_kind = PT_SO_TORUS; break;
                    default: a.so_kind = PT_SO_ONE; break;
                }
                e.aabbs.push_back(a);
            }
            back++;  // Shape::aabb_compile bumps the counter for `if (false)` too
        }
    }

    if (n_ops) *n_ops = uint32_t(e.ops.size());
    if (n_aabb) *n_aabb = uint32_t(e.aabbs.size());
    if (n_data) *n_data = uint32_t(e.data.size());
    if (n_check) *n_check = c;
    bool small = false;
    if (ops) {
        if (ops_cap < e.ops.size()) small = true;
        else std::memcpy(ops, e.ops.data(), e.ops.size() * sizeof(pt_op));
    }
    if (aabbs) {
        if (aabb_cap < e.aabbs.size()) small = true;
        else if (!e.aabbs.empty()) std::memcpy(aabbs, e.aabbs.data(), e.aabbs.size() * sizeof(pt_aabb));
    }
    if (data) {
        if (data_cap < e.data.size()) small = true;
        else std::memcpy(data, e.data.data(), e.data.size() * sizeof(float));
    }
    return small ? PT_ERR_SIZE : PT_OK;
}

extern "C" int pt_compile_scene(const pt_scene_node *nodes, uint32_t n_nodes, pt_op *ops, uint32_t ops_cap,
                                uint32_t *n_ops, pt_aabb *aabbs, uint32_t aabb_cap, uint32_t *n_aabb, float *data,
                                uint32_t data_cap, uint32_t *n_data, uint32_t *n_check) {
    return pt_compile_scene_keyed(nodes, n_nodes, nullptr, ops, ops_cap, n_ops, aabbs, aabb_cap, n_aabb, data, data_cap,
                                  n_data, n_check);
}
