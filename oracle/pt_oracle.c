/*
 * pt_oracle.c -- CPU restatement of the reference SDF path tracer (TEST
 * INFRASTRUCTURE ONLY; see pt_oracle.h for scope and the parity status).
 *
 * Build: oracle/Makefile  (-O3 -ffp-contract=off: no FMA contraction; every
 * fused multiply-add below is an explicit fmaf that the semantics contract
 * asks for).  Each function cites the reference file:line it restates.
 */
#define _GNU_SOURCE
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* test_compute.glsl:26-38 */
#define STEPS 80
#define MHD 0.001f
#define FP 100.0f
#define OFFSET 0.03f
static const float PI = 3.14159265359f;
#define PI2 (2.0f * PI)
#define MAXHIT_D 10000.0f /* sdf_editor.rs:193 */

/* GLSL min/max: naga emits SPIR-V GLSL.std.450 FMin/FMax, which drivers run
 * on the hardware min/max (gfx950 v_min/v_max_f32 = IEEE-754 minNum/maxNum:
 * a NaN operand yields the other operand, -0 < +0).  Spelled out here so the
 * result does not depend on the host libm. */
static inline float gmin(float x, float y)
{
    if (x != x) return y;
    if (y != y) return x;
    if (x == 0.0f && y == 0.0f) return (signbit(x) || signbit(y)) ? -0.0f : 0.0f;
    return (y < x) ? y : x;
}
static inline float gmax(float x, float y)
{
    if (x != x) return y;
    if (y != y) return x;
    if (x == 0.0f && y == 0.0f) return (signbit(x) && signbit(y)) ? -0.0f : 0.0f;
    return (x < y) ? y : x;
}
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
static inline float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline float length3(const float a[3]) { return sqrtf(dot3(a, a)); }
static inline void normalize3(const float a[3], float o[3]) {
    float l = length3(a);
    o[0] = a[0] / l; o[1] = a[1] / l; o[2] = a[2] / l;
}

/* ------------------------------------------------------------------ */
/* RNG: rng.glsl:1-36                                                   */
/* ------------------------------------------------------------------ */
uint32_t pto_wang_hash(uint32_t *seed) /* rng.glsl:1-9 */
{
    uint32_t s = *seed;
    s = (uint32_t)(s ^ 61u) ^ (uint32_t)(s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    *seed = s;
    return s;
}

float pto_random01(uint32_t *state) /* rng.glsl:11-14: float(u) / 4294967296.0 */
{
    return (float)pto_wang_hash(state) / 4294967296.0f;
}

/* sin/cos: the GLSL builtins' precision is driver-defined (unpinned); the
 * contract fixes this polynomial, evaluated with explicit fmaf
 * so the HIP kernel and the host agree bit for bit. */
static float sin_poly(float r)
{
    float s = r * r;
    float p = fmaf(s, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(s, p, -1.6666654611e-1f);
    return fmaf(r * s, p, r);
}
static float cos_poly(float r)
{
    float s = r * r;
    float p = fmaf(s, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(s, p, 4.166664568298827e-2f);
    float t = fmaf(s, p, -0.5f);
    return fmaf(s, t, 1.0f);
}
static float sincos_q(float x, int shift)
{
    if (!(fabsf(x) <= 16777216.0f)) return (x - x) / (x - x); /* NaN for inf/NaN/huge */
    float k = rintf(x * 0.63661977236758134f);
    float r = fmaf(-k, 1.5703125f, x);
    r = fmaf(-k, 4.837512969970703125e-4f, r);
    r = fmaf(-k, 7.549789954891882e-8f, r);
    int q = ((int)k + shift) & 3;
    switch (q) {
    case 0: return sin_poly(r);
    case 1: return cos_poly(r);
    case 2: return -sin_poly(r);
    default: return -cos_poly(r);
    }
}
float pto_sin(float x) { return sincos_q(x, 0); }
float pto_cos(float x) { return sincos_q(x, 1); }

static void random_unit_vector(uint32_t *state, float o[3]) /* rng.glsl:16-24 */
{
    float z = pto_random01(state) * 2.0f - 1.0f;
    float a = pto_random01(state) * PI2;
    float r = sqrtf(1.0f - z * z);
    o[0] = r * pto_cos(a);
    o[1] = r * pto_sin(a);
    o[2] = z;
}

uint32_t pto_gen_rng(int32_t x, int32_t y, int32_t frame, int32_t w, int32_t h) /* rng.glsl:26-36 */
{
    float fx = (float)w, fy = (float)h;
    uint32_t a = (uint32_t)(((float)x * 0.5f + 0.5f) * fx);
    uint32_t b = (uint32_t)(((float)y * 0.5f + 0.5f) * fy);
    return (uint32_t)(a * 1973u + b * 9277u + (uint32_t)frame * 26699u) | 1u;
}

/* ------------------------------------------------------------------ */
/* Scene: the editor tree + data[] slots (SDFEditor::compile restated)  */
/* ------------------------------------------------------------------ */
#define NSLOT 29 /* 8 transform + 3 size + 18 material */
enum { SL_SCALE = 0, SL_POS = 1, SL_ROT = 4, SL_EX = 7, SL_SIZE = 8, SL_MAT = 11 };

typedef struct {
    int kind, parent, utype, aabb;
    int *cu, ncu;  /* child unions */
    int *cs, ncs;  /* child shapes */
    int32_t slot[NSLOT];
    int32_t check; /* map(): check[] index, -1 = if (true) */
    int32_t bidx;  /* bounds(): back[] index, -1 = not visited */
} onode;

struct pto_scene {
    int n;
    onode *nd;
    const uint64_t *keys; /* [node][NSLOT][2] Float hashes while compiling, or NULL */
    int32_t *key_slot;    /* slot of each key position seen so far (first occurrence) */
    int *top, ntop;
    float *data;
    int ndata, cap;
    int ncheck;
    int nbounds;
    int *bshape, *bunion; /* bounds() visiting order */
};

static int alloc_slot(pto_scene *s, float v) /* primitives.rs:117-129 (DataArray::get_index) */
{
    if (s->ndata == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 64;
        s->data = (float *)realloc(s->data, sizeof(float) * (size_t)s->cap);
    }
    s->data[s->ndata] = v;
    return s->ndata++;
}

/* get_index with the Float's hash: a hash seen before returns its slot (the
 * slot keeps the first value); a new hash, or {0, 0} (anonymous), appends. */
static int alloc_keyed(pto_scene *s, float v, int node, int k)
{
    if (s->keys) {
        const uint64_t *key = s->keys + 2 * ((size_t)node * NSLOT + (size_t)k);
        if (key[0] | key[1]) {
            for (size_t j = 0; j < (size_t)s->n * NSLOT; j++) {
                const uint64_t *o = s->keys + 2 * j;
                if (s->key_slot[j] >= 0 && o[0] == key[0] && o[1] == key[1]) return s->key_slot[j];
            }
            return s->key_slot[(size_t)node * NSLOT + (size_t)k] = alloc_slot(s, v);
        }
    }
    return alloc_slot(s, v);
}

static int size_count(int kind)
{
    switch (kind) {
    case PTO_SPHERE: return 1;
    case PTO_CUBE: return 3;
    case PTO_TORUS: return 2;
    case PTO_OCTAHEDRON: return 1;
    default: return 0;
    }
}

/* Transform::compile (data_structures.rs:45-55): scale, position.xyz,
 * (scale again, reused), rotation.xyz, aabb_exaggeration. */
static void alloc_transform(pto_scene *s, onode *o, const pto_node *src, int node)
{
    o->slot[SL_SCALE] = alloc_keyed(s, src->scale, node, SL_SCALE);
    for (int i = 0; i < 3; i++) o->slot[SL_POS + i] = alloc_keyed(s, src->pos[i], node, SL_POS + i);
    for (int i = 0; i < 3; i++) o->slot[SL_ROT + i] = alloc_keyed(s, src->rot[i], node, SL_ROT + i);
    o->slot[SL_EX] = alloc_keyed(s, src->aabb_ex, node, SL_EX);
}

/* Union::compile (containers.rs:143-179) + Shape::compile (:404-440) slot order */
static void compile_union(pto_scene *s, const pto_node *src, int u, int *aabb_index)
{
    onode *o = &s->nd[u];
    alloc_transform(s, o, &src[u], u);
    for (int i = 0; i < o->ncu; i++) compile_union(s, src, o->cu[i], aabb_index);
    for (int i = 0; i < o->ncs; i++) {
        int c = o->cs[i];
        onode *sh = &s->nd[c];
        alloc_transform(s, sh, &src[c], c);
        int nsz = size_count(sh->kind);
        for (int k = 0; k < nsz; k++) sh->slot[SL_SIZE + k] = alloc_keyed(s, src[c].size[k], c, SL_SIZE + k);
        for (int k = 0; k < 18; k++) sh->slot[SL_MAT + k] = alloc_keyed(s, src[c].mat[k], c, SL_MAT + k);
        /* Transform::aabb_check (data_structures.rs:57-66): index bumps for every shape */
        sh->check = sh->aabb ? *aabb_index : -1;
        (*aabb_index)++;
    }
}

int pto_scene_build_keyed(const pto_node *nodes, int n, const uint64_t *keys, pto_scene **out)
{
    *out = NULL;
    if (n < 0 || (n > 0 && !nodes)) return -1;
    pto_scene *s = (pto_scene *)calloc(1, sizeof(pto_scene));
    s->n = n;
    s->nd = (onode *)calloc((size_t)(n > 0 ? n : 1), sizeof(onode));
    s->top = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    int rc = 0;
    for (int i = 0; i < n; i++) {
        onode *o = &s->nd[i];
        o->kind = nodes[i].kind;
        o->parent = nodes[i].parent;
        o->utype = nodes[i].union_type;
        o->aabb = nodes[i].aabb != 0;
        for (int k = 0; k < NSLOT; k++) o->slot[k] = -1;
        o->check = -1;
        o->bidx = -1;
        o->cu = (int *)calloc((size_t)n, sizeof(int));
        o->cs = (int *)calloc((size_t)n, sizeof(int));
        if (o->kind < PTO_UNION || o->kind > PTO_PLANE) rc = -1;
        if (o->kind == PTO_PLANE) rc = rc ? rc : -2; /* containers.rs:287,295 NotImplemented */
        if (o->kind == PTO_UNION && o->utype != PTO_TYPE_UNION && o->utype != PTO_TYPE_SUBTRACTION) rc = -1;
        int p = o->parent;
        if (p == -1) {
            if (o->kind != PTO_UNION) rc = -1; /* header_unions holds unions only */
            else s->top[s->ntop++] = i;
        } else if (p < 0 || p >= i || nodes[p].kind != PTO_UNION) {
            rc = -1;
        } else if (o->kind == PTO_UNION) {
            s->nd[p].cu[s->nd[p].ncu++] = i;
        } else {
            s->nd[p].cs[s->nd[p].ncs++] = i;
        }
    }
    if (rc != 0) { pto_scene_free(s); return rc; }
    alloc_slot(s, 6969.69f); /* reset_data_array, primitives.rs:53-56 */
    if (keys) {
        s->keys = keys;
        s->key_slot = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1) * NSLOT);
        for (size_t j = 0; j < (size_t)(n > 0 ? n : 1) * NSLOT; j++) s->key_slot[j] = -1;
    }
    int aabb_index = 0;
    for (int t = 0; t < s->ntop; t++) compile_union(s, nodes, s->top[t], &aabb_index);
    free(s->key_slot);
    s->key_slot = NULL;
    s->keys = NULL;
    s->ncheck = aabb_index > 0 ? aabb_index : 1; /* sdf_editor.rs:213 */
    /* bounds(): only direct shapes of header unions, own counter (containers.rs:181-202,442-463) */
    s->bshape = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    s->bunion = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    for (int t = 0; t < s->ntop; t++) {
        onode *u = &s->nd[s->top[t]];
        for (int i = 0; i < u->ncs; i++) {
            s->nd[u->cs[i]].bidx = s->nbounds;
            s->bshape[s->nbounds] = u->cs[i];
            s->bunion[s->nbounds] = s->top[t];
            s->nbounds++;
        }
    }
    *out = s;
    return 0;
}

int pto_scene_build(const pto_node *nodes, int n, pto_scene **out)
{
    return pto_scene_build_keyed(nodes, n, NULL, out);
}

void pto_scene_free(pto_scene *s)
{
    if (!s) return;
    for (int i = 0; i < s->n; i++) { free(s->nd[i].cu); free(s->nd[i].cs); }
    free(s->nd); free(s->top); free(s->data); free(s->bshape); free(s->bunion);
    free(s);
}
int pto_scene_n_data(const pto_scene *s) { return s->ndata; }
int pto_scene_n_check(const pto_scene *s) { return s->ncheck; }
void pto_scene_get_data(const pto_scene *s, float *out) { memcpy(out, s->data, sizeof(float) * (size_t)s->ndata); }
int pto_scene_set_data(pto_scene *s, const float *data, int n)
{
    if (n != s->ndata) return -1;
    memcpy(s->data, data, sizeof(float) * (size_t)n);
    return 0;
}
void pto_scene_node_slots(const pto_scene *s, int node, int32_t *slots29, int32_t *check, int32_t *bidx)
{
    memcpy(slots29, s->nd[node].slot, sizeof(int32_t) * NSLOT);
    *check = s->nd[node].check;
    *bidx = s->nd[node].bidx;
}

/* ------------------------------------------------------------------ */
/* map(): the generated code's semantics                                */
/* ------------------------------------------------------------------ */
typedef struct { float d; int32_t mat; } hit_t; /* mat: shape node index, -1 = MDEF */

#define D(i) (s->data[(i)])

/* rot3D (shapes.glsl:34-68): GLSL column-major mat3 constructors, M*v summed
 * column by column left to right. */
static void mat3_mul(const float m[9] /* column-major */, const float v[3], float o[3])
{
    for (int r = 0; r < 3; r++) o[r] = m[0 + r] * v[0] + m[3 + r] * v[1] + m[6 + r] * v[2];
}
static void rot3d(const float p[3], const float rot[3], float o[3])
{
    float cX = pto_cos(rot[0]), sX = pto_sin(rot[0]);
    float mx[9] = {1.0f, 0.0f, 0.0f, 0.0f, cX, -sX, 0.0f, sX, cX};
    float cY = pto_cos(rot[1]), sY = pto_sin(rot[1]);
    float my[9] = {cY, 0.0f, sY, 0.0f, 1.0f, 0.0f, -sY, 0.0f, cY};
    float cZ = pto_cos(rot[2]), sZ = pto_sin(rot[2]);
    float mz[9] = {cZ, -sZ, 0.0f, sZ, cZ, 0.0f, 0.0f, 0.0f, 1.0f};
    float a[3], b[3];
    mat3_mul(mx, p, a);
    mat3_mul(my, a, b);
    mat3_mul(mz, b, o);
}

/* Transform::compile (data_structures.rs:45-55):
 *   p *= 1.0 / s;  p = move(p, pos * (1.0 / s));  p = rot3D(p, rot); */
static void xform(const pto_scene *s, const onode *o, const float in[3], float out[3])
{
    float inv = 1.0f / D(o->slot[SL_SCALE]);
    float p[3] = {in[0] * inv, in[1] * inv, in[2] * inv};
    float inv2 = 1.0f / D(o->slot[SL_SCALE]);
    float m[3] = {D(o->slot[SL_POS]) * inv2, D(o->slot[SL_POS + 1]) * inv2, D(o->slot[SL_POS + 2]) * inv2};
    p[0] = p[0] - m[0]; p[1] = p[1] - m[1]; p[2] = p[2] - m[2]; /* move, shapes.glsl:30-32 */
    float rot[3] = {D(o->slot[SL_ROT]), D(o->slot[SL_ROT + 1]), D(o->slot[SL_ROT + 2])};
    rot3d(p, rot, out);
}

static float sd_sphere(const float p[3], float r) { return length3(p) - r; } /* shapes.glsl:1-3 */
static float sd_cube(const float p[3], const float b[3])                  /* shapes.glsl:5-9 */
{
    float q[3] = {fabsf(p[0]) - b[0], fabsf(p[1]) - b[1], fabsf(p[2]) - b[2]};
    float m[3] = {gmax(q[0], 0.0f), gmax(q[1], 0.0f), gmax(q[2], 0.0f)};
    return length3(m) + gmin(gmax(q[0], gmax(q[1], q[2])), 0.0f);
}
static float sd_octahedron(const float pin[3], float s) /* shapes.glsl:13-25 */
{
    float p[3] = {fabsf(pin[0]), fabsf(pin[1]), fabsf(pin[2])};
    float m = p[0] + p[1] + p[2] - s;
    float q[3];
    if (3.0f * p[0] < m) { q[0] = p[0]; q[1] = p[1]; q[2] = p[2]; }
    else if (3.0f * p[1] < m) { q[0] = p[1]; q[1] = p[2]; q[2] = p[0]; }
    else if (3.0f * p[2] < m) { q[0] = p[2]; q[1] = p[0]; q[2] = p[1]; }
    else return m * 0.57735027f;
    float k = gclamp(0.5f * (q[2] - q[1] + s), 0.0f, s);
    float v[3] = {q[0], q[1] - s + k, q[2] - k};
    return length3(v);
}
/* Build extension (absent upstream): iq's sdTorus(p, vec2(R, r)) =
 * length(vec2(length(p.xz) - R, p.y)) - r. */
static float sd_torus(const float p[3], float R, float r)
{
    float qx = sqrtf(p[0] * p[0] + p[2] * p[2]) - R;
    return sqrtf(qx * qx + p[1] * p[1]) - r;
}

static float sdf(const pto_scene *s, const onode *o, const float p[3])
{
    switch (o->kind) {
    case PTO_SPHERE: return sd_sphere(p, D(o->slot[SL_SIZE]));
    case PTO_CUBE: {
        float b[3] = {D(o->slot[SL_SIZE]), D(o->slot[SL_SIZE + 1]), D(o->slot[SL_SIZE + 2])};
        return sd_cube(p, b);
    }
    case PTO_TORUS: return sd_torus(p, D(o->slot[SL_SIZE]), D(o->slot[SL_SIZE + 1]));
    case PTO_OCTAHEDRON: return sd_octahedron(p, D(o->slot[SL_SIZE]));
    default: return 0.0f;
    }
}

/* opUnion / opSubtraction, shapes.glsl:72-81 */
static hit_t combine(int type, hit_t a, hit_t b, pto_counters *ct)
{
    if (type == PTO_TYPE_UNION) {
        if (ct) ct->comb_union++;
        return a.d < b.d ? a : b;
    }
    if (ct) ct->comb_sub++;
    hit_t n = {-a.d, a.mat};
    float depth = gmax(n.d, b.d);
    return depth == n.d ? n : b;
}

/* Union::compile (containers.rs:143-179), Shape::compile (:404-440),
 * UnionType::compile (:244-252): index 0 is a plain assignment. */
static hit_t map_union(const pto_scene *s, int u, const float pp[3], const uint8_t *check, hit_t ref,
                       int type_in, pto_counters *ct)
{
    const onode *o = &s->nd[u];
    hit_t uk = {MAXHIT_D, -1};
    float p[3];
    xform(s, o, pp, p);
    if (ct) ct->xform_union++;
    for (int i = 0; i < o->ncu; i++) uk = map_union(s, o->cu[i], p, check, uk, o->utype, ct);
    for (int i = 0; i < o->ncs; i++) {
        const onode *sh = &s->nd[o->cs[i]];
        int pass = sh->check < 0 ? 1 : (check[sh->check] != 0);
        if (!pass) continue;
        float q[3];
        xform(s, sh, p, q);
        hit_t h = {sdf(s, sh, q), o->cs[i]};
        h.d /= 1.0f / D(sh->slot[SL_SCALE]); /* finalise_scale, data_structures.rs:94-96 */
        if (ct) { ct->xform_shape++; ct->sdf[sh->kind]++; }
        if (i == 0) { uk = h; if (ct) ct->comb_assign++; }
        else uk = combine(o->utype, uk, h, ct);
    }
    uk.d /= 1.0f / D(o->slot[SL_SCALE]);
    return combine(type_in, ref, uk, ct);
}

static hit_t map_ct(const pto_scene *s, const float p[3], const uint8_t *check, pto_counters *ct)
{
    hit_t start = {MAXHIT_D, -1};
    for (int t = 0; t < s->ntop; t++) start = map_union(s, s->top[t], p, check, start, PTO_TYPE_UNION, ct);
    return start;
}

float pto_map(const pto_scene *s, const float p[3], const uint8_t *check, int32_t *shape)
{
    hit_t h = map_ct(s, p, check, NULL);
    if (shape) *shape = h.mat;
    return h.d;
}

/* ------------------------------------------------------------------ */
/* bounds(): generated by Union/Shape/Transform::aabb_compile           */
/* ------------------------------------------------------------------ */
static void bounds_ct(const pto_scene *s, const float ro[3], const float rd[3], uint8_t *check, float dbg[3],
                      pto_counters *ct)
{
    dbg[0] = dbg[1] = dbg[2] = 0.0f;
    memset(check, 0, (size_t)s->ncheck); /* unset entries read as false */
    for (int b = 0; b < s->nbounds; b++) {
        const onode *sh = &s->nd[s->bshape[b]];
        const onode *un = &s->nd[s->bunion[b]];
        if (!sh->aabb) continue; /* `if (false)` */
        if (ct) ct->aabb_tests++;
        /* from_pos_size(upos + spos, (so * (uscale * sscale)) * ex), data_structures.rs:83 */
        float c[3], so[3], hs[3];
        for (int i = 0; i < 3; i++) c[i] = D(un->slot[SL_POS + i]) + D(sh->slot[SL_POS + i]);
        switch (sh->kind) {
        case PTO_SPHERE: case PTO_OCTAHEDRON:
            so[0] = so[1] = so[2] = D(sh->slot[SL_SIZE]); break;
        case PTO_CUBE:
            for (int i = 0; i < 3; i++) so[i] = D(sh->slot[SL_SIZE + i]);
            break;
        case PTO_TORUS: { /* extension: vec3(R + r, r, R + r) */
            float R = D(sh->slot[SL_SIZE]), r = D(sh->slot[SL_SIZE + 1]);
            so[0] = R + r; so[1] = r; so[2] = R + r;
            break;
        }
        default: so[0] = so[1] = so[2] = 1.0f;
        }
        float sc = D(un->slot[SL_SCALE]) * D(sh->slot[SL_SCALE]);
        float ex = D(sh->slot[SL_EX]);
        for (int i = 0; i < 3; i++) hs[i] = (so[i] * sc) * ex;
        /* aabb.glsl:13-33 */
        float tNear = 0, tFar = 0, t1[3], t2[3];
        for (int i = 0; i < 3; i++) {
            float mn = c[i] - hs[i], mx = c[i] + hs[i];
            float tmin = (mn - ro[i]) / rd[i];
            float tmax = (mx - ro[i]) / rd[i];
            t1[i] = gmin(tmin, tmax);
            t2[i] = gmax(tmin, tmax);
        }
        tNear = gmax(gmax(t1[0], t1[1]), t1[2]);
        tFar = gmin(gmin(t2[0], t2[1]), t2[2]);
        if (tNear < tFar && tFar > 0.0f) {
            check[sh->bidx] = 1;
            dbg[0] += 0.1f; dbg[1] += 0.1f; dbg[2] += 0.1f;
        }
    }
}

void pto_bounds(const pto_scene *s, const float ro[3], const float rd[3], uint8_t *check, float debug[3])
{
    bounds_ct(s, ro, rd, check, debug, NULL);
}

/* ------------------------------------------------------------------ */
/* Kernel body: test_compute.glsl:74-246                                */
/* ------------------------------------------------------------------ */
typedef struct { float ro[3], rd[3]; } ray_t;

static void cast_ray(const pto_scene *s, const ray_t *r, const uint8_t *check, float *t_out, int32_t *m_out,
                     pto_counters *ct) /* test_compute.glsl:74-89 */
{
    float t = 0.0f;
    int32_t mat = -1;
    for (int i = 0; i < STEPS; i++) {
        float p[3] = {r->ro[0] + r->rd[0] * t, r->ro[1] + r->rd[1] * t, r->ro[2] + r->rd[2] * t};
        hit_t h = map_ct(s, p, check, ct);
        if (ct) ct->march_steps++;
        mat = h.mat;
        t += h.d;
        if (fabsf(h.d) < MHD) break;
        if (t > FP) { *t_out = t; *m_out = -1; return; }
    }
    *t_out = t;
    *m_out = mat;
}

static void calc_normal(const pto_scene *s, const float p[3], const uint8_t *check, float n[3],
                        pto_counters *ct) /* funcs.glsl:21-35 */
{
    const float e = 0.0001f;
    float v[3];
    for (int a = 0; a < 3; a++) {
        float ep[3] = {0.0f, 0.0f, 0.0f}, en[3] = {-0.0f, -0.0f, -0.0f};
        ep[a] = e; en[a] = -e;
        float qp[3] = {p[0] + ep[0], p[1] + ep[1], p[2] + ep[2]};
        float qn[3] = {p[0] + en[0], p[1] + en[1], p[2] + en[2]};
        float dp = map_ct(s, qp, check, ct).d;
        float dn = map_ct(s, qn, check, ct).d;
        if (ct) ct->normal_maps += 2;
        v[a] = dp - dn;
    }
    normalize3(v, n);
}

typedef struct { float col[3], brightness, light[3], spec, spec_col[3], rough; } mat_t;
static void get_mat(const pto_scene *s, int32_t id, mat_t *m)
{
    if (id < 0) { memset(m, 0, sizeof(*m)); return; } /* MDEF */
    const int32_t *sl = s->nd[id].slot + SL_MAT;
    for (int i = 0; i < 3; i++) { m->col[i] = D(sl[i]); m->light[i] = D(sl[4 + i]); m->spec_col[i] = D(sl[8 + i]); }
    m->brightness = D(sl[3]);
    m->spec = D(sl[7]);
    m->rough = D(sl[11]);
}

/* Optional segment log (analysis aid, single-threaded renders only). */
static pto_segment *g_seglog = NULL;
static int g_seglog_cap = 0, g_seglog_n = 0;
void pto_set_segment_log(pto_segment *buf, int cap) { g_seglog = buf; g_seglog_cap = cap; g_seglog_n = 0; }
int pto_segment_log_count(void) { return g_seglog_n; }

static void path_trace(const pto_scene *s, const pto_settings *st, ray_t ray, uint32_t rng, uint8_t *check,
                       float out[3], pto_counters *ct) /* test_compute.glsl:91-166 */
{
    float ret[3] = {0.0f, 0.0f, 0.0f}, thr[3] = {1.0f, 1.0f, 1.0f};
    int i;
    for (i = 0; i <= st->bounces; i++) {
        float dbg[3];
        bounds_ct(s, ray.ro, ray.rd, check, dbg, ct);
        if (ct) ct->segments++;
        float t;
        int32_t mid;
        uint64_t steps0 = ct ? ct->march_steps : 0;
        cast_ray(s, &ray, check, &t, &mid, ct);
        if (g_seglog && g_seglog_n < g_seglog_cap) {
            pto_segment *sg = &g_seglog[g_seglog_n++];
            for (int k = 0; k < 3; k++) { sg->ro[k] = ray.ro[k]; sg->rd[k] = ray.rd[k]; }
            sg->mask[0] = sg->mask[1] = 0;
            for (int k = 0; k < s->ncheck && k < 128; k++)
                if (check[k]) sg->mask[k >> 6] |= 1ull << (k & 63);
            sg->seg = i;
            sg->steps = ct ? (int32_t)(ct->march_steps - steps0) : -1;
            sg->hit = t <= FP;
        }
        if (t > FP) break;
        float hp[3] = {ray.ro[0] + ray.rd[0] * t, ray.ro[1] + ray.rd[1] * t, ray.ro[2] + ray.rd[2] * t};
        float n[3];
        calc_normal(s, hp, check, n, ct);
        for (int k = 0; k < 3; k++) ray.ro[k] = hp[k] + n[k] * OFFSET;
        if (ct) ct->shaded++;
        mat_t m;
        get_mat(s, mid, &m);
        float spec_chance = m.spec;
        int do_spec = pto_random01(&rng) < spec_chance;
        float ray_prob = do_spec ? spec_chance : 1.0f - spec_chance;
        ray_prob = gmax(ray_prob, 0.0001f);
        float ruv[3], dv[3], diffuse[3];
        random_unit_vector(&rng, ruv);
        for (int k = 0; k < 3; k++) dv[k] = n[k] + ruv[k];
        normalize3(dv, diffuse);
        if (do_spec) {
            float dni = dot3(n, ray.rd); /* reflect(I, N) = I - 2.0 * dot(N, I) * N */
            float kk = 2.0f * dni;
            float sr[3], mx[3];
            for (int k = 0; k < 3; k++) sr[k] = ray.rd[k] - kk * n[k];
            float a = m.rough * m.rough; /* mix(x, y, a) = x * (1 - a) + y * a */
            for (int k = 0; k < 3; k++) mx[k] = sr[k] * (1.0f - a) + diffuse[k] * a;
            normalize3(mx, ray.rd);
        } else {
            for (int k = 0; k < 3; k++) ray.rd[k] = diffuse[k];
        }
        float nl[3];
        normalize3(m.light, nl);
        float fs = (float)do_spec;
        for (int k = 0; k < 3; k++) {
            ret[k] += (nl[k] * m.brightness) * thr[k];
            thr[k] *= m.col[k] * (1.0f - fs) + m.spec_col[k] * fs;
            thr[k] /= ray_prob;
        }
        float p = gmax(thr[0], gmax(thr[1], thr[2]));
        if (pto_random01(&rng) > p) { if (ct) ct->rr_break++; break; }
        float ip = 1.0f / p;
        for (int k = 0; k < 3; k++) thr[k] *= ip;
    }
    if (st->debug == 3) {
        float v = (float)i / (float)st->bounces;
        out[0] = out[1] = out[2] = v;
        return;
    }
    out[0] = ret[0]; out[1] = ret[1]; out[2] = ret[2];
}

static void calc_color(const pto_scene *s, const pto_settings *st, const ray_t *ray, uint32_t rng, uint8_t *check,
                       float out[3], pto_counters *ct) /* test_compute.glsl:170-215 */
{
    if (st->debug == 0 || st->debug == 3) { path_trace(s, st, *ray, rng, check, out, ct); return; }
    if (st->debug == 1) { /* normals() */
        float dbg[3], t;
        int32_t mid;
        bounds_ct(s, ray->ro, ray->rd, check, dbg, ct);
        cast_ray(s, ray, check, &t, &mid, ct);
        if (t > FP) { out[0] = dbg[0]; out[1] = dbg[1]; out[2] = dbg[2]; return; }
        float hp[3] = {ray->ro[0] + ray->rd[0] * t, ray->ro[1] + ray->rd[1] * t, ray->ro[2] + ray->rd[2] * t};
        float n[3], nn[3];
        calc_normal(s, hp, check, n, ct);
        normalize3(n, nn);
        for (int k = 0; k < 3; k++) out[k] = (nn[k] * 0.5f + 0.5f) * 0.2f + dbg[k];
        return;
    }
    if (st->debug == 2) { /* colors() */
        float dbg[3], t;
        int32_t mid;
        bounds_ct(s, ray->ro, ray->rd, check, dbg, ct);
        cast_ray(s, ray, check, &t, &mid, ct);
        mat_t m;
        get_mat(s, mid, &m);
        out[0] = m.col[0]; out[1] = m.col[1]; out[2] = m.col[2];
        return;
    }
    out[0] = out[1] = out[2] = 0.0f;
}

static void render_pixel(const pto_scene *s, const pto_constants *c, const pto_settings *st, int x, int y, int w,
                         int h, int spp, float *px, uint8_t *check, pto_counters *ct) /* test_compute.glsl:218-246 */
{
    for (int j = 0; j < spp; j++) {
        int32_t frame = (int32_t)((uint32_t)c->frame + (uint32_t)j);
        int32_t last_clear = (int32_t)((uint32_t)c->last_clear + (uint32_t)j);
        uint32_t rng = pto_gen_rng(x, y, frame, w, h);
        float jx = pto_random01(&rng), jy = pto_random01(&rng);
        jx = jx - 0.5f;
        jy = jy - 0.5f;
        float ux = ((float)x + jx) / (float)w, uy = ((float)y + jy) / (float)h; /* calc_uv, funcs.glsl:1-7 */
        ux = ux * 2.0f - 1.0f;
        uy = uy * 2.0f - 1.0f;
        ux *= c->aspect;
        ray_t ray = {{0.0f, 0.0f, -3.0f}, {0, 0, 0}};
        float dir[3] = {ux, uy, st->fov};
        normalize3(dir, ray.rd);
        if (ct) ct->samples++;
        float col[3];
        calc_color(s, st, &ray, rng, check, col, ct);
        if (st->debug != 0) {
            px[0] = col[0]; px[1] = col[1]; px[2] = col[2]; px[3] = 1.0f;
            continue;
        }
        float wgt = 1.0f / (float)(last_clear + 1);
        for (int k = 0; k < 3; k++) px[k] = px[k] * (1.0f - wgt) + col[k] * wgt;
        px[3] = 1.0f;
    }
}

typedef struct {
    const pto_scene *s;
    float *image;
    int w, h, spp, rank, nranks, row_stride, tx, ty;
    const pto_constants *c;
    const pto_settings *st;
    int nthreads, tid;
    pto_counters ct;
    int want_ct;
} job_t;

static void *render_worker(void *arg)
{
    job_t *j = (job_t *)arg;
    uint8_t *check = (uint8_t *)calloc((size_t)j->s->ncheck + 1, 1);
    int ntiles = j->tx * j->ty;
    int k = 0;
    for (int t = 0; t < ntiles; t++) {
        if (t % j->nranks != j->rank) continue;
        if ((k++ % j->nthreads) != j->tid) continue;
        int bx = (t % j->tx) * 8, by = (t / j->tx) * 8;
        for (int y = by; y < by + 8 && y < j->h; y++) {
            if (y % j->row_stride != 0) continue;
            for (int x = bx; x < bx + 8 && x < j->w; x++)
                render_pixel(j->s, j->c, j->st, x, y, j->w, j->h, j->spp, j->image + ((size_t)y * j->w + x) * 4, check,
                             j->want_ct ? &j->ct : NULL);
        }
    }
    free(check);
    return NULL;
}

void pto_render(const pto_scene *s, float *image, int w, int h, const pto_constants *c, const pto_settings *st,
                int spp, int rank, int nranks, int row_stride, int nthreads, pto_counters *counters)
{
    if (nthreads <= 0) nthreads = 1;
    if (nranks <= 0) nranks = 1;
    if (row_stride <= 0) row_stride = 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; i++) {
        job_t *j = &jobs[i];
        j->s = s; j->image = image; j->w = w; j->h = h; j->spp = spp; j->rank = rank; j->nranks = nranks;
        j->row_stride = row_stride; j->tx = (w + 7) / 8; j->ty = (h + 7) / 8; j->c = c; j->st = st;
        j->nthreads = nthreads; j->tid = i; j->want_ct = counters != NULL;
        if (nthreads == 1) render_worker(j);
        else pthread_create(&th[i], NULL, render_worker, j);
    }
    if (nthreads > 1)
        for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    if (counters) {
        memset(counters, 0, sizeof(*counters));
        uint64_t *dst = (uint64_t *)counters;
        for (int i = 0; i < nthreads; i++) {
            const uint64_t *src = (const uint64_t *)&jobs[i].ct;
            for (size_t k = 0; k < sizeof(pto_counters) / sizeof(uint64_t); k++) dst[k] += src[k];
        }
    }
    free(jobs);
    free(th);
}

/* ---- display pass (render_texture_shader.wgsl:23-94) --------------------- */
/* pow(x, y), x > 0: log2 by frexp + 2*atanh series on [sqrt(1/2), sqrt(2)),
 * exp2 by rounding off the integer part + Taylor series of e^(f ln 2),
 * all in double with fma, rounded once to f32 (DESIGN.md display contract). */
static double d_log2(double x)
{
    int e = 0;
    double m = frexp(x, &e) * 2.0, s, s2, p;
    static const double inv_odd[12] = {1.0 / 23.0, 1.0 / 21.0, 1.0 / 19.0, 1.0 / 17.0, 1.0 / 15.0, 1.0 / 13.0,
                                       1.0 / 11.0, 1.0 / 9.0,  1.0 / 7.0,  1.0 / 5.0,  1.0 / 3.0,  1.0};
    e -= 1;
    if (m > 1.4142135623730951) {
        m *= 0.5;
        e += 1;
    }
    s = (m - 1.0) / (m + 1.0);
    s2 = s * s;
    p = inv_odd[0];
    for (int k = 1; k < 12; ++k) p = fma(p, s2, inv_odd[k]);
    return (double)e + ((2.0 * s) * p) * 1.4426950408889634;
}

static double d_exp2(double t)
{
    static const double inv_fact[14] = {1.0 / 6227020800.0, 1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0,
                                        1.0 / 362880.0,     1.0 / 40320.0,     1.0 / 5040.0,     1.0 / 720.0,
                                        1.0 / 120.0,        1.0 / 24.0,        1.0 / 6.0,        0.5,
                                        1.0,                1.0};
    const double k = floor(t + 0.5), z = (t - k) * 0.6931471805599453;
    double p = inv_fact[0];
    for (int i = 1; i < 14; ++i) p = fma(p, z, inv_fact[i]);
    return ldexp(p, (int)k);
}

float pto_pow_pos(float x, float y)
{
    if (!(x > 0.0f)) return 0.0f;
    return (float)d_exp2((double)y * d_log2((double)x));
}

static float lin_to_srgb(float v)
{
    const float c = gclamp(v, 0.0f, 1.0f);
    const float a = pto_pow_pos(c, (float)(1.0 / 2.4)) * 1.055f - 0.055f;
    const float b = c * 12.92f;
    const float t = c < 0.0031308f ? 1.0f : 0.0f;
    return a * (1.0f - t) + b * t;
}

static float aces(float x)
{
    const float n = x * (2.51f * x + 0.03f), d = x * (2.43f * x + 0.59f) + 0.14f;
    return gclamp(n / d, 0.0f, 1.0f);
}

static float fs_channel(float x) { return lin_to_srgb(aces(x * 1.0f)); }

void pto_display(const float *image, int w, int h, int fmt, void *out)
{
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            if (fmt == 0) {
                const float *t = image + ((size_t)y * w + x) * 4;
                float *o = (float *)out + ((size_t)y * w + x) * 4;
                o[0] = fs_channel(t[0]);
                o[1] = fs_channel(t[1]);
                o[2] = fs_channel(t[2]);
                o[3] = 1.0f;
            } else {
                const float *t = image + ((size_t)(h - 1 - y) * w + x) * 4;
                uint8_t *o = (uint8_t *)out + ((size_t)y * w + x) * 4;
                for (int k = 0; k < 3; ++k) o[k] = (uint8_t)rintf(lin_to_srgb(fs_channel(t[k])) * 255.0f);
                o[3] = 255;
            }
        }
}
