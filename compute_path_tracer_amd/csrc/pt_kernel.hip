// pt_kernel.hip -- the SDF sphere-trace + Monte-Carlo path-trace hot path for
// CDNA4 (gfx950).  Restates assets/shaders/path_tracer/test_compute.glsl
// (+ rng/funcs/shapes/aabb.glsl and the scene code SDFEditor::compile emits)
// under the semantics contract of DESIGN.md section 3.
//
// Geometry: one workgroup = one wave64 = one 8x8 pixel tile; lane = pixel.
// A launch renders `spp` successive frames per pixel with the accumulation
// texel held in registers, so the image costs one 16 B load + one 16 B store
// per pixel per launch instead of per frame (test_compute.glsl:242-245).
// The scene program is interpreted wave-uniformly: every node record is read
// with scalar loads; only the per-lane AABB mask (check[]) predicates work.
#include "pt_device.h"
#include "pt_math.h"

namespace {

constexpr int kSteps = 80;         // test_compute.glsl:26 STEPS
constexpr float kMhd = 0.001f;     // :28 MHD
constexpr float kFp = 100.0f;      // :29 FP
constexpr float kOffset = 0.03f;   // :30 OFFSET
constexpr float kPi = 3.14159265359f;
constexpr float kPi2 = 2.0f * kPi;  // :37-38
constexpr float kMaxHit = 10000.0f;  // sdf_editor.rs:193

// Scene tables are read wave-uniformly: address space 4 (constant) makes the
// compiler fetch them with scalar loads (s_load) into SGPRs.
// (The host pass of this translation unit never runs these functions.)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const PtNode *cnode_ptr;
typedef __attribute__((address_space(4))) const PtAabb *caabb_ptr;
#else
typedef const PtNode *cnode_ptr;
typedef const PtAabb *caabb_ptr;
#endif

struct Hit {
    float d;
    int32_t m;  // material index, 0 = MDEF
};

struct Check {
    uint64_t lo, hi;
};
__device__ __forceinline__ bool check_bit(const Check &c, int k) {
    return k < 64 ? ((c.lo >> k) & 1ull) != 0 : ((c.hi >> (k - 64)) & 1ull) != 0;
}

template <bool ST>
struct Stats {
    uint32_t c[PT_ST_COUNT];
    __device__ __forceinline__ void init() {
        if constexpr (ST)
            for (int i = 0; i < PT_ST_COUNT; ++i) c[i] = 0;
    }
    __device__ __forceinline__ void add(int k, uint32_t v = 1) {
        if constexpr (ST) c[k] += v;
    }
};

// Transform::compile (data_structures.rs:45-55) with hoisted constants:
// p *= 1/s; p = p - pos*(1/s); p = rotZ*(rotY*(rotX*p)) (shapes.glsl:34-68,
// column-major constructors).  Identity factors are skipped; skipping them is
// exact up to the sign of zero, which no SDF below can observe.
__device__ __forceinline__ void xform(const PtNode &n, float &x, float &y, float &z) {
    const uint32_t f = n.flags;
    if (f & PT_NF_SCALE) {
        x = x * n.inv;
        y = y * n.inv;
        z = z * n.inv;
    }
    if (f & PT_NF_POS) {
        x = x - n.m[0];
        y = y - n.m[1];
        z = z - n.m[2];
    }
    if (f & PT_NF_RX) {
        float ny = n.cx * y + n.sx * z;
        float nz = (-n.sx) * y + n.cx * z;
        y = ny;
        z = nz;
    }
    if (f & PT_NF_RY) {
        float nx = n.cy * x + (-n.sy) * z;
        float nz = n.sy * x + n.cy * z;
        x = nx;
        z = nz;
    }
    if (f & PT_NF_RZ) {
        float nx = n.cz * x + n.sz * y;
        float ny = (-n.sz) * x + n.cz * y;
        x = nx;
        y = ny;
    }
}

// shapes.glsl:1-25 (+ torus extension)
__device__ __forceinline__ float sdf(const PtNode &n, float x, float y, float z) {
    switch (n.shape) {
        case PT_NODE_SPHERE: return sqrtf(x * x + y * y + z * z) - n.size[0];
        case PT_NODE_CUBE: {
            float qx = fabsf(x) - n.size[0], qy = fabsf(y) - n.size[1], qz = fabsf(z) - n.size[2];
            float mx = pt_gmax(qx, 0.0f), my = pt_gmax(qy, 0.0f), mz = pt_gmax(qz, 0.0f);
            return sqrtf(mx * mx + my * my + mz * mz) + pt_gmin(pt_gmax(qx, pt_gmax(qy, qz)), 0.0f);
        }
        case PT_NODE_TORUS: {
            float qx = sqrtf(x * x + z * z) - n.size[0];
            return sqrtf(qx * qx + y * y) - n.size[1];
        }
        case PT_NODE_OCTAHEDRON: {
            const float s = n.size[0];
            float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
            float m = ax + ay + az - s;
            float q0, q1, q2;
            if (3.0f * ax < m) { q0 = ax; q1 = ay; q2 = az; }
            else if (3.0f * ay < m) { q0 = ay; q1 = az; q2 = ax; }
            else if (3.0f * az < m) { q0 = az; q1 = ax; q2 = ay; }
            else return m * 0.57735027f;
            float k = pt_gmin(pt_gmax(0.5f * (q2 - q1 + s), 0.0f), s);
            float vy = q1 - s + k, vz = q2 - k;
            return sqrtf(q0 * q0 + vy * vy + vz * vz);
        }
        default: return 0.0f;
    }
}

// opUnion / opSubtraction (shapes.glsl:72-81); ASSIGN = index-0 shape.
__device__ __forceinline__ Hit combine(int32_t how, Hit a, Hit b) {
    if (how == PT_COMBINE_ASSIGN) return b;
    if (how == PT_COMBINE_UNION) return a.d < b.d ? a : b;
    Hit n{-a.d, a.m};
    float depth = pt_gmax(n.d, b.d);
    return depth == n.d ? n : b;
}

// The generated map() (sdf_editor.rs:192-210), interpreted.  Depth 0 is the
// `start` accumulator, depth 1 a header union; deeper nesting spills to a
// private stack (scratch) that flat scenes never touch.
template <bool ST>
__device__ Hit scene_map(const PtLaunch &L, float qx, float qy, float qz, const Check &ck, Stats<ST> &st) {
    Hit cur{kMaxHit, 0};
    Hit s0{kMaxHit, 0};
    float px = qx, py = qy, pz = qz;
    int depth = 0;
    float stk[PT_MAX_DEPTH][5];
    cnode_ptr nodes = (cnode_ptr)L.nodes;
    for (int i = 0; i < L.n_nodes; ++i) {
        const PtNode n = nodes[i];
        if (n.op == PT_OP_SHAPE) {
            bool pass = n.check < 0 || check_bit(ck, n.check);
            if (pass) {
                float x = px, y = py, z = pz;
                xform(n, x, y, z);
                float d = sdf(n, x, y, z);
                if (n.flags & PT_NF_SCALE) d = d / n.inv;  // finalise_scale: d /= 1.0 / s
                cur = combine(n.combine, cur, Hit{d, n.mat});
                st.add(PT_ST_XFORM_SHAPE);
                st.add(PT_ST_SDF_SPHERE + (n.shape - PT_NODE_SPHERE));
                st.add(n.combine == PT_COMBINE_ASSIGN ? PT_ST_COMB_ASSIGN
                                                      : (n.combine == PT_COMBINE_UNION ? PT_ST_COMB_UNION : PT_ST_COMB_SUB));
            }
        } else if (n.op == PT_OP_UNION_BEGIN) {
            if (depth == 0) {
                s0 = cur;
            } else {
                stk[depth - 1][0] = px;
                stk[depth - 1][1] = py;
                stk[depth - 1][2] = pz;
                stk[depth - 1][3] = cur.d;
                stk[depth - 1][4] = __int_as_float(cur.m);
            }
            ++depth;
            xform(n, px, py, pz);
            cur = Hit{kMaxHit, 0};
            st.add(PT_ST_XFORM_UNION);
        } else {  // PT_OP_UNION_END
            float d = cur.d;
            if (n.flags & PT_NF_SCALE) d = d / n.inv;
            Hit h{d, cur.m};
            --depth;
            if (depth == 0) {
                cur = s0;
                px = qx;
                py = qy;
                pz = qz;
            } else {
                px = stk[depth - 1][0];
                py = stk[depth - 1][1];
                pz = stk[depth - 1][2];
                cur = Hit{stk[depth - 1][3], __float_as_int(stk[depth - 1][4])};
            }
            cur = combine(n.combine, cur, h);
            st.add(n.combine == PT_COMBINE_UNION ? PT_ST_COMB_UNION : PT_ST_COMB_SUB);
        }
    }
    return cur;
}

// bounds() generated by the aabb_compile functions (containers.rs:181-202,
// 442-463; aabb.glsl:21-33).  Returns the per-lane check mask and the debug
// tint (debug += 0.1 per hit box).
template <bool ST>
__device__ Check bounds(const PtLaunch &L, pt_f3 ro, pt_f3 rd, float &tint, Stats<ST> &st) {
    Check c{0ull, 0ull};
    tint = 0.0f;
    caabb_ptr boxes = (caabb_ptr)L.aabbs;
    for (int a = 0; a < L.n_aabb; ++a) {
        const PtAabb b = boxes[a];
        float tminx = (b.bmin[0] - ro.x) / rd.x, tmaxx = (b.bmax[0] - ro.x) / rd.x;
        float tminy = (b.bmin[1] - ro.y) / rd.y, tmaxy = (b.bmax[1] - ro.y) / rd.y;
        float tminz = (b.bmin[2] - ro.z) / rd.z, tmaxz = (b.bmax[2] - ro.z) / rd.z;
        float t1x = pt_gmin(tminx, tmaxx), t2x = pt_gmax(tminx, tmaxx);
        float t1y = pt_gmin(tminy, tmaxy), t2y = pt_gmax(tminy, tmaxy);
        float t1z = pt_gmin(tminz, tmaxz), t2z = pt_gmax(tminz, tmaxz);
        float tnear = pt_gmax(pt_gmax(t1x, t1y), t1z);
        float tfar = pt_gmin(pt_gmin(t2x, t2y), t2z);
        st.add(PT_ST_AABB);
        if (tnear < tfar && tfar > 0.0f) {
            const int k = b.back;
            if (k < 64) c.lo |= 1ull << k;
            else c.hi |= 1ull << (k - 64);
            tint += 0.1f;
        }
    }
    return c;
}

// CastRay (test_compute.glsl:74-89): returns t (> FP means miss) and material.
template <bool ST>
__device__ __noinline__ Hit cast_ray(const PtLaunch &L, pt_f3 ro, pt_f3 rd, const Check &ck, Stats<ST> &st) {
    float t = 0.0f;
    int32_t mat = 0;
    for (int i = 0; i < kSteps; ++i) {
        Hit h = scene_map<ST>(L, ro.x + rd.x * t, ro.y + rd.y * t, ro.z + rd.z * t, ck, st);
        st.add(PT_ST_MARCH);
        mat = h.m;
        t += h.d;
        if (fabsf(h.d) < kMhd) break;
        if (t > kFp) return Hit{t, 0};
    }
    return Hit{t, mat};
}

// calc_normal (funcs.glsl:21-35): central differences, e = 1e-4, the six
// taps p + e.xyy, p - e.xyy, p + e.yxy, ... in that order; the zero
// components of -e are -0.0 (so p.y + (-0.0) == p.y exactly).
template <bool ST>
__device__ __noinline__ pt_f3 calc_normal(const PtLaunch &L, pt_f3 p, const Check &ck, Stats<ST> &st) {
    const float e = 0.0001f;
    float dv[3];
    float dplus = 0.0f;
#pragma unroll 1
    for (int k = 0; k < 6; ++k) {
        const int axis = k >> 1;
        const bool neg = (k & 1) != 0;
        const float on = neg ? -e : e, off = neg ? -0.0f : 0.0f;
        const float qx = p.x + (axis == 0 ? on : off);
        const float qy = p.y + (axis == 1 ? on : off);
        const float qz = p.z + (axis == 2 ? on : off);
        const float d = scene_map<ST>(L, qx, qy, qz, ck, st).d;
        if (!neg) dplus = d;
        else dv[axis] = dplus - d;
    }
    st.add(PT_ST_NORMAL_MAPS, 6);
    return pt_normalize(pt_f3{dv[0], dv[1], dv[2]});
}

// path_trace (test_compute.glsl:91-166)
template <bool ST>
__device__ pt_f3 path_trace(const PtLaunch &L, pt_f3 ro, pt_f3 rd, uint32_t rng, Stats<ST> &st) {
    pt_f3 ret{0.0f, 0.0f, 0.0f}, thr{1.0f, 1.0f, 1.0f};
    int i;
    for (i = 0; i <= L.bounces; ++i) {
        float tint;
        Check ck = bounds<ST>(L, ro, rd, tint, st);
        st.add(PT_ST_SEGMENTS);
        Hit hit = cast_ray<ST>(L, ro, rd, ck, st);
        if (hit.d > kFp) break;
        pt_f3 hp{ro.x + rd.x * hit.d, ro.y + rd.y * hit.d, ro.z + rd.z * hit.d};
        pt_f3 n = calc_normal<ST>(L, hp, ck, st);
        ro = pt_f3{hp.x + n.x * kOffset, hp.y + n.y * kOffset, hp.z + n.z * kOffset};
        st.add(PT_ST_SHADED);
        const PtMat &m = L.mats[hit.m];
        const float spec_chance = m.spec;
        const bool do_spec = pt_random01(rng) < spec_chance;
        float ray_prob = do_spec ? spec_chance : 1.0f - spec_chance;
        ray_prob = pt_gmax(ray_prob, 0.0001f);
        // RandomUnitVector (rng.glsl:16-24)
        float uz = pt_random01(rng) * 2.0f - 1.0f;
        float ua = pt_random01(rng) * kPi2;
        float ur = sqrtf(1.0f - uz * uz);
        float sa, ca;
        pt_sincos(ua, sa, ca);
        pt_f3 diffuse = pt_normalize(pt_f3{n.x + ur * ca, n.y + ur * sa, n.z + uz});
        if (do_spec) {
            float k = 2.0f * pt_dot(n, rd);  // reflect(I, N) = I - 2 * dot(N, I) * N
            pt_f3 sr{rd.x - k * n.x, rd.y - k * n.y, rd.z - k * n.z};
            float a = m.rough2, oma = 1.0f - a;  // mix(x, y, a) = x * (1 - a) + y * a
            rd = pt_normalize(pt_f3{sr.x * oma + diffuse.x * a, sr.y * oma + diffuse.y * a, sr.z * oma + diffuse.z * a});
        } else {
            rd = diffuse;
        }
        const float fs = do_spec ? 1.0f : 0.0f, omf = 1.0f - fs;
        ret.x += m.emis[0] * thr.x;
        ret.y += m.emis[1] * thr.y;
        ret.z += m.emis[2] * thr.z;
        thr.x *= m.col[0] * omf + m.spec_col[0] * fs;
        thr.y *= m.col[1] * omf + m.spec_col[1] * fs;
        thr.z *= m.col[2] * omf + m.spec_col[2] * fs;
        thr.x /= ray_prob;
        thr.y /= ray_prob;
        thr.z /= ray_prob;
        // Russian roulette (:152-159)
        float p = pt_gmax(thr.x, pt_gmax(thr.y, thr.z));
        if (pt_random01(rng) > p) {
            st.add(PT_ST_RR_BREAK);
            break;
        }
        float ip = 1.0f / p;
        thr.x *= ip;
        thr.y *= ip;
        thr.z *= ip;
    }
    if (L.debug == 3) {
        float v = float(i) / float(L.bounces);
        return pt_f3{v, v, v};
    }
    return ret;
}

// calc_color (test_compute.glsl:199-215) with normals() :170-179, colors() :183-195
template <bool ST>
__device__ pt_f3 calc_color(const PtLaunch &L, pt_f3 ro, pt_f3 rd, uint32_t rng, Stats<ST> &st) {
    if (L.debug == 0 || L.debug == 3) return path_trace<ST>(L, ro, rd, rng, st);
    if (L.debug == 1 || L.debug == 2) {
        float tint;
        Check ck = bounds<ST>(L, ro, rd, tint, st);
        Hit hit = cast_ray<ST>(L, ro, rd, ck, st);
        if (L.debug == 2) {
            const PtMat &m = L.mats[hit.m];
            return pt_f3{m.col[0], m.col[1], m.col[2]};
        }
        if (hit.d > kFp) return pt_f3{tint, tint, tint};
        pt_f3 hp{ro.x + rd.x * hit.d, ro.y + rd.y * hit.d, ro.z + rd.z * hit.d};
        pt_f3 n = pt_normalize(calc_normal<ST>(L, hp, ck, st));
        return pt_f3{(n.x * 0.5f + 0.5f) * 0.2f + tint, (n.y * 0.5f + 0.5f) * 0.2f + tint,
                     (n.z * 0.5f + 0.5f) * 0.2f + tint};
    }
    return pt_f3{0.0f, 0.0f, 0.0f};
}

template <bool ST>
__device__ __forceinline__ void flush_stats(const PtLaunch &L, Stats<ST> &st) {
    if constexpr (ST) {
        for (int k = 0; k < PT_ST_COUNT; ++k) {
            unsigned long long v = st.c[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if ((threadIdx.x & 63) == 0) atomicAdd(&L.stats[k], v);
        }
    }
}

}  // namespace

// main (test_compute.glsl:218-246), `spp` frames per launch.
template <bool ST>
__global__ __launch_bounds__(64) void pt_render_kernel(PtLaunch L) {
    const int g = L.rank + int(blockIdx.x) * L.nranks;  // cyclic tile ownership
    const int tx = g % L.tiles_x, ty = g / L.tiles_x;
    const int lane = int(threadIdx.x);
    const int x = tx * PT_TILE + (lane & 7), y = ty * PT_TILE + (lane >> 3);
    Stats<ST> st;
    st.init();
    const bool inside = x < L.width && y < L.height;  // bounds_check uses '>' upstream; OOB texel ops are dropped there
    if (inside) {
        float *texel = L.accum + (size_t(y) * size_t(L.width) + size_t(x)) * 4;
        float ar = 0.0f, ag = 0.0f, ab = 0.0f;
        if (L.debug == 0 && L.write) {
            float4 v = *reinterpret_cast<const float4 *>(texel);
            ar = v.x;
            ag = v.y;
            ab = v.z;
        }
        const int j0 = L.debug != 0 ? L.spp - 1 : 0;  // direct stores: only the last frame survives
        for (int j = j0; j < L.spp; ++j) {
            const int32_t frame = int32_t(uint32_t(L.frame0) + uint32_t(j));
            const int32_t last_clear = int32_t(uint32_t(L.last_clear0) + uint32_t(j));
            uint32_t rng = pt_gen_rng(x, y, frame, L.width, L.height);
            float jx = pt_random01(rng);
            float jy = pt_random01(rng);
            jx = jx - 0.5f;
            jy = jy - 0.5f;
            float ux = (float(x) + jx) / float(L.width), uy = (float(y) + jy) / float(L.height);  // calc_uv
            ux = ux * 2.0f - 1.0f;
            uy = uy * 2.0f - 1.0f;
            ux *= L.aspect;
            pt_f3 rd = pt_normalize(pt_f3{ux, uy, L.fov});
            st.add(PT_ST_SAMPLES);
            pt_f3 col = calc_color<ST>(L, pt_f3{0.0f, 0.0f, -3.0f}, rd, rng, st);
            if (L.debug != 0) {
                ar = col.x;
                ag = col.y;
                ab = col.z;
            } else {
                const float w = 1.0f / float(last_clear + 1), omw = 1.0f - w;  // mix(last, col, w)
                ar = ar * omw + col.x * w;
                ag = ag * omw + col.y * w;
                ab = ab * omw + col.z * w;
            }
        }
        if (L.write) *reinterpret_cast<float4 *>(texel) = make_float4(ar, ag, ab, 1.0f);
    }
    flush_stats<ST>(L, st);
}

template __global__ void pt_render_kernel<false>(PtLaunch);
template __global__ void pt_render_kernel<true>(PtLaunch);

// ---------------------------------------------------------------------------
// Wavefront kernel.  Same per-sample arithmetic as pt_render_kernel, different
// schedule: each lane runs a state machine and every loop iteration performs
// exactly one map() for every lane that is marching or taking a normal tap,
// so march-length, bounce-count and Russian-roulette divergence no longer
// idle lanes.  The tile's V pixels x spp frames form a job pool; a lane whose
// path ends takes the next job (wave ballot + prefix count).  Finished samples
// land in an LDS ring (PT_RING slots per pixel) and the pixel's owner lane
// folds them in frame order, so the accumulation is bit-identical to the
// reference's frame-by-frame mix (test_compute.glsl:242-245).  bounds() is
// redistributed: the (ray, box) slab tests of all lanes that start a segment
// are spread over the 64 lanes, one pair per lane per pass.
// ---------------------------------------------------------------------------
namespace {

enum : int { ST_FREE = 0, ST_BOUNDS = 1, ST_MARCH = 2, ST_NORMAL = 3, ST_SHADE = 4 };

struct WaveLds {
    float col[PT_RING][3][64];
    uint8_t ready[PT_RING][64];
    int folded[64];
    uint32_t mask[64][4];
    int list[64];
    int valid[64];
};

__device__ __forceinline__ int lane_rank(uint64_t m) {  // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

}  // namespace

template <bool ST>
__global__ __launch_bounds__(64) void pt_wave_kernel(PtLaunch L) {
    __shared__ WaveLds S;
    const int lane = int(threadIdx.x);
    const int g = L.rank + int(blockIdx.x) * L.nranks;
    const int tx0 = (g % L.tiles_x) * PT_TILE, ty0 = (g / L.tiles_x) * PT_TILE;
    Stats<ST> st;
    st.init();

    // pixels of this tile inside the image, compacted (edge tiles are ragged)
    const int my_x = tx0 + (lane & 7), my_y = ty0 + (lane >> 3);
    const bool inside = my_x < L.width && my_y < L.height;
    const uint64_t vmask = __ballot(inside);
    const int V = __popcll(vmask);
    const int vidx = lane_rank(vmask);
    if (inside) S.valid[vidx] = lane;
    S.folded[lane] = 0;
#pragma unroll
    for (int r = 0; r < PT_RING; ++r) S.ready[r][lane] = 0;

    // debug 3 stores the last frame only; debug 0 folds every frame
    const int j0 = L.debug != 0 ? L.spp - 1 : 0;
    const int nsmp = L.spp - j0;
    float ar = 0.0f, ag = 0.0f, ab = 0.0f;
    float *texel = L.accum + (size_t(my_y) * size_t(L.width) + size_t(my_x)) * 4;
    if (inside && L.debug == 0 && L.write) {
        const float4 v = *reinterpret_cast<const float4 *>(texel);
        ar = v.x;
        ag = v.y;
        ab = v.z;
    }
    int folded = 0;
    __syncthreads();

    // q / V for small q by multiply-high (exact for q < 2^16)
    const uint32_t vmagic = V > 0 ? uint32_t((0x100000000ull + uint64_t(V) - 1) / uint64_t(V)) : 0u;
    // bounds redistribution: (lane / n_aabb, lane % n_aabb) and the per-pass step
    const int nbox = L.n_aabb;
    const int la = nbox > 0 ? lane / nbox : 0, lb = nbox > 0 ? lane % nbox : 0;
    const int da = nbox > 0 ? 64 / nbox : 0, db = nbox > 0 ? 64 % nbox : 0;
    const PtAabb *__restrict__ boxes = L.aabbs;
    const int shade_batch = L.shade_batch > 0 ? L.shade_batch : 1;

    const int total = V * nsmp;
    int next_p = 0, next_s = 0, issued = 0;  // wave-uniform issue cursor

    // per-lane path state
    int state = ST_FREE;
    int jp = 0, js = 0;              // job: pixel slot, frame index
    uint32_t rng = 0;
    pt_f3 ro{0.0f, 0.0f, 0.0f}, rd{0.0f, 0.0f, 1.0f};
    pt_f3 thr{1.0f, 1.0f, 1.0f}, ret{0.0f, 0.0f, 0.0f};
    int seg = 0, step = 0, mat = 0;
    float t = 0.0f;
    float dv0 = 0.0f, dv1 = 0.0f, dv2 = 0.0f;
    Check ck{0ull, 0ull};

    for (;;) {
        // ---- 1. refill free lanes from the job pool (in job order) -------
        const uint64_t freem = __ballot(state == ST_FREE);
        if (freem != 0ull && issued < total) {
            const int r = lane_rank(freem);
            const uint32_t q = uint32_t(next_p + r);
            const int wrap = int(__umulhi(q, vmagic));
            const int p = int(q) - wrap * V;
            const int s = next_s + wrap;
            const bool cand = state == ST_FREE && issued + r < total;
            const bool ok = cand && s < S.folded[p] + PT_RING;
            const uint64_t candm = __ballot(cand), bad = candm & ~__ballot(ok);
            int n = __popcll(candm);
            if (bad != 0ull) {
                const int first_bad = __builtin_ctzll(bad);
                n = __popcll(freem & ((1ull << first_bad) - 1ull));
            }
            if (cand && r < n) {
                jp = p;
                js = s;
                const int lp = S.valid[p];
                const int x = tx0 + (lp & 7), y = ty0 + (lp >> 3);
                const int32_t frame = int32_t(uint32_t(L.frame0) + uint32_t(j0 + s));
                rng = pt_gen_rng(x, y, frame, L.width, L.height);
                float jx = pt_random01(rng);
                float jy = pt_random01(rng);
                jx = jx - 0.5f;
                jy = jy - 0.5f;
                float ux = (float(x) + jx) / float(L.width), uy = (float(y) + jy) / float(L.height);
                ux = ux * 2.0f - 1.0f;
                uy = uy * 2.0f - 1.0f;
                ux *= L.aspect;
                rd = pt_normalize(pt_f3{ux, uy, L.fov});
                ro = pt_f3{0.0f, 0.0f, -3.0f};
                thr = pt_f3{1.0f, 1.0f, 1.0f};
                ret = pt_f3{0.0f, 0.0f, 0.0f};
                seg = 0;
                state = ST_BOUNDS;
                st.add(PT_ST_SAMPLES);
            }
            // advance the cursor by n jobs
            const uint32_t qn = uint32_t(next_p + n);
            const int wn = int(__umulhi(qn, vmagic));
            next_p = int(qn) - wn * V;
            next_s += wn;
            issued += n;
        }

        // ---- 2. bounds() for lanes starting a segment, (ray, box) pairs ---
        const uint64_t needm = __ballot(state == ST_BOUNDS);
        if (needm != 0ull) {
            if (state == ST_BOUNDS) {
                S.list[lane_rank(needm)] = lane;
                S.mask[lane][0] = S.mask[lane][1] = S.mask[lane][2] = S.mask[lane][3] = 0u;
                st.add(PT_ST_SEGMENTS);
            }
            __syncthreads();
            const int pairs = __popcll(needm) * nbox;
            int a = la, b = lb;
            for (int base = 0; base < pairs; base += 64) {
                const bool act = base + lane < pairs;
                const int src = act ? S.list[a] : lane;
                const float ox = __shfl(ro.x, src, 64), oy = __shfl(ro.y, src, 64), oz = __shfl(ro.z, src, 64);
                const float dx = __shfl(rd.x, src, 64), dy = __shfl(rd.y, src, 64), dz = __shfl(rd.z, src, 64);
                if (act) {
                    const PtAabb bx = boxes[b];
                    const float tminx = (bx.bmin[0] - ox) / dx, tmaxx = (bx.bmax[0] - ox) / dx;
                    const float tminy = (bx.bmin[1] - oy) / dy, tmaxy = (bx.bmax[1] - oy) / dy;
                    const float tminz = (bx.bmin[2] - oz) / dz, tmaxz = (bx.bmax[2] - oz) / dz;
                    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
                    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
                    st.add(PT_ST_AABB);
                    if (tnear < tfar && tfar > 0.0f) atomicOr(&S.mask[src][bx.back >> 5], 1u << (bx.back & 31));
                }
                a += da;
                b += db;
                if (b >= nbox) {
                    b -= nbox;
                    a += 1;
                }
            }
            __syncthreads();
            if (state == ST_BOUNDS) {
                ck.lo = uint64_t(S.mask[lane][0]) | (uint64_t(S.mask[lane][1]) << 32);
                ck.hi = uint64_t(S.mask[lane][2]) | (uint64_t(S.mask[lane][3]) << 32);
                t = 0.0f;
                step = 0;
                state = ST_MARCH;
            }
        }

        // ---- 3. one map() per marching / normal-tap lane ---------------------
        const bool mapping = state == ST_MARCH || state == ST_NORMAL;
        if (__ballot(mapping) != 0ull) {
            if (mapping) {
                float qx, qy, qz;
                if (state == ST_MARCH) {  // CastRay: p = ro + rd * t
                    qx = ro.x + rd.x * t;
                    qy = ro.y + rd.y * t;
                    qz = ro.z + rd.z * t;
                } else {  // calc_normal tap `step` around hit point (held in ro)
                    const float e = 0.0001f;
                    const int axis = step >> 1;
                    const bool neg = (step & 1) != 0;
                    const float on = neg ? -e : e, off = neg ? -0.0f : 0.0f;
                    qx = ro.x + (axis == 0 ? on : off);
                    qy = ro.y + (axis == 1 ? on : off);
                    qz = ro.z + (axis == 2 ? on : off);
                }
                const Hit h = scene_map<ST>(L, qx, qy, qz, ck, st);
                // ---- 4. advance the state machine ------------------------------
                if (state == ST_MARCH) {
                    st.add(PT_ST_MARCH);
                    mat = h.m;
                    t += h.d;
                    ++step;
                    if (fabsf(h.d) < kMhd || t > kFp || step == kSteps) {
                        if (t > kFp) {
                            state = ST_SHADE;  // miss: path ends (seg stays)
                            step = -1;
                        } else {
                            ro = pt_f3{ro.x + rd.x * t, ro.y + rd.y * t, ro.z + rd.z * t};  // calc_point
                            state = ST_NORMAL;
                            step = 0;
                        }
                    }
                } else {
                    if ((step & 1) == 0) {
                        t = h.d;  // d(p + e)
                    } else {
                        const float dd = t - h.d;
                        if (step == 1) dv0 = dd;
                        else if (step == 3) dv1 = dd;
                        else dv2 = dd;
                    }
                    ++step;
                    if (step == 6) {
                        st.add(PT_ST_NORMAL_MAPS, 6);
                        state = ST_SHADE;
                    }
                }
            }
        }

        // ---- 5. shading (batched) and path completion ----------------------
        const uint64_t shadem = __ballot(state == ST_SHADE);
        if (shadem != 0ull &&
            (__popcll(shadem) >= shade_batch || __ballot(state == ST_MARCH || state == ST_NORMAL) == 0ull ||
             issued >= total)) {
            if (state == ST_SHADE) {
                bool done = step < 0;  // miss
                if (!done) {
                    const pt_f3 n = pt_normalize(pt_f3{dv0, dv1, dv2});
                    const pt_f3 hp = ro;
                    ro = pt_f3{hp.x + n.x * kOffset, hp.y + n.y * kOffset, hp.z + n.z * kOffset};
                    st.add(PT_ST_SHADED);
                    const PtMat &m = L.mats[mat];
                    const float spec_chance = m.spec;
                    const bool do_spec = pt_random01(rng) < spec_chance;
                    float ray_prob = do_spec ? spec_chance : 1.0f - spec_chance;
                    ray_prob = pt_gmax(ray_prob, 0.0001f);
                    const float uz = pt_random01(rng) * 2.0f - 1.0f;
                    const float ua = pt_random01(rng) * kPi2;
                    const float ur = sqrtf(1.0f - uz * uz);
                    float sa, ca;
                    pt_sincos(ua, sa, ca);
                    const pt_f3 diffuse = pt_normalize(pt_f3{n.x + ur * ca, n.y + ur * sa, n.z + uz});
                    if (do_spec) {
                        const float k = 2.0f * pt_dot(n, rd);
                        const pt_f3 sr{rd.x - k * n.x, rd.y - k * n.y, rd.z - k * n.z};
                        const float al = m.rough2, oma = 1.0f - al;
                        rd = pt_normalize(pt_f3{sr.x * oma + diffuse.x * al, sr.y * oma + diffuse.y * al,
                                                sr.z * oma + diffuse.z * al});
                    } else {
                        rd = diffuse;
                    }
                    const float fs = do_spec ? 1.0f : 0.0f, omf = 1.0f - fs;
                    ret.x += m.emis[0] * thr.x;
                    ret.y += m.emis[1] * thr.y;
                    ret.z += m.emis[2] * thr.z;
                    thr.x *= m.col[0] * omf + m.spec_col[0] * fs;
                    thr.y *= m.col[1] * omf + m.spec_col[1] * fs;
                    thr.z *= m.col[2] * omf + m.spec_col[2] * fs;
                    thr.x /= ray_prob;
                    thr.y /= ray_prob;
                    thr.z /= ray_prob;
                    const float pmax = pt_gmax(thr.x, pt_gmax(thr.y, thr.z));
                    if (pt_random01(rng) > pmax) {
                        st.add(PT_ST_RR_BREAK);
                        done = true;
                    } else {
                        const float ip = 1.0f / pmax;
                        thr.x *= ip;
                        thr.y *= ip;
                        thr.z *= ip;
                        ++seg;
                        if (seg > L.bounces) done = true;
                        else state = ST_BOUNDS;
                    }
                }
                if (done) {
                    pt_f3 c = ret;
                    if (L.debug == 3) {
                        const float v = float(seg) / float(L.bounces);
                        c = pt_f3{v, v, v};
                    }
                    const int slot = js & (PT_RING - 1);
                    S.col[slot][0][jp] = c.x;
                    S.col[slot][1][jp] = c.y;
                    S.col[slot][2][jp] = c.z;
                    S.ready[slot][jp] = 1;
                    state = ST_FREE;
                }
            }
            __syncthreads();
            // ---- 6. owners fold finished frames in order --------------------
            if (inside) {
                for (;;) {
                    const int slot = folded & (PT_RING - 1);
                    if (folded >= nsmp || S.ready[slot][vidx] == 0) break;
                    const float cr = S.col[slot][0][vidx], cg = S.col[slot][1][vidx], cb = S.col[slot][2][vidx];
                    if (L.debug != 0) {
                        ar = cr;
                        ag = cg;
                        ab = cb;
                    } else {
                        const int32_t lc = int32_t(uint32_t(L.last_clear0) + uint32_t(j0 + folded));
                        const float w = 1.0f / float(lc + 1), omw = 1.0f - w;
                        ar = ar * omw + cr * w;
                        ag = ag * omw + cg * w;
                        ab = ab * omw + cb * w;
                    }
                    S.ready[slot][vidx] = 0;
                    ++folded;
                }
                S.folded[vidx] = folded;
            }
            __syncthreads();
        }

        if (issued >= total && __ballot(state != ST_FREE) == 0ull) break;
    }
    if (inside && L.write) *reinterpret_cast<float4 *>(texel) = make_float4(ar, ag, ab, 1.0f);
    flush_stats<ST>(L, st);
}

template __global__ void pt_wave_kernel<false>(PtLaunch);
template __global__ void pt_wave_kernel<true>(PtLaunch);

void pt_launch_render(const PtLaunch &L, bool stats, hipStream_t stream) {
    dim3 grid(unsigned(L.n_tiles)), block(64);
    const bool simple = L.kernel == PT_KERNEL_SIMPLE || L.debug == 1 || L.debug == 2;
    if (simple) {
        if (stats) hipLaunchKernelGGL(pt_render_kernel<true>, grid, block, 0, stream, L);
        else hipLaunchKernelGGL(pt_render_kernel<false>, grid, block, 0, stream, L);
    } else {
        if (stats) hipLaunchKernelGGL(pt_wave_kernel<true>, grid, block, 0, stream, L);
        else hipLaunchKernelGGL(pt_wave_kernel<false>, grid, block, 0, stream, L);
    }
}
