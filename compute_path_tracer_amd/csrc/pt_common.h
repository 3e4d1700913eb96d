// pt_common.h -- device building blocks shared by the ahead-of-time kernels
// (pt_kernel.hip) and the per-scene kernels compiled at run time with hipRTC
// (pt_jit.cpp).  One definition of every f32 expression, so the AOT
// interpreter, the JIT-specialised map() and the oracle stay bit-identical.
#pragma once

#include "pt_device.h"
#include "pt_math.h"

namespace pt {

constexpr int kSteps = 80;           // test_compute.glsl:26 STEPS
constexpr float kMhd = 0.001f;       // :28 MHD
constexpr float kFp = 100.0f;        // :29 FP
constexpr float kOffset = 0.03f;     // :30 OFFSET
constexpr float kPi = 3.14159265359f;
constexpr float kPi2 = 2.0f * kPi;   // :37-38
constexpr float kMaxHit = 10000.0f;  // sdf_editor.rs:193 MAXHIT

// Scene tables are read wave-uniformly: address space 4 (constant) makes the
// compiler fetch them with scalar loads (s_load) into SGPRs.  (The host pass
// of a HIP translation unit never runs these functions.)
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
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

struct Check {  // check[] of the generated bounds(), one bit per entry
    uint64_t lo, hi;
    // a superset of the check[] bits of every lane of the wave that maps with
    // this mask, wave-uniform (scene kernels test it first: a shape no lane
    // needs is skipped by a scalar branch); all ones = no information
    uint64_t alo = ~0ull, ahi = ~0ull;
};
// a lane's check[] bit behind the wave-uniform test of Check.alo/ahi: the
// empty volatile asm keeps the compiler from merging the two tests into one
// vector test (it may not speculate a block with side effects), so the
// uniform one stays a scalar branch
__device__ __forceinline__ bool lane_check(uint64_t m, int k) {
    __asm__ volatile("");
    return ((m >> k) & 1ull) != 0;
}
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
    // wave clock for the per-phase cycle counters (instrumented kernel only)
    __device__ __forceinline__ uint64_t clk() const {
        if constexpr (ST) return __builtin_readcyclecounter();
        return 0;
    }
    // charge the cycles since `t` to slot k (lane 0 only), return the new mark
    __device__ __forceinline__ uint64_t lap(int k, uint64_t t) {
        if constexpr (ST) {
            const uint64_t now = __builtin_readcyclecounter();
            if ((threadIdx.x & 63) == 0) c[k] += uint32_t(now - t);
            return now;
        }
        return 0;
    }
};

// OR of v over the 64 lanes of the wave (every lane active), wave-uniform:
// an inclusive row scan by DPP row shifts, then the rows' totals by row
// broadcasts; lane 63 holds the OR of all 64 lanes
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));  // row_shr:1
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));  // row_shr:2
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));  // row_shr:4
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));  // row_shr:8
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
    v |= uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
    return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}
__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
    return uint64_t(wave_or_u32(uint32_t(v))) | (uint64_t(wave_or_u32(uint32_t(v >> 32))) << 32);
}
// min / max of v over the 64 lanes (every lane active; a lane that must not
// count passes the identity, +inf / -inf), wave-uniform: the same scan as
// fused v_min / v_max_f32_dpp.  A lane without a source lane (row edge,
// bound_ctrl off) is not written and keeps its value.  Two wait states before
// each step (a VALU write read by the next DPP), which the compiler cannot
// see inside the asm.  (The builtin form, update_dpp + min with the identity
// shifted in, compiled to three instructions per step: the first pass's
// kernel 25.5 vs 24.9 ms per launch, profiles/r05i_*.)
#define PT_WRED_ASM(op, v)                                                                          \
    __asm__ volatile("s_nop 1\n\t" op "_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"     \
                     "s_nop 1\n\t" op "_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"     \
                     "s_nop 1\n\t" op "_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"     \
                     "s_nop 1\n\t" op "_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"     \
                     "s_nop 1\n\t" op "_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"  \
                     "s_nop 1\n\t" op "_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"  \
                     "s_nop 1"                                                                      \
                     : "+v"(v))
__device__ __forceinline__ float wave_min_f32(float v) {
    PT_WRED_ASM("v_min_f32", v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_max_f32(float v) {
    PT_WRED_ASM("v_max_f32", v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ int lane_rank(uint64_t m) {  // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

// Transform::compile (data_structures.rs:45-55) with hoisted constants:
// p *= 1/s; p = p - pos*(1/s); p = rotZ*(rotY*(rotX*p)) (shapes.glsl:34-68,
// column-major constructors).  Identity factors (flag bit clear) are skipped;
// skipping is exact up to the sign of zero, which no SDF can observe.
template <uint32_t F>
__device__ __forceinline__ void xform_f(const PtNode &n, float &x, float &y, float &z) {
    if constexpr ((F & PT_NF_SCALE) != 0) {
        x = x * n.inv;
        y = y * n.inv;
        z = z * n.inv;
    }
    if constexpr ((F & PT_NF_POS) != 0) {
        x = x - n.m[0];
        y = y - n.m[1];
        z = z - n.m[2];
    }
    if constexpr ((F & PT_NF_RX) != 0) {
        const float ny = n.cx * y + n.sx * z;
        const float nz = (-n.sx) * y + n.cx * z;
        y = ny;
        z = nz;
    }
    if constexpr ((F & PT_NF_RY) != 0) {
        const float nx = n.cy * x + (-n.sy) * z;
        const float nz = n.sy * x + n.cy * z;
        x = nx;
        z = nz;
    }
    if constexpr ((F & PT_NF_RZ) != 0) {
        const float nx = n.cz * x + n.sz * y;
        const float ny = (-n.sz) * x + n.cz * y;
        x = nx;
        y = ny;
    }
}
// runtime-flag form (interpreter)
__device__ __forceinline__ void xform(const PtNode &n, float &x, float &y, float &z) {
    const uint32_t f = n.flags;
    if (f & PT_NF_SCALE) xform_f<PT_NF_SCALE>(n, x, y, z);
    if (f & PT_NF_POS) xform_f<PT_NF_POS>(n, x, y, z);
    if (f & PT_NF_RX) xform_f<PT_NF_RX>(n, x, y, z);
    if (f & PT_NF_RY) xform_f<PT_NF_RY>(n, x, y, z);
    if (f & PT_NF_RZ) xform_f<PT_NF_RZ>(n, x, y, z);
}

// sdCube (shapes.glsl:5-9) from q = abs(p) - b and qm = max(q): the
// bound-culled scene map computes q first for its test.
//
// FAST (scene kernels, cubes whose faces are large next to the scene): when
// at most one of mx, my, mz is nonzero (their median is 0) and that one, m,
// is 0 or in [2^-60, 2^60], the sum of squares is RN(m^2) (the other terms
// are +0) and sqrt(RN(m^2)) = m exactly (binary RN; checked for every
// significand), so length(max(q, 0)) = m without the squares and the sqrt.
// A wave takes that path when all its active lanes qualify.
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
// max(x, 0), min(x, 0), max3 and med3 as the bare instructions.  fmaxf's
// IEEE-mode lowering first quiets each operand produced in another basic
// block (one `v_max_f32 v, v, v` each; the cube's q comes from before the
// cull branch).  No operand here is a signalling NaN, and for the rest (quiet
// NaN included: the other operand) the instructions return fmaxf's / fminf's
// / fmed3's values (DESIGN.md 5 history, round 3).
__device__ __forceinline__ float pt_max0(float x) {
    float r;
    __asm__("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ float pt_min0(float x) {
    float r;
    __asm__("v_min_f32 %0, 0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ float pt_max3v(float a, float b, float c) {
    float r;
    __asm__("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float pt_med3v(float a, float b, float c) {
    float r;
    __asm__("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
#define PT_BARE_MINMAX 1
#else
__device__ __forceinline__ float pt_max0(float x) { return pt_gmax(x, 0.0f); }
__device__ __forceinline__ float pt_min0(float x) { return pt_gmin(x, 0.0f); }
#endif
template <bool FAST = false>
__device__ __forceinline__ float cube_from_q(float qx, float qy, float qz, float qm) {
#if defined(PT_BARE_MINMAX)
    // (no bare instruction inside a branch: clang marks inline asm convergent,
    // which kept the ballot's branch from folding into the compares)
    const float mx = pt_max0(qx), my = pt_max0(qy), mz = pt_max0(qz), mq = pt_min0(qm);
    if constexpr (FAST) {
        const float m = pt_max3v(mx, my, mz);
        const bool easy = pt_med3v(mx, my, mz) == 0.0f &&
                          (m == 0.0f || __builtin_amdgcn_fmed3f(m, 0x1p-60f, 0x1p60f) == m);
        if (__ballot(!easy) == 0ull) return m + mq;
    }
    return pt_sqrt(mx * mx + my * my + mz * mz) + mq;
#else  // host
    const float mx = pt_gmax(qx, 0.0f), my = pt_gmax(qy, 0.0f), mz = pt_gmax(qz, 0.0f);
    return pt_sqrt(mx * mx + my * my + mz * mz) + pt_gmin(qm, 0.0f);
#endif
}

// cull target: the smaller of the parent's running distance a and the
// point's map() bound b; a NaN bound leaves a
__device__ __forceinline__ float cull_target(float a, float b) { return b < a ? b : a; }

// SDFs, shapes.glsl:1-25 (+ torus extension)
template <int K, bool FASTCUBE = false>
__device__ __forceinline__ float sdf_k(const PtNode &n, float x, float y, float z) {
    if constexpr (K == PT_NODE_SPHERE) {
        return pt_sqrt(x * x + y * y + z * z) - n.size[0];
    } else if constexpr (K == PT_NODE_CUBE) {
        const float qx = fabsf(x) - n.size[0], qy = fabsf(y) - n.size[1], qz = fabsf(z) - n.size[2];
        return cube_from_q<FASTCUBE>(qx, qy, qz, pt_gmax(qx, pt_gmax(qy, qz)));
    } else if constexpr (K == PT_NODE_TORUS) {
        const float qx = pt_sqrt(x * x + z * z) - n.size[0];
        return pt_sqrt(qx * qx + y * y) - n.size[1];
    } else {  // PT_NODE_OCTAHEDRON
        const float s = n.size[0];
        const float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
        const float m = ax + ay + az - s;
        float q0, q1, q2;
        if (3.0f * ax < m) {
            q0 = ax; q1 = ay; q2 = az;
        } else if (3.0f * ay < m) {
            q0 = ay; q1 = az; q2 = ax;
        } else if (3.0f * az < m) {
            q0 = az; q1 = ax; q2 = ay;
        } else {
            return m * 0.57735027f;
        }
        const float k = pt_gmin(pt_gmax(0.5f * (q2 - q1 + s), 0.0f), s);
        const float vy = q1 - s + k, vz = q2 - k;
        return pt_sqrt(q0 * q0 + vy * vy + vz * vz);
    }
}
__device__ __forceinline__ float sdf(const PtNode &n, float x, float y, float z) {
    switch (n.shape) {
        case PT_NODE_SPHERE: return sdf_k<PT_NODE_SPHERE>(n, x, y, z);
        case PT_NODE_CUBE: return sdf_k<PT_NODE_CUBE>(n, x, y, z);
        case PT_NODE_TORUS: return sdf_k<PT_NODE_TORUS>(n, x, y, z);
        case PT_NODE_OCTAHEDRON: return sdf_k<PT_NODE_OCTAHEDRON>(n, x, y, z);
        default: return 0.0f;
    }
}

// opUnion / opSubtraction (shapes.glsl:72-81); ASSIGN = index-0 shape.
template <int C>
__device__ __forceinline__ Hit combine_c(Hit a, Hit b) {
    if constexpr (C == PT_COMBINE_ASSIGN) {
        return b;
    } else if constexpr (C == PT_COMBINE_UNION) {
        return a.d < b.d ? a : b;
    } else {
        const Hit n{-a.d, a.m};
        const float depth = pt_gmax(n.d, b.d);
        return depth == n.d ? n : b;
    }
}
__device__ __forceinline__ Hit combine(int32_t how, Hit a, Hit b) {
    if (how == PT_COMBINE_ASSIGN) return combine_c<PT_COMBINE_ASSIGN>(a, b);
    if (how == PT_COMBINE_UNION) return combine_c<PT_COMBINE_UNION>(a, b);
    return combine_c<PT_COMBINE_SUBTRACTION>(a, b);
}

// lane-0-of-the-active-set bookkeeping for wave-level counters
__device__ __forceinline__ bool first_active_lane() {
    return __builtin_amdgcn_readfirstlane(int(threadIdx.x)) == int(threadIdx.x);
}

template <bool ST>
__device__ __forceinline__ void count_shape(Stats<ST> &st, int shape, int how) {
    if constexpr (ST)
        if (first_active_lane()) st.add(PT_ST_WAVE_SHAPES);
    st.add(PT_ST_XFORM_SHAPE);
    st.add(PT_ST_SDF_SPHERE + (shape - PT_NODE_SPHERE));
    st.add(how == PT_COMBINE_ASSIGN ? PT_ST_COMB_ASSIGN : (how == PT_COMBINE_UNION ? PT_ST_COMB_UNION : PT_ST_COMB_SUB));
}

template <bool ST>
__device__ __forceinline__ void count_eval(Stats<ST> &st) {
    if constexpr (ST)
        if (first_active_lane()) st.add(PT_ST_WAVE_EVALS);
}

// The generated map() (sdf_editor.rs:192-210) interpreted from the op list.
// Depth 0 is the `start` accumulator, depth 1 a header union; deeper nesting
// spills to a private stack (scratch) that flat scenes never touch.
struct InterpMap {
    template <bool ST>
    static __device__ Hit eval(const PtLaunch &L, float qx, float qy, float qz, const Check &ck, float /*bnd*/,
                               float /*bndw*/, uint64_t & /*live*/, Stats<ST> &st) {
        Hit cur{kMaxHit, 0};
        Hit s0{kMaxHit, 0};
        float px = qx, py = qy, pz = qz;
        int depth = 0;
        float stk[PT_MAX_DEPTH][5];
        cnode_ptr nodes = (cnode_ptr)L.nodes;
        for (int i = 0; i < L.n_nodes; ++i) {
            const PtNode n = nodes[i];
            if (n.op == PT_OP_SHAPE) {
                const bool pass = n.check < 0 || check_bit(ck, n.check);
                if (pass) {
                    float x = px, y = py, z = pz;
                    xform(n, x, y, z);
                    float d = sdf(n, x, y, z);
                    if (n.flags & PT_NF_SCALE) d = d / n.inv;  // finalise_scale: d /= 1.0 / s
                    cur = combine(n.combine, cur, Hit{d, n.mat});
                    count_shape(st, n.shape, n.combine);
                    count_eval(st);
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
                const Hit h{d, cur.m};
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
};

// (base: PT_ST_COUNT for the second half, the shade pass's normal taps)
template <bool ST>
__device__ __forceinline__ void flush_stats(const PtLaunch &L, Stats<ST> &st, int base = 0) {
    if constexpr (ST) {
        for (int k = 0; k < PT_ST_COUNT; ++k) {
            unsigned long long v = st.c[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if ((threadIdx.x & 63) == 0) atomicAdd(&L.stats[base + k], v);
        }
    }
}

}  // namespace pt
