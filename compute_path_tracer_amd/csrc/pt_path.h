// pt_path.h -- the per-lane path arithmetic of the state-machine kernels
// (pt_wave.h: tile-resident wavefront, pt_binned.h: mask-binned passes).
// One definition of each step, so both schedules compute every sample with
// the same f32 operations as pt_kernel.hip's reference-structured loop and
// the oracle.
#pragma once

#include "pt_common.h"

namespace pt {

enum : int { ST_FREE = 0, ST_BOUNDS = 1, ST_MARCH = 2, ST_NORMAL = 3, ST_SHADE = 4 };

// Camera ray of pixel (x, y) in frame `frame`: gen_rng, sub-pixel jitter,
// calc_uv and the pinhole camera (test_compute.glsl:224-235).
__device__ __forceinline__ void camera_ray(int x, int y, int32_t frame, int width, int height, float aspect, float fov,
                                           uint32_t &rng, pt_f3 &ro, pt_f3 &rd) {
    rng = pt_gen_rng(x, y, frame, width, height);
    float jx = pt_random01(rng);
    float jy = pt_random01(rng);
    jx = jx - 0.5f;
    jy = jy - 0.5f;
    float ux = (float(x) + jx) / float(width), uy = (float(y) + jy) / float(height);
    ux = ux * 2.0f - 1.0f;
    uy = uy * 2.0f - 1.0f;
    ux *= aspect;
    rd = pt_normalize(pt_f3{ux, uy, fov});
    ro = pt_f3{0.0f, 0.0f, -3.0f};
}

// bounds(): one box's slab test, intersectAABB + bool_hit (aabb.glsl:21-33),
// as the generated bounds() applies it per check[] entry.
__device__ __forceinline__ bool ray_box(const PtAabb &bx, float ox, float oy, float oz, float dx, float dy, float dz) {
    const float tminx = (bx.bmin[0] - ox) / dx, tmaxx = (bx.bmax[0] - ox) / dx;
    const float tminy = (bx.bmin[1] - oy) / dy, tmaxy = (bx.bmax[1] - oy) / dy;
    const float tminz = (bx.bmin[2] - oz) / dz, tmaxz = (bx.bmax[2] - oz) / dz;
    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
    return tnear < tfar && tfar > 0.0f;
}

// The same test with the divisions as pt_div_rcp from per-ray reciprocals
// (y = RN(1/d)); bit-identical results when the pt_div_*_ok guards hold for
// the ray and the box (bounds_fast in pt_binned.h).
__device__ __forceinline__ bool ray_box_rcp(const PtAabb &bx, float ox, float oy, float oz, float dx, float dy,
                                            float dz, float yx, float yy, float yz) {
    const float tminx = pt_div_rcp(bx.bmin[0] - ox, dx, yx), tmaxx = pt_div_rcp(bx.bmax[0] - ox, dx, yx);
    const float tminy = pt_div_rcp(bx.bmin[1] - oy, dy, yy), tmaxy = pt_div_rcp(bx.bmax[1] - oy, dy, yy);
    const float tminz = pt_div_rcp(bx.bmin[2] - oz, dz, yz), tmaxz = pt_div_rcp(bx.bmax[2] - oz, dz, yz);
    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
    return tnear < tfar && tfar > 0.0f;
}

// The slab test from the reciprocal products alone: t' = RN(a * y) with a =
// RN(bmin - o) as in ray_box_rcp and y = RN(1/d).  Under the same guards,
// |t' - t| <= 3 * 2^-24 |t| for every slab value t = RN(a / d), and t' has
// t's sign and zeros, so:
//  * tfar' > 0 exactly when tfar > 0 (min / max keep the signs);
//  * tnear < tfar is decided by tnear' < tfar' whenever |tfar' - tnear'| >
//    2^-20 (|tnear'| + |tfar'|) (min / max move each end by <= 2^-22 of
//    itself); `gap` keeps the least |tfar' - tnear'| - that margin over the
//    boxes tested, and a lane whose gap is <= 0 takes ray_box_rcp.
__device__ __forceinline__ bool ray_box_approx(const PtAabb &bx, float ox, float oy, float oz, float yx, float yy,
                                               float yz, float &gap) {
    const float tminx = (bx.bmin[0] - ox) * yx, tmaxx = (bx.bmax[0] - ox) * yx;
    const float tminy = (bx.bmin[1] - oy) * yy, tmaxy = (bx.bmax[1] - oy) * yy;
    const float tminz = (bx.bmin[2] - oz) * yz, tmaxz = (bx.bmax[2] - oz) * yz;
    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
    gap = fminf(gap, fabsf(tfar - tnear) - (fabsf(tnear) + fabsf(tfar)) * 0x1p-20f);
    return tnear < tfar && tfar > 0.0f;
}

// ray_box_approx with the margin in units of the last place (DESIGN.md
// 3.19): each slab value t' is within 4 representable steps of the IEEE slab
// value (3 roundings of <= 2^-24 relative each), with the same sign and
// zeros, so min / max keep tnear' and tfar' within 4 steps of the IEEE tnear
// and tfar, and tnear' < tfar' decides tnear < tfar whenever the two bit
// patterns differ by more than 8 (opposite signs differ by >= 2^31 and are
// decided by the signs).  `gapu` keeps the least |bits(tfar') -
// bits(tnear')| (v_sad_u32: one instruction, against four for the float
// margin); a lane whose gapu is <= PT_ULP_MARGIN takes ray_box_rcp.
#define PT_ULP_MARGIN 16u
// (SAD false: max - min, for loops the compiler is to unroll -- inline asm is
// convergent, which blocks a runtime-count unroll)
template <bool SAD = true>
__device__ __forceinline__ uint32_t pt_absdiff_u32(uint32_t a, uint32_t b) {
    if constexpr (!SAD) return max(a, b) - min(a, b);
    uint32_t d;
    __asm__("v_sad_u32 %0, %1, %2, 0" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
template <bool SAD = true>
__device__ __forceinline__ bool ray_box_ulp(const PtAabb &bx, float ox, float oy, float oz, float yx, float yy,
                                            float yz, uint32_t &gapu) {
    const float tminx = (bx.bmin[0] - ox) * yx, tmaxx = (bx.bmax[0] - ox) * yx;
    const float tminy = (bx.bmin[1] - oy) * yy, tmaxy = (bx.bmax[1] - oy) * yy;
    const float tminz = (bx.bmin[2] - oz) * yz, tmaxz = (bx.bmax[2] - oz) * yz;
    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
    gapu = min(gapu, pt_absdiff_u32<SAD>(__float_as_uint(tfar), __float_as_uint(tnear)));
    return tnear < tfar && tfar > 0.0f;
}

// The slab test from one fma per slab: t' = RN(b * y + n) with n = -RN(o * y)
// per ray and axis, y = RN(1/d).  Under the guards of ray_box_rcp,
// |t' - t| <= 2^-21 |t| + 2^-23 M for every slab value t = RN(RN(b - o) / d),
// M = max over the axes of |n| (the product's rounding adds an absolute
// term: DESIGN.md 3.18).  `gap` as in ray_box_approx and `tfa` (the least
// |tfar'|) decide a lane when gap > 2^-21 M and tfa > 2^-22 M (fma_decided);
// an undecided lane takes ray_box_rcp.  One fma per slab instead of a
// subtraction and a product.
__device__ __forceinline__ bool ray_box_fma(const PtAabb &bx, float nx, float ny, float nz, float yx, float yy,
                                            float yz, float &gap, float &tfa) {
    const float tminx = fmaf(bx.bmin[0], yx, nx), tmaxx = fmaf(bx.bmax[0], yx, nx);
    const float tminy = fmaf(bx.bmin[1], yy, ny), tmaxy = fmaf(bx.bmax[1], yy, ny);
    const float tminz = fmaf(bx.bmin[2], yz, nz), tmaxz = fmaf(bx.bmax[2], yz, nz);
    const float tnear = pt_gmax(pt_gmax(pt_gmin(tminx, tmaxx), pt_gmin(tminy, tmaxy)), pt_gmin(tminz, tmaxz));
    const float tfar = pt_gmin(pt_gmin(pt_gmax(tminx, tmaxx), pt_gmax(tminy, tmaxy)), pt_gmax(tminz, tmaxz));
    gap = fminf(gap, fabsf(tfar - tnear) - (fabsf(tnear) + fabsf(tfar)) * 0x1p-20f);
    tfa = fminf(tfa, fabsf(tfar));
    return tnear < tfar && tfar > 0.0f;
}
__device__ __forceinline__ bool fma_decided(float gap, float tfa, float nx, float ny, float nz) {
    const float m = pt_gmax(fabsf(nx), pt_gmax(fabsf(ny), fabsf(nz)));
    return gap > m * 0x1p-21f && tfa > m * 0x1p-22f;
}

// The map() argument of a lane: CastRay's p = ro + rd*t (MARCH), or normal
// tap `step` (0..5 = +x,-x,+y,-y,+z,-z) around the hit point held in ro
// (calc_normal, test_compute.glsl:57-66).
__device__ __forceinline__ void map_point(int state, int step, const pt_f3 &ro, const pt_f3 &rd, float t, float &qx,
                                          float &qy, float &qz) {
    if (state == ST_MARCH) {
        qx = ro.x + rd.x * t;
        qy = ro.y + rd.y * t;
        qz = ro.z + rd.z * t;
    } else {
        const float e = 0.0001f;
        const int axis = step >> 1;
        const bool neg = (step & 1) != 0;
        const float on = neg ? -e : e, off = neg ? -0.0f : 0.0f;
        qx = ro.x + (axis == 0 ? on : off);
        qy = ro.y + (axis == 1 ? on : off);
        qz = ro.z + (axis == 2 ? on : off);
    }
}

// Advance a MARCH / NORMAL lane by the map() result h.  MARCH: CastRay's loop
// body and exit tests (test_compute.glsl:42-54); on exit either a miss
// (-> SHADE with step = -1) or calc_point into ro (-> NORMAL).  NORMAL: the
// six taps give the central differences d(p+e) - d(p-e) per axis.
// MARCH_ONLY: the caller never maps a NORMAL lane (the binned trace pass
// whose shade pass takes the taps), so the taps' branch is left out.
template <bool ST, bool MARCH_ONLY = false>
__device__ __forceinline__ void after_map(const Hit &h, int &state, int &step, float &t, pt_f3 &ro, const pt_f3 &rd,
                                          int &mat, float &dv0, float &dv1, float &dv2, Stats<ST> &st) {
    if (MARCH_ONLY || state == ST_MARCH) {
        st.add(PT_ST_MARCH);
        mat = h.m;
        t += h.d;
        ++step;
        if (fabsf(h.d) < kMhd || t > kFp || step == kSteps) {
            if (t > kFp) {
                state = ST_SHADE;  // miss: path ends
                step = -1;
            } else {
                ro = pt_f3{ro.x + rd.x * t, ro.y + rd.y * t, ro.z + rd.z * t};  // calc_point
                state = ST_NORMAL;
                step = 0;
            }
        }
    } else if constexpr (!MARCH_ONLY) {
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

// Upper bound on map() at every calc_normal tap of a hit:
// the march's last map() value was d at point q (t: the ray parameter after
// t += d), the hit point is |d| further along the ray and each tap e = 1e-4
// from it.  map() is 1-Lipschitz (a min/max/assign composition of exact SDFs
// under rotations, scales and translations) up to the rotation constants'
// rounding (x(1 + 2^-16)); mg covers the f32 rounding of the two evaluations
// and of the point arithmetic: a few tens of ulp of |q|_1 + |d| + t + bk,
// bk = the scene's transform-chain magnitude (pt_bound_k; NaN: no bound).
__device__ __forceinline__ float tap_bound(float d, float qx, float qy, float qz, float t, float bk) {
    const float ad = fabsf(d);
    const float mg = 0x1p-10f * (fabsf(qx) + fabsf(qy) + fabsf(qz) + ad + fabsf(t) + bk);
    return ((d + ad) * 0x1.0001p+0f + mg) + 0x1.a38p-14f;  // + e = 1e-4 (x(1 + 2^-16), rounded up)
}

// Shading of a hit and Russian roulette (test_compute.glsl:116-159).
// Returns true when the path ends here (miss: step < 0, roulette, or the
// bounce limit); otherwise ro/rd/thr hold the next segment's ray and seg was
// incremented.
template <bool ST>
__device__ __forceinline__ bool shade_lane(const PtMat *__restrict__ mats, int bounces, int mat, float dv0, float dv1,
                                           float dv2, int step, uint32_t &rng, pt_f3 &ro, pt_f3 &rd, pt_f3 &thr,
                                           pt_f3 &ret, int &seg, Stats<ST> &st) {
    if (step < 0) return true;  // miss
    const pt_f3 n = pt_normalize(pt_f3{dv0, dv1, dv2});
    const pt_f3 hp = ro;
    ro = pt_f3{hp.x + n.x * kOffset, hp.y + n.y * kOffset, hp.z + n.z * kOffset};
    st.add(PT_ST_SHADED);
    const PtMat &m = mats[mat];
    const float spec_chance = m.spec;
    const bool do_spec = pt_random01(rng) < spec_chance;
    float ray_prob = do_spec ? spec_chance : 1.0f - spec_chance;
    ray_prob = pt_gmax(ray_prob, 0.0001f);
    const float uz = pt_random01(rng) * 2.0f - 1.0f;
    const float ua = pt_random01(rng) * kPi2;
    const float ur = pt_sqrt(1.0f - uz * uz);
    float sa, ca;
    pt_sincos(ua, sa, ca);
    const pt_f3 diffuse = pt_normalize(pt_f3{n.x + ur * ca, n.y + ur * sa, n.z + uz});
    if (do_spec) {
        const float k = 2.0f * pt_dot(n, rd);
        const pt_f3 sr{rd.x - k * n.x, rd.y - k * n.y, rd.z - k * n.z};
        const float al = m.rough2, oma = 1.0f - al;
        rd = pt_normalize(pt_f3{sr.x * oma + diffuse.x * al, sr.y * oma + diffuse.y * al, sr.z * oma + diffuse.z * al});
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
        return true;
    }
    const float ip = 1.0f / pmax;
    thr.x *= ip;
    thr.y *= ip;
    thr.z *= ip;
    ++seg;
    return seg > bounces;
}

// The sample's colour once its path ended (debug 3: bounce count, :163).
__device__ __forceinline__ pt_f3 final_color(int debug, int seg, int bounces, const pt_f3 &ret) {
    if (debug == 3) {
        const float v = float(seg) / float(bounces);
        return pt_f3{v, v, v};
    }
    return ret;
}

}  // namespace pt
