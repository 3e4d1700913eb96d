// pt_math.h -- f32 helpers shared by the HIP kernel and the host-side scene
// derivation in pt_runtime.hip.  Compiled with -ffp-contract=off on both
// sides: every fused multiply-add is an explicit fmaf.
//
// The GLSL builtins' precision is left to the driver by the spec (naga +
// vendor driver upstream, parity unpinned there); this file is the semantics
// contract of DESIGN.md section 3 that makes host and device agree bitwise.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#else  // hipRTC (per-scene JIT, pt_jit.cpp): no std headers
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::size_t size_t;
#endif

#define PT_HD __host__ __device__ __forceinline__

// GLSL min/max/clamp.  naga lowers them to SPIR-V GLSL.std.450 FMin/FMax/
// FClamp, which GPU drivers implement with the hardware min/max; on gfx950
// that is v_min_f32/v_max_f32 = IEEE-754 minNum/maxNum (a NaN operand yields
// the other operand; -0 < +0).  The contract adopts exactly
// that; oracle/pt_oracle.c spells it out bit for bit and the device self-test
// (pt_selftest) checks the hardware against it.
PT_HD float pt_gmin(float x, float y) { return fminf(x, y); }
PT_HD float pt_gmax(float x, float y) { return fmaxf(x, y); }

// rng.glsl:1-9
PT_HD uint32_t pt_wang_hash(uint32_t &seed) {
    seed = (seed ^ 61u) ^ (seed >> 16);
    seed *= 9u;
    seed = seed ^ (seed >> 4);
    seed *= 0x27d4eb2du;
    seed = seed ^ (seed >> 15);
    return seed;
}
// rng.glsl:11-14: float(u) / 2^32 (exact scaling of the RN conversion)
PT_HD float pt_random01(uint32_t &state) { return float(pt_wang_hash(state)) * 2.3283064365386963e-10f; }

// rng.glsl:26-36
PT_HD uint32_t pt_gen_rng(int32_t x, int32_t y, int32_t frame, int32_t w, int32_t h) {
    uint32_t a = uint32_t((float(x) * 0.5f + 0.5f) * float(w));
    uint32_t b = uint32_t((float(y) * 0.5f + 0.5f) * float(h));
    return (a * 1973u + b * 9277u + uint32_t(frame) * 26699u) | 1u;
}

// sin/cos contract: Cody-Waite reduction by pi/2 + minimax polynomials on
// [-pi/4, pi/4]; identical to oracle/pt_oracle.c:sincos_q.
PT_HD float pt_sin_poly(float r) {
    float s = r * r;
    float p = fmaf(s, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(s, p, -1.6666654611e-1f);
    return fmaf(r * s, p, r);
}
PT_HD float pt_cos_poly(float r) {
    float s = r * r;
    float p = fmaf(s, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(s, p, 4.166664568298827e-2f);
    float t = fmaf(s, p, -0.5f);
    return fmaf(s, t, 1.0f);
}
// Reduced argument and quadrant of x (|x| <= 2^24; callers map the rest to NaN).
PT_HD float pt_reduce(float x, int &q) {
    float k = rintf(x * 0.63661977236758134f);
    float r = fmaf(-k, 1.5703125f, x);
    r = fmaf(-k, 4.837512969970703125e-4f, r);
    r = fmaf(-k, 7.549789954891882e-8f, r);
    q = int(k);
    return r;
}
PT_HD void pt_sincos(float x, float &s, float &c) {
    if (!(fabsf(x) <= 16777216.0f)) {
        s = c = (x - x) / (x - x);
        return;
    }
    int q;
    float r = pt_reduce(x, q);
    float sp = pt_sin_poly(r), cp = pt_cos_poly(r);
    switch (q & 3) {
        case 0: s = sp; c = cp; break;
        case 1: s = cp; c = -sp; break;
        case 2: s = -sp; c = -cp; break;
        default: s = -cp; c = sp; break;
    }
}

// Correctly rounded f32 sqrt: g = x*rsq(x) and one residual correction
// g + (x - g*g) * rsq(x)/2 (exact residual by fma) for x in [2^-96, 2^128);
// the rest (zeros, negatives, tiny, inf, NaN) takes the wave through the
// IEEE sqrtf.  Verified equal to sqrtf for all 2^32 inputs by pt_selftest /
// tests/test_gpu_selftest.py.
PT_HD float pt_sqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    // x in [2^-96, 2^128) as an unsigned range test on the bits; anything else
    // (zeros, negatives, tiny, inf, NaN) takes the IEEE sqrtf for the wave.
    // The fast result is formed first and replaced afterwards (one rarely
    // taken branch, no flow block around the common path).
    const float y = __builtin_amdgcn_rsqf(x);
    const float g = x * y;
    const float h = 0.5f * y;
    const float r = fmaf(-g, g, x);
    float s = fmaf(r, h, g);
    if (__builtin_expect(__ballot((__float_as_uint(x) - 0x0F800000u) >= (0x7F800000u - 0x0F800000u)) != 0ull, 0))
        s = sqrtf(x);
    return s;
#else
    return sqrtf(x);
#endif
}

// Correctly rounded a / b from y = RN(1/b) with one residual correction
// (Markstein): q = RN(a*y), r = a - q*b (exact by fma), RN(q + r*y).  Equal
// to IEEE a / b whenever nothing under/overflows; bounds() takes it under the
// guards below, which keep every intermediate normal.
// Proven on the device for every pair of significands (pt_check_div_exhaustive)
// -- power-of-two scaling carries that to all guarded exponents.
PT_HD float pt_div_rcp(float a, float b, float y) {
    const float q = a * y;
    const float r = fmaf(-q, b, a);
    return fmaf(r, y, q);
}
// a / b for a constant b, |b| in [2^-4, 2^4], and y = RN(1/b) (the baked
// scene kernels' scale divisions): pt_div_rcp, then v_div_fixup for a's
// specials (zeros, infinities, NaN -- the IEEE division ends in the same
// instruction, so the same results), and the IEEE division for a wave with a
// finite a outside [2^-60, 2^120) (there an intermediate could leave the
// normal range).  tests/test_gpu_selftest.py checks it against a / b.
PT_HD float pt_div_k(float a, float b, float y) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    float q = __builtin_amdgcn_div_fixupf(pt_div_rcp(a, b, y), b, a);
    const uint32_t e = uint32_t(__builtin_amdgcn_frexp_expf(a) + 59);  // a = m 2^e, m in [0.5, 1); 0 for 0/inf/NaN
    if (__builtin_expect(__ballot(e > 179u) != 0ull, 0)) q = a / b;
    return q;
#else
    (void)y;
    return a / b;
#endif
}
// slab operand guard: 0 or |x| in [2^-36, 2^59] (then a difference of two
// such values is 0 or in [2^-60, 2^60])
PT_HD bool pt_div_coord_ok(float x) {
    const uint32_t u = __builtin_bit_cast(uint32_t, x) & 0x7fffffffu;
    return u == 0u || (u - 0x2D800000u) <= (0x5D000000u - 0x2D800000u);
}
// divisor guard: |d| in [2^-20, 2^59]
PT_HD bool pt_div_dir_ok(float d) {
    const uint32_t u = __builtin_bit_cast(uint32_t, d) & 0x7fffffffu;
    return (u - 0x35800000u) <= (0x5D000000u - 0x35800000u);
}

struct pt_f3 {
    float x, y, z;
};
PT_HD float pt_dot(pt_f3 a, pt_f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD float pt_length(pt_f3 a) { return pt_sqrt(pt_dot(a, a)); }
// GLSL normalize(v) = v / length(v)
PT_HD pt_f3 pt_normalize(pt_f3 a) {
    float l = pt_length(a);
    return pt_f3{a.x / l, a.y / l, a.z / l};
}

// ---- display contract (render_texture_shader.wgsl) ------------------------
// WGSL pow's precision is the driver's (parity unpinned there).  Contract:
// pow(x, y) for x > 0 evaluated in double with fixed series and explicit
// fma (log2 via 2*atanh on [sqrt(1/2), sqrt(2)), exp2 via Taylor on
// [-1/2, 1/2]), rounded once to f32 -- identical on host and device and
// within one f32 ulp of the true value.  x == 0 gives 0.
PT_HD double pt_log2_d(double x) {
    int e = 0;
    double m = frexp(x, &e);  // x = m * 2^e, m in [0.5, 1)
    m *= 2.0;
    e -= 1;
    if (m > 1.4142135623730951) {
        m *= 0.5;
        e += 1;
    }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 1.0 / 23.0;
    p = fma(p, s2, 1.0 / 21.0);
    p = fma(p, s2, 1.0 / 19.0);
    p = fma(p, s2, 1.0 / 17.0);
    p = fma(p, s2, 1.0 / 15.0);
    p = fma(p, s2, 1.0 / 13.0);
    p = fma(p, s2, 1.0 / 11.0);
    p = fma(p, s2, 1.0 / 9.0);
    p = fma(p, s2, 1.0 / 7.0);
    p = fma(p, s2, 1.0 / 5.0);
    p = fma(p, s2, 1.0 / 3.0);
    p = fma(p, s2, 1.0);
    const double ln_m = (2.0 * s) * p;
    return double(e) + ln_m * 1.4426950408889634;  // 1 / ln 2
}
PT_HD double pt_exp2_d(double t) {  // |t| < 1000
    const double k = floor(t + 0.5), z = (t - k) * 0.6931471805599453;
    double p = 1.0 / 6227020800.0;  // 1/13!
    p = fma(p, z, 1.0 / 479001600.0);
    p = fma(p, z, 1.0 / 39916800.0);
    p = fma(p, z, 1.0 / 3628800.0);
    p = fma(p, z, 1.0 / 362880.0);
    p = fma(p, z, 1.0 / 40320.0);
    p = fma(p, z, 1.0 / 5040.0);
    p = fma(p, z, 1.0 / 720.0);
    p = fma(p, z, 1.0 / 120.0);
    p = fma(p, z, 1.0 / 24.0);
    p = fma(p, z, 1.0 / 6.0);
    p = fma(p, z, 0.5);
    p = fma(p, z, 1.0);
    p = fma(p, z, 1.0);
    return ldexp(p, int(k));
}
PT_HD float pt_pow_pos(float x, float y) {
    if (!(x > 0.0f)) return 0.0f;
    return float(pt_exp2_d(double(y) * pt_log2_d(double(x))));
}
// LinearToSRGB (render_texture_shader.wgsl:31-38): clamp, pow(1/2.4) branch,
// linear branch, mix by LessThan.  The constant 1/2.4 is WGSL abstract-float
// arithmetic rounded to f32.
PT_HD float pt_linear_to_srgb(float v) {
    const float c = pt_gmin(pt_gmax(v, 0.0f), 1.0f);
    const float a = pt_pow_pos(c, float(1.0 / 2.4)) * 1.055f - 0.055f;
    const float b = c * 12.92f;
    const float t = c < 0.0031308f ? 1.0f : 0.0f;
    return a * (1.0f - t) + b * t;
}
// ACESFilm (render_texture_shader.wgsl:49-56)
PT_HD float pt_aces(float x) {
    const float n = x * (2.51f * x + 0.03f), d = x * (2.43f * x + 0.59f) + 0.14f;
    return pt_gmin(pt_gmax(n / d, 0.0f), 1.0f);
}
// color_corection + fs_main's output (:62-72, :81-94): exposure 1, ACES, sRGB
PT_HD float pt_display_channel(float x) { return pt_linear_to_srgb(pt_aces(x * 1.0f)); }
// The sRGB swapchain (setup.rs:53-59 picks an sRGB format) encodes the
// fragment output once more and stores 8 bits (round to nearest even).
PT_HD uint32_t pt_srgb8(float fs_out) {
    const float s = pt_linear_to_srgb(fs_out);
    return uint32_t(rintf(s * 255.0f));
}
