// pt_selftest.hip -- device arithmetic probes for the semantics contract
// (DESIGN.md 3): the tests compare the GPU's min/max/sqrt/sin/cos/divide on
// chosen operands with the host restatements, check the kernels' fast
// correctly-rounded sqrt against the compiler's IEEE sqrtf for every one of
// the 2^32 f32 bit patterns, and the reciprocal-based division of bounds()
// (pt_div_rcp) against IEEE division for every pair of significands plus
// random guarded operands.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/pt_abi.h"
#include "pt_path.h"

namespace {

__global__ void math_kernel(int op, const float *a, const float *b, float *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = a[i], y = b[i];
    float r = 0.0f;
    switch (op) {
        case PT_MATH_MAX: r = pt_gmax(x, y); break;
        case PT_MATH_MIN: r = pt_gmin(x, y); break;
        case PT_MATH_SQRT: r = pt_sqrt(x); break;
        case PT_MATH_SQRTF: r = sqrtf(x); break;
        case PT_MATH_SIN: {
            float s, c;
            pt_sincos(x, s, c);
            r = s;
            break;
        }
        case PT_MATH_COS: {
            float s, c;
            pt_sincos(x, s, c);
            r = c;
            break;
        }
        case PT_MATH_DIV: r = x / y; break;
        case PT_MATH_FMA: r = fmaf(x, y, 1.0f); break;
        default: r = 0.0f;
    }
    out[i] = r;
}

__global__ void sqrt_sweep(uint64_t base, uint32_t count, unsigned long long *bad, uint32_t *first) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += stride) {
        const uint32_t bits = uint32_t(base + k);
        const float x = __uint_as_float(bits);
        const uint32_t got = __float_as_uint(pt_sqrt(x)), want = __float_as_uint(sqrtf(x));
        const bool nan_both = (got & 0x7fffffffu) > 0x7f800000u && (want & 0x7fffffffu) > 0x7f800000u;
        if (got != want && !nan_both) {
            ++nbad;
            atomicMin(first, bits);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

// pt_div_rcp vs IEEE a / b for a = 1.ma, b = 1.mb over a block of
// significands: one b per thread, a looping.  The first mismatch is kept as
// (b bits << 32 | a bits).
__global__ void div_sweep(uint32_t a0, uint32_t na, uint32_t b0, uint32_t nb, unsigned long long *bad,
                          unsigned long long *first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nb) return;
    const float b = __uint_as_float(0x3F800000u | (b0 + i));
    const float y = 1.0f / b;
    unsigned long long nbad = 0;
    for (uint32_t k = 0; k < na; ++k) {
        const float a = __uint_as_float(0x3F800000u | (a0 + k));
        const float got = pt_div_rcp(a, b, y), want = a / b;
        if (__float_as_uint(got) != __float_as_uint(want)) {
            ++nbad;
            atomicMin(first, (static_cast<unsigned long long>(__float_as_uint(b)) << 32) | __float_as_uint(a));
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// random slab operand inside the guard: 0 (1/16) or sign * 2^[-36, 58] * 1.m
__device__ __forceinline__ float guard_coord(uint32_t h, uint32_t m) {
    if ((h & 15u) == 0u) return (h & 16u) ? -0.0f : 0.0f;
    const uint32_t e = 91u + (h >> 8) % 95u;  // [2^-36, 2^59)
    return __uint_as_float(((h & 32u) << 26) | (e << 23) | (m & 0x7fffffu));
}
// random divisor inside the guard: sign * 2^[-20, 58] * 1.m, or exactly +-1
__device__ __forceinline__ float guard_dir(uint32_t h, uint32_t m) {
    if ((h & 63u) == 0u) return (h & 64u) ? -1.0f : 1.0f;
    const uint32_t e = 107u + (h >> 8) % 79u;
    return __uint_as_float(((h & 128u) << 24) | (e << 23) | (m & 0x7fffffu));
}
// The composed bounds() claim: a = x - o for guarded x, o; guarded d; then
// pt_div_rcp(a, d, 1/d) == a / d, except that a zero quotient may differ in
// sign (which no slab comparison can observe).
__global__ void div_random(uint32_t seed, uint32_t n, unsigned long long *bad, unsigned long long *first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h0 = mix32(seed ^ mix32(i * 4u)), h1 = mix32(h0 + 1u), h2 = mix32(h0 + 2u), h3 = mix32(h0 + 3u);
    const float x = guard_coord(h0, h1), o = guard_coord(h1 * 3u + 7u, h2), d = guard_dir(h2 * 5u + 1u, h3);
    const float a = x - o;
    const float got = pt_div_rcp(a, d, 1.0f / d), want = a / d;
    const bool same = __float_as_uint(got) == __float_as_uint(want) || (got == 0.0f && want == 0.0f);
    if (!same || !pt_div_coord_ok(x) || !pt_div_coord_ok(o) || !pt_div_dir_ok(d)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, (static_cast<unsigned long long>(__float_as_uint(d)) << 32) | __float_as_uint(a));
    }
}

// The margin-decided slab test (pt_path.h ray_box_approx):
// random guarded (box, ray) pairs; mode 1 puts the ray through a box edge
// (entry and exit faces meet at one point, +-a few ulps), the near-ties the
// margin must leave undecided.  Modes 2 / 3: the same pairs through the
// one-fma slabs (ray_box_fma); modes 4 / 5: those with the
// origin 64x farther out and the box 100x closer along the ray (the fma
// form's absolute error term at its largest next to the slab values); modes
// 6 / 7: the pairs of modes 0 / 1 through the ulp-margin test (ray_box_ulp,
// DESIGN.md 3.19).  Counts: [0] decided lanes whose answer differs
// from the IEEE slab test, [1] undecided lanes whose exact answer
// (ray_box_rcp) differs, [2] undecided lanes, [3] pairs outside the guards.
__global__ void box_random(uint32_t seed, uint32_t n, int mode, unsigned long long *cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = mix32(seed ^ mix32(i * 16u + 1u));
    auto next = [&]() { return h = mix32(h + 0x9E3779B9u); };
    float o[3], d[3], p[3];
    const bool far = mode == 4 || mode == 5;
    const float t = far ? 0.005f + float(next() >> 8) * (0.16f / 16777216.0f)
                        : 0.5f + float(next() >> 8) * (16.0f / 16777216.0f);
    for (int k = 0; k < 3; ++k) {
        o[k] = float(int32_t(next() >> 16) - 32768) * ((far ? 256.0f : 4.0f) / 32768.0f);
        d[k] = guard_dir(next(), next());
        d[k] = fminf(fmaxf(d[k], -64.0f), 64.0f);
        if (fabsf(d[k]) < 0x1p-20f) d[k] = 1.0f;
        p[k] = o[k] + d[k] * t;
    }
    PtAabb b{};
    for (int k = 0; k < 3; ++k) {
        const float r1 = 0.01f + float(next() >> 8) * (2.0f / 16777216.0f);
        const float r2 = 0.01f + float(next() >> 8) * (2.0f / 16777216.0f);
        b.bmin[k] = p[k] - r1;
        b.bmax[k] = p[k] + r2;
    }
    if (mode == 1 || mode == 3 || mode == 5 || mode == 7) {  // entry through face a1 and exit through face a2 at p, jittered by a few ulps
        const int a1 = int(next() % 3u), a2 = (a1 + 1 + int(next() % 2u)) % 3;
        const int u1 = int(next() % 9u) - 4, u2 = int(next() % 9u) - 4;
        if (d[a1] > 0.0f) b.bmin[a1] = __uint_as_float(__float_as_uint(p[a1]) + uint32_t(u1));
        else b.bmax[a1] = __uint_as_float(__float_as_uint(p[a1]) + uint32_t(u1));
        if (d[a2] > 0.0f) b.bmax[a2] = __uint_as_float(__float_as_uint(p[a2]) + uint32_t(u2));
        else b.bmin[a2] = __uint_as_float(__float_as_uint(p[a2]) + uint32_t(u2));
    }
    bool ok = true;
    for (int k = 0; k < 3; ++k)
        ok = ok && pt_div_coord_ok(o[k]) && pt_div_dir_ok(d[k]) && pt_div_coord_ok(b.bmin[k]) &&
             pt_div_coord_ok(b.bmax[k]);
    if (!ok) {
        atomicAdd(cnt + 3, 1ull);
        return;
    }
    const float yx = 1.0f / d[0], yy = 1.0f / d[1], yz = 1.0f / d[2];
    float gap = __builtin_inff();
    bool approx, decided;
    if (mode >= 6) {  // the ulp margin (ray_box_ulp)
        uint32_t gapu = 0xffffffffu;
        approx = pt::ray_box_ulp(b, o[0], o[1], o[2], yx, yy, yz, gapu);
        decided = gapu > PT_ULP_MARGIN;
    } else if (mode >= 2) {  // the one-fma slabs (ray_box_fma)
        const float nx = -(o[0] * yx), ny = -(o[1] * yy), nz = -(o[2] * yz);
        float tfa = __builtin_inff();
        approx = pt::ray_box_fma(b, nx, ny, nz, yx, yy, yz, gap, tfa);
        decided = pt::fma_decided(gap, tfa, nx, ny, nz);
    } else {
        approx = pt::ray_box_approx(b, o[0], o[1], o[2], yx, yy, yz, gap);
        decided = gap > 0.0f;
    }
    const bool want = pt::ray_box(b, o[0], o[1], o[2], d[0], d[1], d[2]);
    if (decided) {
        if (approx != want) atomicAdd(cnt + 0, 1ull);
    } else {
        atomicAdd(cnt + 2, 1ull);
        if (pt::ray_box_rcp(b, o[0], o[1], o[2], d[0], d[1], d[2], yx, yy, yz) != want) atomicAdd(cnt + 1, 1ull);
    }
}

// pt_div_k(a, b, RN(1/b)) against the IEEE a / b, bit for bit, for every a
// of a slice of the 2^32 patterns (zeros, subnormals, infinities and NaNs
// included).
__global__ void divk_sweep(uint32_t a0, float b, unsigned long long *bad, unsigned long long *first) {
    const uint32_t a_bits = a0 + blockIdx.x * blockDim.x + threadIdx.x;
    const float a = __uint_as_float(a_bits);
    volatile float bv = b;  // (no constant folding of the reference division)
    const float bb = bv;
    const float y = 1.0f / bb;
    const float want = a / bb;
    const float got = pt_div_k(a, bb, y);
    if (__float_as_uint(got) != __float_as_uint(want)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, (unsigned long long)a_bits);
    }
}

}  // namespace

extern "C" int pt_check_div_k(int hip_device, float b, uint32_t a0, uint32_t na, uint64_t *mismatches,
                              uint64_t *first_bad) {
    if (!mismatches || !first_bad || na % 256u != 0u || a0 + uint64_t(na) > (1ull << 32)) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(*d)) != hipSuccess) return PT_ERR_HIP;
    const unsigned long long init[2] = {0ull, ~0ull};
    int rc = hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice) == hipSuccess ? PT_OK : PT_ERR_HIP;
    for (uint64_t a = a0; rc == PT_OK && a < uint64_t(a0) + na; a += 1ull << 28) {  // 2^28 per launch
        const uint64_t cnt = std::min<uint64_t>(1ull << 28, uint64_t(a0) + na - a);
        hipLaunchKernelGGL(divk_sweep, dim3(unsigned(cnt / 256u)), dim3(256), 0, 0, uint32_t(a), b, d, d + 1);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PT_ERR_HIP;
    }
    unsigned long long h[2] = {0ull, 0ull};
    if (rc == PT_OK && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) rc = PT_ERR_HIP;
    *mismatches = h[0];
    *first_bad = h[1];
    (void)hipFree(d);
    return rc;
}

extern "C" int pt_check_box_random(int hip_device, uint32_t seed, uint32_t n, int mode, uint64_t *counts) {
    if (!counts) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(*d)) != hipSuccess) return PT_ERR_HIP;
    int rc = hipMemset(d, 0, 4 * sizeof(*d)) == hipSuccess ? PT_OK : PT_ERR_HIP;
    if (rc == PT_OK && n > 0) {
        hipLaunchKernelGGL(box_random, dim3((n + 255) / 256), dim3(256), 0, 0, seed, n, mode, d);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PT_ERR_HIP;
    }
    unsigned long long h[4] = {0ull, 0ull, 0ull, 0ull};
    if (rc == PT_OK && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) rc = PT_ERR_HIP;
    for (int k = 0; k < 4; ++k) counts[k] = h[k];
    (void)hipFree(d);
    return rc;
}

extern "C" int pt_check_div_exhaustive(int hip_device, uint32_t a0, uint32_t na, uint32_t b0, uint32_t nb,
                                       uint64_t *mismatches, uint64_t *first_bad) {
    if (!mismatches || !first_bad || a0 + uint64_t(na) > (1u << 23) || b0 + uint64_t(nb) > (1u << 23))
        return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(*d)) != hipSuccess) return PT_ERR_HIP;
    const unsigned long long init[2] = {0ull, ~0ull};
    int rc = hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice) == hipSuccess ? PT_OK : PT_ERR_HIP;
    // slices of a keep each launch well under a second
    for (uint32_t a = a0; rc == PT_OK && a < a0 + na; a += 1u << 15) {
        const uint32_t cnt = std::min<uint32_t>(1u << 15, a0 + na - a);
        hipLaunchKernelGGL(div_sweep, dim3((nb + 255) / 256), dim3(256), 0, 0, a, cnt, b0, nb, d, d + 1);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PT_ERR_HIP;
    }
    unsigned long long h[2] = {0ull, 0ull};
    if (rc == PT_OK && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) rc = PT_ERR_HIP;
    *mismatches = h[0];
    *first_bad = h[1];
    (void)hipFree(d);
    return rc;
}

extern "C" int pt_check_div_random(int hip_device, uint32_t seed, uint32_t n, uint64_t *mismatches,
                                   uint64_t *first_bad) {
    if (!mismatches || !first_bad) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(*d)) != hipSuccess) return PT_ERR_HIP;
    const unsigned long long init[2] = {0ull, ~0ull};
    int rc = hipMemcpy(d, init, sizeof init, hipMemcpyHostToDevice) == hipSuccess ? PT_OK : PT_ERR_HIP;
    if (rc == PT_OK && n > 0) {
        hipLaunchKernelGGL(div_random, dim3((n + 255) / 256), dim3(256), 0, 0, seed, n, d, d + 1);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PT_ERR_HIP;
    }
    unsigned long long h[2] = {0ull, 0ull};
    if (rc == PT_OK && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) rc = PT_ERR_HIP;
    *mismatches = h[0];
    *first_bad = h[1];
    (void)hipFree(d);
    return rc;
}

extern "C" int pt_device_math(int hip_device, int op, const float *a, const float *b, float *out, uint32_t n) {
    if (!a || !b || !out) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    const size_t bytes = size_t(n > 0 ? n : 1) * sizeof(float);
    int rc = PT_OK;
    if (hipMalloc(&da, bytes) != hipSuccess || hipMalloc(&db, bytes) != hipSuccess || hipMalloc(&dout, bytes) != hipSuccess)
        rc = PT_ERR_HIP;
    if (rc == PT_OK && n > 0) {
        if (hipMemcpy(da, a, n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(db, b, n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
            rc = PT_ERR_HIP;
        if (rc == PT_OK) {
            hipLaunchKernelGGL(math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, op, da, db, dout, n);
            if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
                hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
                rc = PT_ERR_HIP;
        }
    }
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    return rc;
}

extern "C" int pt_check_sqrt_exhaustive(int hip_device, uint64_t *mismatches, uint32_t *first_bad) {
    if (!mismatches || !first_bad) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    unsigned long long *dbad = nullptr;
    uint32_t *dfirst = nullptr;
    if (hipMalloc(&dbad, sizeof(*dbad)) != hipSuccess || hipMalloc(&dfirst, sizeof(*dfirst)) != hipSuccess)
        return PT_ERR_HIP;
    const uint32_t init_first = 0xffffffffu;
    int rc = PT_OK;
    if (hipMemset(dbad, 0, sizeof(*dbad)) != hipSuccess ||
        hipMemcpy(dfirst, &init_first, sizeof(init_first), hipMemcpyHostToDevice) != hipSuccess)
        rc = PT_ERR_HIP;
    // 2^32 inputs in 4 chunks of 2^30
    for (uint64_t base = 0; rc == PT_OK && base < (1ull << 32); base += (1ull << 30)) {
        hipLaunchKernelGGL(sqrt_sweep, dim3(8192), dim3(256), 0, 0, base, uint32_t(1u << 30), dbad, dfirst);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PT_ERR_HIP;
    }
    unsigned long long hb = 0;
    uint32_t hf = 0;
    if (rc == PT_OK && (hipMemcpy(&hb, dbad, sizeof(hb), hipMemcpyDeviceToHost) != hipSuccess ||
                        hipMemcpy(&hf, dfirst, sizeof(hf), hipMemcpyDeviceToHost) != hipSuccess))
        rc = PT_ERR_HIP;
    *mismatches = hb;
    *first_bad = hf;
    (void)hipFree(dbad);
    (void)hipFree(dfirst);
    return rc;
}
