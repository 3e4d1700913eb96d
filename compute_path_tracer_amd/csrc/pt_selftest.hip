// pt_selftest.hip -- device arithmetic probes for the semantics contract
// (DESIGN.md 3): the tests compare the GPU's min/max/sqrt/sin/cos/divide on
// chosen operands with the host restatements, and check the kernels' fast
// correctly-rounded sqrt against the compiler's IEEE sqrtf for every one of
// the 2^32 f32 bit patterns.
#include <hip/hip_runtime.h>

#include "../../include/pt_abi.h"
#include "pt_math.h"

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

}  // namespace

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
