// pt_probe.hip -- known-byte-count access patterns for calibrating
// rocprofv3's FETCH_SIZE / WRITE_SIZE on the pipeline's own access shapes.
//
// MI355X_MICROARCH.md ("HBM"): on gfx950 FETCH_SIZE reports half the bytes of
// a wide coalesced 16 B/lane read, WRITE_SIZE is exact for 16 B/lane
// streaming stores, and other widths are uncalibrated.  The binned pipeline's
// traffic is mostly other shapes: 64 B ray records gathered by slot (trace
// and shade passes), 16 B hit quads stored at scattered binned positions
// (trace), 64 B records stored whole (shade).  Each probe kernel below moves
// a known number of bytes in one of those shapes over a buffer far larger
// than the 256 MiB Infinity Cache, so the counters' ratio to the known bytes
// is the correction for that shape (scripts/pmc_calib.sh, profiles/*_calib*).
//
//   gather64   read n 64 B records, record j = perm(i) (4 x dwordx4 per lane)
//   stream16   read n 16 B quads in order (1 x dwordx4 per lane, coalesced)
//   scatter16  store n 16 B quads at perm(i)
//   store64    store n 64 B records in order (4 x dwordx4 per lane)
//
// perm(i) = (i * A + B) mod n for a power-of-two n and odd A: a bijection
// that scatters consecutive i over the whole buffer.
#include <hip/hip_runtime.h>

#include "../../include/pt_abi.h"

namespace {

constexpr uint32_t kPermA = 0x9E3779B1u;  // odd
constexpr uint32_t kPermB = 0x7F4A7C15u;

__device__ __forceinline__ uint32_t perm(uint32_t i, uint32_t mask) { return (i * kPermA + kPermB) & mask; }

__global__ __launch_bounds__(256) void pt_probe_gather64(const uint4 *rec, uint32_t n, uint32_t *sink) {
    uint32_t acc = 0u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4 *r = rec + size_t(perm(i, n - 1u)) * 4u;
        const uint4 a = r[0], b = r[1], c = r[2], d = r[3];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    if (acc == 0x5A5A5A5Au) sink[0] = acc;  // (keeps the loads; practically never stores)
}

__global__ __launch_bounds__(256) void pt_probe_stream16(const uint4 *q, uint32_t n, uint32_t *sink) {
    uint32_t acc = 0u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint4 a = q[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x5A5A5A5Au) sink[0] = acc;
}

__global__ __launch_bounds__(256) void pt_probe_scatter16(uint4 *q, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        q[perm(i, n - 1u)] = make_uint4(i, i + 1u, i + 2u, i + 3u);
}

__global__ __launch_bounds__(256) void pt_probe_store64(uint4 *rec, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint4 *r = rec + size_t(i) * 4u;
        r[0] = make_uint4(i, 1u, 2u, 3u);
        r[1] = make_uint4(i, 5u, 6u, 7u);
        r[2] = make_uint4(i, 9u, 10u, 11u);
        r[3] = make_uint4(i, 13u, 14u, 15u);
    }
}

}  // namespace

// Runs the four probes once each on 2^log2n items (log2n in [16, 26]:
// the gather reads up to 4 GiB) and returns each one's device time in ms
// (HIP events) and its known byte count.  Test / calibration aid.
extern "C" int pt_traffic_probe(int hip_device, uint32_t log2n, float ms[4], uint64_t bytes[4]) {
    if (log2n < 16 || log2n > 26 || !ms || !bytes) return PT_ERR_INVALID;
    if (hipSetDevice(hip_device) != hipSuccess) return PT_ERR_HIP;
    const uint32_t n = 1u << log2n;
    uint4 *rec = nullptr, *q = nullptr;
    uint32_t *sink = nullptr;
    hipEvent_t e[5] = {};
    int rc = PT_OK;
    if (hipMalloc(&rec, size_t(n) * 64) != hipSuccess || hipMalloc(&q, size_t(n) * 16) != hipSuccess ||
        hipMalloc(&sink, 4) != hipSuccess) {
        rc = PT_ERR_HIP;
    }
    for (int k = 0; rc == PT_OK && k < 5; ++k)
        if (hipEventCreate(&e[k]) != hipSuccess) rc = PT_ERR_HIP;
    if (rc == PT_OK) {
        const dim3 grid(1024), block(256);
        (void)hipMemset(rec, 0x11, size_t(n) * 64);
        (void)hipMemset(q, 0x22, size_t(n) * 16);
        (void)hipEventRecord(e[0], nullptr);
        hipLaunchKernelGGL(pt_probe_gather64, grid, block, 0, nullptr, rec, n, sink);
        (void)hipEventRecord(e[1], nullptr);
        hipLaunchKernelGGL(pt_probe_stream16, grid, block, 0, nullptr, q, n, sink);
        (void)hipEventRecord(e[2], nullptr);
        hipLaunchKernelGGL(pt_probe_scatter16, grid, block, 0, nullptr, q, n);
        (void)hipEventRecord(e[3], nullptr);
        hipLaunchKernelGGL(pt_probe_store64, grid, block, 0, nullptr, rec, n);
        (void)hipEventRecord(e[4], nullptr);
        if (hipGetLastError() != hipSuccess || hipEventSynchronize(e[4]) != hipSuccess) rc = PT_ERR_HIP;
        for (int k = 0; rc == PT_OK && k < 4; ++k)
            if (hipEventElapsedTime(&ms[k], e[k], e[k + 1]) != hipSuccess) rc = PT_ERR_HIP;
        bytes[0] = uint64_t(n) * 64;
        bytes[1] = uint64_t(n) * 16;
        bytes[2] = uint64_t(n) * 16;
        bytes[3] = uint64_t(n) * 64;
    }
    for (hipEvent_t ev : e)
        if (ev) (void)hipEventDestroy(ev);
    (void)hipFree(rec);
    (void)hipFree(q);
    (void)hipFree(sink);
    return rc;
}
