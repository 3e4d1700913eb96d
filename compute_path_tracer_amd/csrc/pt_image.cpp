// pt_image.cpp -- the save-image pixel transform of State::save_image
// (src/state.rs:277-289), host side, after the pt_read_accum readback that
// replaces its copy_texture_to_buffer + map_async (state.rs:238-270).
//
//   output row y (row 0 = top of the PNG) = input row height - 1 - y   (:283)
//   r, g, b: (v.powf(1.0 / 2.2) * 255.0) as u8                          (:285-287)
//   a:       (v * 255.0) as u8                                          (:288)
//
// Rust evaluates `1.0 / 2.2` in f32 (both literals take the f32 type of
// `powf`'s argument): RN32(1 / RN32(2.2)) = 0x3EE8BA2E, one ulp below the
// f32 rounding of the real 1/2.2.  f32::powf lowers to the platform libm's
// powf (glibc on Linux), which is what this file calls.  `as u8` from a
// float saturates: NaN and values <= 0 give 0, values >= 255 give 255,
// everything else truncates towards zero.  Host code only.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/pt_abi.h"

namespace {

inline uint8_t as_u8(float v) {
    if (!(v > 0.0f)) return 0;  // NaN, -0, +0, negatives
    if (v >= 255.0f) return 255;
    return uint8_t(v);  // truncation towards zero
}

void save_rows(const float *rgba, uint32_t w, uint32_t h, uint8_t *out, uint32_t y0, uint32_t y1, float g) {
    for (uint32_t y = y0; y < y1; ++y) {
        const float *src = rgba + size_t(h - 1 - y) * w * 4;
        uint8_t *dst = out + size_t(y) * w * 4;
        for (uint32_t x = 0; x < w; ++x) {
            for (int k = 0; k < 3; ++k) dst[4 * x + k] = as_u8(::powf(src[4 * x + k], g) * 255.0f);
            dst[4 * x + 3] = as_u8(src[4 * x + 3] * 255.0f);
        }
    }
}

}  // namespace

extern "C" int pt_save_rgba8(const float *rgba, uint32_t width, uint32_t height, uint8_t *out, size_t bytes) {
    const size_t n = size_t(width) * height;
    if (n && (!rgba || !out)) return PT_ERR_INVALID;
    if (bytes < n * 4) return PT_ERR_SIZE;
    volatile float one = 1.0f, two_point_two = 2.2f;  // the f32 division, not a folded double
    const float g = one / two_point_two;
    const uint32_t threads = std::min<uint32_t>(std::max(1u, std::thread::hardware_concurrency()),
                                                std::min<uint32_t>(16u, std::max<uint32_t>(1u, height / 64u)));
    if (threads <= 1) {
        save_rows(rgba, width, height, out, 0, height, g);
        return PT_OK;
    }
    // rows [y0 of band t, ...) per thread; a band whose thread cannot be
    // started runs on the calling thread (no exception crosses the C ABI)
    std::vector<std::thread> pool;
    uint32_t t = 0;
    try {
        pool.reserve(threads);
        for (; t < threads; ++t) {
            const uint32_t y0 = uint32_t(uint64_t(height) * t / threads);
            const uint32_t y1 = uint32_t(uint64_t(height) * (t + 1) / threads);
            pool.emplace_back(save_rows, rgba, width, height, out, y0, y1, g);
        }
    } catch (const std::exception &) {
        // (std::system_error from std::thread, std::bad_alloc from reserve)
    }
    save_rows(rgba, width, height, out, uint32_t(uint64_t(height) * t / threads), height, g);
    for (auto &th : pool) th.join();
    return PT_OK;
}
