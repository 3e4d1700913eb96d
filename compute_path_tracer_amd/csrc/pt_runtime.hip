// pt_runtime.hip -- implementation of the C ABI in include/pt_abi.h.
//
// Owns what the reference's wgpu objects owned (path_tracer.rs:18-163,
// structs.rs:113-184, primitives.rs:59-157): the RGBA32F accumulation image,
// the scene program and its parameter buffer, and the dispatch.  One HIP
// stream per context; RCCL communicator for the multi-GPU image reduce.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <future>
#include <map>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <vector>

#include "../../include/pt_abi.h"
#include "pt_device.h"
#include "pt_host.h"
#include "pt_math.h"


static_assert(sizeof(pt_constants) == 16, "Constants is 16 B (path_tracer.rs:149-155)");
static_assert(sizeof(pt_settings) == 20, "Settings is 20 B (path_tracer.rs:157-163)");
static_assert(sizeof(pt_op) == 33 * 4, "pt_op layout");
static_assert(sizeof(pt_aabb) == 14 * 4, "pt_aabb layout");
static_assert(sizeof(pt_scene_node) == 33 * 4, "pt_scene_node layout");
static_assert(PT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "RCCL unique id size");

// A scene-kernel code object and where it came from: compiled by this
// process's hipRTC, or read from the shipped on-disk cache (lib/jitcache)
enum JitFrom { kJitCompiled = 0, kJitDisk = 1 };
struct JitBuild {
    std::vector<char> code;  // empty: the compile failed (log set)
    double seconds = 0.0;
    int from = kJitCompiled;
};

struct pt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t width = 0, height = 0;
    float *accum = nullptr;
    float *reduced = nullptr;
    // program
    std::vector<pt_op> ops;
    std::vector<pt_aabb> aabbs;
    uint32_t n_check = 1;
    bool have_program = false, have_data = false;
    uint32_t n_data_expected = 0;
    // device tables
    PtNode *d_nodes = nullptr;
    PtAabb *d_aabbs = nullptr;
    PtMat *d_mats = nullptr;
    size_t cap_nodes = 0, cap_aabbs = 0, cap_mats = 0;
    unsigned long long *d_stats = nullptr;  // 2 x PT_ST_COUNT (second half: the shade pass's normal taps)
    unsigned long long tap_stats[PT_ST_COUNT] = {};  // last pt_dispatch_stats: the shade-pass taps' share
    // tiles
    uint32_t rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    uint32_t comm_nranks = 0;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    // options (pt_set_option)
    int kernel = PT_KERNEL_AUTO;  // PT_KERNEL_*
    int shade_batch = 16;         // state-machine kernels: lanes waiting before a shading pass (measured best)
    int jit = 1;                  // 1 use per-scene hipRTC kernels, 0 interpreter
    int jit_bake = 2;             // 0 values from the node table, 1 baked as literals, 2 tier-up
    int bin_samples = 0;          // binned pipeline: samples per chunk; 0 = automatic (bin_samples())
    size_t bin_auto = 0;          // the automatic chunk size, fixed at the first binned dispatch
    bool bin_fallback = false;    // bin_auto came from the free memory (the total-memory size did not fit)
    uint32_t last_chunks = 0;     // chunks of the last timed binned dispatch
    PtJitModule jit_mod;   // scene kernel for the topology (key = its source)
    // tier-up (jit_bake 2): the same kernel with the current values baked in as
    // literals, compiled on a worker thread and used once ready while the
    // values stay unchanged -- value edits never wait for a compile
    PtJitModule jit_tier;
    std::string tier_want;  // baked source for the current values
    std::string tier_job_src;
    std::string tier_failed;  // a baked source that did not build (not retried)
    // code object (empty: compile failed) and its compile seconds; the worker
    // returns both through the future, so no field is shared with it
    std::future<JitBuild> tier_job;
    double tier_seconds = 0.0;
    int jit_from = -1, tier_from = -1;  // where the loaded builds came from (JitFrom)
    // binned pipeline buffers (pt_binned.h).  A chunk's frames are split over
    // up to kMaxLanes independent pipelines ("lanes"), each on its own stream,
    // so one lane's memory-bound passes (shade, gen, scatter) run beside
    // another's VALU-bound trace pass and fill its tail.  bin_cap samples per
    // lane; the colour buffer holds the whole chunk.
    struct BinLane {
        PtRay *ray[2] = {nullptr, nullptr};  // ping-pong: pass k traces ray[k & 1], its shade pass writes the other
        uint4 *hq = nullptr;                 // trace -> shade: the hit quads (taps in the shade pass)
        uint2 *mask_hi = nullptr;            // check[] bits 64..127 (scenes with > 64 entries)
        uint32_t *key = nullptr, *idx = nullptr, *hist = nullptr, *offs = nullptr, *ctrl = nullptr;
        float4 *hitn = nullptr;  // trace -> shade: normal differences per position
        hipStream_t stream = nullptr;
    };
    static constexpr int kMaxLanes = 4;
    BinLane lane[kMaxLanes];
    int n_lanes = 0;  // lanes allocated
    float4 *d_color = nullptr;
    size_t bin_cap = 0, ctrl_words = 0;
    hipStream_t xstream[kMaxLanes] = {};   // lanes 1.. streams (created on first use; lane 0 = stream)
    hipEvent_t fork_ev = nullptr, join_ev[kMaxLanes] = {};
    int bin_lanes = 2;                     // pt_set_option "bin_lanes" (2: +6 % over 1; 3-4 equal or worse)
    int bin_table = 1;                     // pt_set_option "bin_table": bins from the table of check[] sets
    unsigned long long *d_btab = nullptr;  // that table, [PT_BINS] (pt_binned.h bin_probe / bin_resolve), shared by the lanes
    int shade_taps = 1;                    // pt_set_option "shade_taps": normal taps in the shade pass
    int gen_trace_used = 0;                // the last timed dispatch's first pass made its own camera rays
    int gen_norec_used = 0;                // ... and stored no ray records (shade pass 0 made them again)
    bool btab_used = false;                // the last timed binned dispatch binned by the table of check[] sets
    bool btab_counted = false;             // the last instrumented one did, and counted its overflows
    int cu_count = 0;
    bool fast_bounds = false;  // every box coordinate inside the reciprocal-division guard
    float bound_k = 0.0f;      // pt_bound_k of the uploaded scene (NaN: no map() bound)
    // HIP events around each trace-pass launch of the last dispatch (pairs)
    // HIP event pairs around the last dispatch's binned trace / shade launches
    // (on each pipeline's stream): their summed device time per kernel
    struct EventLog {
        std::vector<hipEvent_t> ev;
        size_t used = 0;
    } tlog, slog;
    // display pass output (device) and its timing
    void *d_display = nullptr;
    size_t cap_display = 0;
    hipEvent_t dev0 = nullptr, dev1 = nullptr;
    bool display_timed = false;
    std::string jit_log;
    double jit_seconds = 0.0;
    std::string err;
};

namespace {

// code objects by generated source, shared by every context of the process
std::map<std::string, JitBuild> &jit_cache() {
    static std::map<std::string, JitBuild> cache;
    return cache;
}
std::mutex &jit_mutex() {
    static std::mutex m;
    return m;
}

// Code object for a generated source: from the process-wide cache, else
// from the on-disk cache or compiled (without holding the cache lock).
JitBuild jit_code(const std::string &src, std::string &log) {
    JitBuild b;
    {
        std::lock_guard<std::mutex> g(jit_mutex());
        auto it = jit_cache().find(src);
        if (it != jit_cache().end()) {
            b = it->second;
            b.seconds = 0.0;
            return b;
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    bool disk = false;
    if (!pt_jit_compile_source(src, b.code, log, &disk)) b.code.clear();
    b.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    b.from = disk ? kJitDisk : kJitCompiled;
    if (!b.code.empty()) {
        std::lock_guard<std::mutex> g(jit_mutex());
        jit_cache()[src] = b;
    }
    return b;
}

// Install a finished tier-up compile if it is still the one the current
// values want; start the wanted one if nothing is pending.  wait: block on a
// pending compile first.
void jit_tier_poll(pt_ctx *c, bool wait) {
    if (c->tier_job.valid() &&
        (wait || c->tier_job.wait_for(std::chrono::seconds(0)) == std::future_status::ready)) {
        JitBuild done = c->tier_job.get();
        c->tier_seconds = done.seconds;
        if (done.code.empty()) c->tier_failed = c->tier_job_src;
        if (!done.code.empty() && c->tier_job_src == c->tier_want && !c->jit_tier.module) {
            std::string err;
            if (pt_jit_load(done.code, c->jit_tier, err)) {
                c->jit_tier.key = c->tier_job_src;
                c->tier_from = done.from;
            } else {
                c->jit_log = err;
                c->tier_failed = c->tier_job_src;
            }
        }
        c->tier_job_src.clear();
    }
    if (!c->tier_job.valid() && !c->tier_want.empty() && c->jit_tier.key != c->tier_want &&
        c->tier_want != c->tier_failed) {
        std::string src = c->tier_want;
        c->tier_job_src = src;
        c->tier_job = std::async(std::launch::async, [src]() {
            std::string log;
            return jit_code(src, log);
        });
        if (wait) jit_tier_poll(c, true);
    }
}

// The scene kernel in use: the tier-up build when loaded, else the topology one.
const PtJitModule *jit_active(const pt_ctx *c) {
    if (c->jit_tier.module) return &c->jit_tier;
    return c->jit_mod.module ? &c->jit_mod : nullptr;
}


// (Re)build the scene-specialised kernel when the generated source changed.
// A failure leaves the interpreter kernel in use and records the log.
void jit_refresh(pt_ctx *c, const std::vector<PtNode> &nodes, const std::vector<PtAabb> &boxes) {
    if (!c->jit) {
        pt_jit_unload(c->jit_mod);
        pt_jit_unload(c->jit_tier);
        c->tier_want.clear();
        return;
    }
    const int bake = c->jit_bake;
    std::string src = pt_jit_source(nodes, boxes, c->fast_bounds, bake == 1);
    // the tier-up build for these values (jit_bake 2); a stale one is dropped
    c->tier_want = bake == 2 ? pt_jit_source(nodes, boxes, c->fast_bounds, true) : std::string();
    if (c->jit_tier.module && c->jit_tier.key != c->tier_want) pt_jit_unload(c->jit_tier);
    if (!(c->jit_mod.module && c->jit_mod.key == src)) {
        pt_jit_unload(c->jit_mod);
        std::string log;
        JitBuild b = jit_code(src, log);
        c->jit_seconds = b.seconds;
        if (b.code.empty()) {
            c->jit_log = "hipRTC compile failed: " + log;
            return;
        }
        std::string err;
        if (!pt_jit_load(b.code, c->jit_mod, err)) {
            c->jit_log = err;
            return;
        }
        c->jit_mod.key = std::move(src);
        c->jit_from = b.from;
        c->jit_log.clear();
    }
    if (bake == 2) jit_tier_poll(c, false);
}

int fail(pt_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(ctx, PT_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));     \
    } while (0)

int ensure(pt_ctx *c, void **ptr, size_t &cap, size_t need) {
    if (need <= cap && *ptr) return PT_OK;
    if (*ptr) HIPCHK(c, hipFree(*ptr));
    *ptr = nullptr;
    size_t bytes = std::max<size_t>(need, 1);
    HIPCHK(c, hipMalloc(ptr, bytes));
    cap = bytes;
    return PT_OK;
}

int alloc_image(pt_ctx *c, uint32_t w, uint32_t h) {
    if (c->accum) HIPCHK(c, hipFree(c->accum));
    if (c->reduced) HIPCHK(c, hipFree(c->reduced));
    c->accum = c->reduced = nullptr;
    c->width = w;
    c->height = h;
    size_t bytes = size_t(w) * size_t(h) * 16;
    HIPCHK(c, hipMalloc(&c->accum, std::max<size_t>(bytes, 16)));
    HIPCHK(c, hipMemsetAsync(c->accum, 0, std::max<size_t>(bytes, 16), c->stream));
    return PT_OK;
}

// Host expansion of (program, data[]) into the device tables.  Every value is
// the f32 expression the generated GLSL evaluates on the GPU, evaluated here
// once with the same rounding (see pt_device.h).
}  // namespace

// Distance-bound culling data for the scene kernels (pt_jit.cpp, DESIGN.md
// 3.12), in PtNode.pad[0]:
//  * shape: R' = R + 2^-12 (|R| + |m|_1), where R bounds the shape from its
//    local origin (sdf(q) >= |q| - R: sphere r, cube |b|, torus |R1| + r,
//    octahedron s), or NaN when the node's values are outside the range the
//    rounding argument covers (never culled);
//  * union begin: the matching end's 1/s when the union may drop shapes that
//    cannot beat its parent's running distance (it combines into the parent by
//    union, has no child unions, only assign/union shapes, all with finite
//    R'), else NaN.
void pt_cull_bounds(std::vector<PtNode> &nodes) {
    const float nan = std::numeric_limits<float>::quiet_NaN();
    const double big = 1099511627776.0;  // 2^40
    auto fin = [&](float v) { return std::isfinite(v) && std::fabs(double(v)) <= big; };
    for (PtNode &d : nodes) {
        d.pad[0] = nan;
        if (d.op != PT_OP_SHAPE) continue;
        bool ok = std::isfinite(d.inv) && d.inv >= 0x1p-20f && d.inv <= 0x1p20f && fin(d.m[0]) && fin(d.m[1]) &&
                  fin(d.m[2]) && fin(d.cx) && fin(d.sx) && fin(d.cy) && fin(d.sy) && fin(d.cz) && fin(d.sz);
        double R = 0.0;
        switch (d.shape) {
            case PT_NODE_SPHERE: ok = ok && fin(d.size[0]); R = d.size[0]; break;
            case PT_NODE_CUBE:
                ok = ok && fin(d.size[0]) && fin(d.size[1]) && fin(d.size[2]) && d.size[0] >= 0.0f &&
                     d.size[1] >= 0.0f && d.size[2] >= 0.0f;
                R = std::sqrt(double(d.size[0]) * d.size[0] + double(d.size[1]) * d.size[1] +
                              double(d.size[2]) * d.size[2]);
                break;
            case PT_NODE_TORUS:
                ok = ok && fin(d.size[0]) && fin(d.size[1]);
                R = std::fabs(double(d.size[0])) + double(d.size[1]);
                break;
            case PT_NODE_OCTAHEDRON: ok = ok && fin(d.size[0]) && d.size[0] >= 0.0f; R = d.size[0]; break;
            default: ok = false;
        }
        if (!ok) continue;
        const double m1 = std::fabs(double(d.m[0])) + std::fabs(double(d.m[1])) + std::fabs(double(d.m[2]));
        d.pad[0] = float(R + 0x1p-12 * (std::fabs(R) + m1));
    }
    for (size_t i = 0; i < nodes.size(); ++i) {
        if (nodes[i].op != PT_OP_UNION_BEGIN) continue;
        size_t j = i + 1;
        bool ok = true;
        for (; j < nodes.size() && nodes[j].op != PT_OP_UNION_END; ++j) {
            const PtNode &c = nodes[j];
            if (c.op != PT_OP_SHAPE || !(c.combine == PT_COMBINE_ASSIGN || c.combine == PT_COMBINE_UNION) ||
                !std::isfinite(c.pad[0]))
                ok = false;  // a child union, a subtraction, or a shape without a bound
        }
        if (j == nodes.size()) continue;
        const PtNode &e = nodes[j];
        ok = ok && e.combine == PT_COMBINE_UNION && std::isfinite(e.inv) && e.inv > 0.0f;
        if (ok) nodes[i].pad[0] = e.inv;
    }
}

// Margin constant of the map() bound (pt_path.h tap_bound):
// the largest transform-chain magnitude of any shape in world units -- the
// |pos| of every enclosing union and of the shape, plus the shape's radius
// bound R, each in world units.  The rounding error of a map() evaluation at
// q is a few tens of ulp of |q|_1 + K; the kernels' margin is 2^-10 times
// that.  NaN (no bound) when any 1/s is outside [1/2, 2] or any value is
// beyond 2^20.
float pt_bound_k(const std::vector<PtNode> &nodes) {
    const float nan = std::numeric_limits<float>::quiet_NaN();
    auto fin = [](double v) { return std::isfinite(v) && std::fabs(v) <= 1048576.0; };
    double K = 0.0;
    std::vector<double> scale(1, 1.0), reach(1, 0.0);  // world units per local unit; |pos| chain so far
    for (const PtNode &d : nodes) {
        if (d.op == PT_OP_UNION_END) {
            if (scale.size() > 1) {
                scale.pop_back();
                reach.pop_back();
            }
            continue;
        }
        if (!(std::isfinite(d.inv) && d.inv >= 0.5f && d.inv <= 2.0f)) return nan;
        for (float v : {d.m[0], d.m[1], d.m[2], d.size[0], d.size[1], d.size[2]})
            if (!fin(v)) return nan;
        const double sc = scale.back() / double(d.inv);  // this node's local unit in world units
        const double r = reach.back() + (std::fabs(double(d.m[0])) + std::fabs(double(d.m[1])) +
                                         std::fabs(double(d.m[2]))) * sc;
        if (d.op == PT_OP_UNION_BEGIN) {
            scale.push_back(sc);
            reach.push_back(r);
            continue;
        }
        double R;
        switch (d.shape) {
            case PT_NODE_SPHERE: R = std::fabs(double(d.size[0])); break;
            case PT_NODE_CUBE:
                R = std::sqrt(double(d.size[0]) * d.size[0] + double(d.size[1]) * d.size[1] +
                              double(d.size[2]) * d.size[2]);
                break;
            case PT_NODE_TORUS: R = std::fabs(double(d.size[0])) + std::fabs(double(d.size[1])); break;
            case PT_NODE_OCTAHEDRON: R = std::fabs(double(d.size[0])); break;
            default: return nan;
        }
        K = std::max(K, r + R * sc);
    }
    return float(K * (1.0 + 0x1p-20));
}

int pt_derive(const std::vector<pt_op> &ops, const std::vector<pt_aabb> &aabbs, const float *data, uint32_t n,
              std::vector<PtNode> &nodes, std::vector<PtAabb> &boxes, std::vector<PtMat> &mats, std::string &err) {
    auto bad = [&](const char *msg) {
        err = msg;
        return PT_ERR_INVALID;
    };
    auto in = [&](uint32_t s) { return s < n; };
    nodes.resize(ops.size());
    mats.clear();
    PtMat mdef;
    std::memset(&mdef, 0, sizeof mdef);
    {
        pt_f3 z{0.0f, 0.0f, 0.0f};
        pt_f3 nl = pt_normalize(z);  // MDEF light = vec3(0): normalize -> NaN, as upstream
        mdef.emis[0] = nl.x * 0.0f;
        mdef.emis[1] = nl.y * 0.0f;
        mdef.emis[2] = nl.z * 0.0f;
    }
    mats.push_back(mdef);
    for (size_t i = 0; i < ops.size(); ++i) {
        const pt_op &op = ops[i];
        PtNode &d = nodes[i];
        std::memset(&d, 0, sizeof d);
        d.op = int32_t(op.opcode);
        d.shape = int32_t(op.shape);
        d.combine = int32_t(op.combine);
        d.check = op.check;
        if (!in(op.scale)) return bad("op references data slot out of range");
        for (int k = 0; k < 3; ++k)
            if (!in(op.position[k]) || !in(op.rotation[k]))
                return bad("op references data slot out of range");
        const float s = data[op.scale];
        const float inv = 1.0f / s;  // `1.0 / data[scale]`
        d.inv = inv;
        for (int k = 0; k < 3; ++k) d.m[k] = data[op.position[k]] * inv;  // pos * (1.0 / s)
        uint32_t f = 0;
        if (inv != 1.0f) f |= PT_NF_SCALE;
        if (d.m[0] != 0.0f || d.m[1] != 0.0f || d.m[2] != 0.0f) f |= PT_NF_POS;
        pt_sincos(data[op.rotation[0]], d.sx, d.cx);
        pt_sincos(data[op.rotation[1]], d.sy, d.cy);
        pt_sincos(data[op.rotation[2]], d.sz, d.cz);
        if (!(d.cx == 1.0f && d.sx == 0.0f)) f |= PT_NF_RX;
        if (!(d.cy == 1.0f && d.sy == 0.0f)) f |= PT_NF_RY;
        if (!(d.cz == 1.0f && d.sz == 0.0f)) f |= PT_NF_RZ;
        d.flags = f;
        if (op.opcode == PT_OP_SHAPE) {
            for (int k = 0; k < 3; ++k) {
                if (!in(op.size[k])) return bad("size slot out of range");
                d.size[k] = data[op.size[k]];
            }
            for (int k = 0; k < 18; ++k)
                if (!in(op.material[k])) return bad("material slot out of range");
            const uint32_t *ms = op.material;
            PtMat m;
            std::memset(&m, 0, sizeof m);
            for (int k = 0; k < 3; ++k) {
                m.col[k] = data[ms[k]];
                m.spec_col[k] = data[ms[8 + k]];
            }
            m.spec = data[ms[7]];
            m.rough2 = data[ms[11]] * data[ms[11]];
            pt_f3 nl = pt_normalize(pt_f3{data[ms[4]], data[ms[5]], data[ms[6]]});
            const float br = data[ms[3]];
            m.emis[0] = nl.x * br;
            m.emis[1] = nl.y * br;
            m.emis[2] = nl.z * br;
            d.mat = int32_t(mats.size());
            mats.push_back(m);
        }
    }
    pt_cull_bounds(nodes);
    boxes.resize(aabbs.size());
    for (size_t i = 0; i < aabbs.size(); ++i) {
        const pt_aabb &a = aabbs[i];
        for (int k = 0; k < 3; ++k)
            if (!in(a.union_position[k]) || !in(a.shape_position[k]) || !in(a.size[k]))
                return bad("aabb slot out of range");
        if (!in(a.union_scale) || !in(a.shape_scale) || !in(a.aabb_exaggeration))
            return bad("aabb slot out of range");
        float so[3];
        switch (a.so_kind) {
            case PT_SO_SCALAR: so[0] = so[1] = so[2] = data[a.size[0]]; break;
            case PT_SO_VEC3:
                for (int k = 0; k < 3; ++k) so[k] = data[a.size[k]];
                break;
            case PT_SO_TORUS: {
                const float R = data[a.size[0]], r = data[a.size[1]];
                so[0] = R + r;
                so[1] = r;
                so[2] = R + r;
                break;
            }
            default: so[0] = so[1] = so[2] = 1.0f; break;
        }
        const float sc = data[a.union_scale] * data[a.shape_scale];
        const float ex = data[a.aabb_exaggeration];
        PtAabb &b = boxes[i];
        std::memset(&b, 0, sizeof b);
        for (int k = 0; k < 3; ++k) {
            const float ctr = data[a.union_position[k]] + data[a.shape_position[k]];
            const float hs = (so[k] * sc) * ex;
            b.bmin[k] = ctr - hs;  // from_pos_size (aabb.glsl:13-19)
            b.bmax[k] = ctr + hs;
        }
        b.back = a.back;
    }
    return PT_OK;
}

namespace {

}  // namespace

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_create(int hip_device, uint32_t width, uint32_t height, pt_ctx **out) {
    if (!out) return PT_ERR_INVALID;
    *out = nullptr;
    pt_ctx *c = new (std::nothrow) pt_ctx();
    if (!c) return PT_ERR_INVALID;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0 || hip_device < 0 || hip_device >= ndev) {
        delete c;
        return PT_ERR_HIP;
    }
    c->device = hip_device;
    if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->d_stats, sizeof(unsigned long long) * 2 * PT_ST_COUNT) != hipSuccess) {
        pt_destroy(c);
        return PT_ERR_HIP;
    }
    if (alloc_image(c, width, height) != PT_OK) {
        pt_destroy(c);
        return PT_ERR_HIP;
    }
    *out = c;
    return PT_OK;
}

int pt_resize_clear(pt_ctx *c, uint32_t width, uint32_t height) {
    if (!c) return PT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    if (width == c->width && height == c->height) {
        HIPCHK(c, hipMemsetAsync(c->accum, 0, std::max<size_t>(size_t(width) * height * 16, 16), c->stream));
        return PT_OK;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return alloc_image(c, width, height);
}

int pt_set_program(pt_ctx *c, const pt_op *ops, uint32_t n_ops, const pt_aabb *aabbs, uint32_t n_aabb,
                   uint32_t n_check) {
    if (!c) return PT_ERR_INVALID;
    if ((n_ops && !ops) || (n_aabb && !aabbs)) return fail(c, PT_ERR_INVALID, "null program arrays");
    if (n_check > PT_MAX_CHECK) return fail(c, PT_ERR_UNSUPPORTED, "more than 128 check[] entries");
    int depth = 0, max_depth = 0;
    for (uint32_t i = 0; i < n_ops; ++i) {
        const pt_op &o = ops[i];
        if (o.opcode == PT_OP_UNION_BEGIN) {
            max_depth = std::max(max_depth, ++depth);
        } else if (o.opcode == PT_OP_UNION_END) {
            if (--depth < 0) return fail(c, PT_ERR_INVALID, "unbalanced UNION_END");
            if (o.combine != PT_COMBINE_UNION && o.combine != PT_COMBINE_SUBTRACTION)
                return fail(c, PT_ERR_INVALID, "UNION_END combine must be union/subtraction");
        } else if (o.opcode == PT_OP_SHAPE) {
            if (depth < 1) return fail(c, PT_ERR_INVALID, "shape outside a union");
            if (o.shape == PT_NODE_PLANE) return fail(c, PT_ERR_UNSUPPORTED, "Shapes::Plane is not implemented upstream");
            if (o.shape < PT_NODE_SPHERE || o.shape > PT_NODE_OCTAHEDRON) return fail(c, PT_ERR_INVALID, "bad shape");
            if (o.combine > PT_COMBINE_SUBTRACTION) return fail(c, PT_ERR_INVALID, "bad combine");
            if (o.check >= int32_t(n_check)) return fail(c, PT_ERR_INVALID, "check index out of range");
        } else {
            return fail(c, PT_ERR_INVALID, "bad opcode");
        }
    }
    if (depth != 0) return fail(c, PT_ERR_INVALID, "unbalanced UNION_BEGIN");
    if (max_depth > PT_MAX_DEPTH) return fail(c, PT_ERR_UNSUPPORTED, "union nesting deeper than 8");
    for (uint32_t i = 0; i < n_aabb; ++i)
        if (aabbs[i].back < 0 || aabbs[i].back >= int32_t(n_check) || aabbs[i].so_kind > PT_SO_TORUS)
            return fail(c, PT_ERR_INVALID, "bad aabb record");
    c->ops.assign(ops, ops + n_ops);
    c->aabbs.assign(aabbs, aabbs + n_aabb);
    c->n_check = n_check;
    c->have_program = true;
    c->have_data = false;  // queue_compile reallocates data[] (sdf_editor.rs:36-40)
    return PT_OK;
}

int pt_set_data(pt_ctx *c, const float *data, uint32_t n) {
    if (!c) return PT_ERR_INVALID;
    if (!c->have_program) return fail(c, PT_ERR_STATE, "pt_set_data before pt_set_program");
    if (n && !data) return fail(c, PT_ERR_INVALID, "null data");
    std::vector<PtNode> nodes;
    std::vector<PtAabb> boxes;
    std::vector<PtMat> mats;
    std::string err;
    int rc = pt_derive(c->ops, c->aabbs, data, n, nodes, boxes, mats, err);
    if (rc != PT_OK) return fail(c, rc, err);
    HIPCHK(c, hipSetDevice(c->device));
    // stream-ordered upload: in-flight dispatches finish with the old tables
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = ensure(c, reinterpret_cast<void **>(&c->d_nodes), c->cap_nodes, nodes.size() * sizeof(PtNode))) != PT_OK)
        return rc;
    if ((rc = ensure(c, reinterpret_cast<void **>(&c->d_aabbs), c->cap_aabbs, boxes.size() * sizeof(PtAabb))) != PT_OK)
        return rc;
    if ((rc = ensure(c, reinterpret_cast<void **>(&c->d_mats), c->cap_mats, mats.size() * sizeof(PtMat))) != PT_OK)
        return rc;
    if (!nodes.empty())
        HIPCHK(c, hipMemcpyAsync(c->d_nodes, nodes.data(), nodes.size() * sizeof(PtNode), hipMemcpyHostToDevice, c->stream));
    if (!boxes.empty())
        HIPCHK(c, hipMemcpyAsync(c->d_aabbs, boxes.data(), boxes.size() * sizeof(PtAabb), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_mats, mats.data(), mats.size() * sizeof(PtMat), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->have_data = true;
    c->bound_k = pt_bound_k(nodes);
    c->fast_bounds = true;
    for (const PtAabb &b : boxes)
        for (int k = 0; k < 3; ++k)
            if (!pt_div_coord_ok(b.bmin[k]) || !pt_div_coord_ok(b.bmax[k])) c->fast_bounds = false;
    jit_refresh(c, nodes, boxes);
    return PT_OK;
}

int pt_set_tiles(pt_ctx *c, uint32_t rank, uint32_t nranks) {
    if (!c) return PT_ERR_INVALID;
    if (nranks == 0 || rank >= nranks) return fail(c, PT_ERR_INVALID, "rank must be < nranks");
    c->rank = rank;
    c->nranks = nranks;
    return pt_resize_clear(c, c->width, c->height);
}

// ---- binned pipeline (pt_binned.h) -------------------------------------------
// per sample of a chunk: two ray buffers, hit quad, bin key, binned slot,
// colour (+ the high mask words and hits' high check[] words of scenes with
// > 64 entries)
constexpr size_t kBinBytesPerSample = 2 * sizeof(PtRay) + sizeof(uint4) + 2 * sizeof(uint32_t) + sizeof(float4);
constexpr size_t kBinBytesWide = sizeof(uint2) + sizeof(float4);

static size_t bin_bytes_per_sample(const pt_ctx *c) {
    return kBinBytesPerSample + (c->n_check > 64 ? kBinBytesWide : 0);
}

// Samples per chunk: pt_set_option "bin_samples", else automatic: 2^29 (a
// whole 256-spp 1080p render: 90 GB of HBM at 168 B per sample; every pass's
// tail is paid once per chunk, so larger chunks are faster: 64 -> 256 frames
// per chunk +5 %), at most half of the device's TOTAL memory.  The total,
// not the free memory: a torch-first process's caching allocator moves the
// free figure, and every rank of a multi-GPU run must chunk its share the
// same way whatever else it holds.  Only when the
// chunk buffers then do not fit (several contexts sharing one GPU) does the
// size fall back to half of what this context could hold -- the free
// memory plus the buffers it already owns (bin_samples_free; launch_binned).
// The automatic size is fixed at the context's first binned dispatch.  The
// caller's current device is left as it was.
static bool device_mem(const pt_ctx *c, size_t &free_b, size_t &total_b) {
    free_b = total_b = 0;
    int prev = -1;
    const bool have_prev = hipGetDevice(&prev) == hipSuccess;
    const bool ok = hipSetDevice(c->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                    total_b != 0;
    if (have_prev) (void)hipSetDevice(prev);
    return ok;
}

static size_t bin_samples(pt_ctx *c) {
    if (c->bin_samples > 0) return size_t(c->bin_samples);
    if (c->bin_auto) return c->bin_auto;
    size_t free_b = 0, total_b = 0;
    if (!device_mem(c, free_b, total_b)) return size_t(1) << 27;
    const size_t cap = std::max<size_t>(size_t(1) << 20, total_b / 2 / bin_bytes_per_sample(c));
    return std::min<size_t>(size_t(1) << 29, cap);
}

// The fallback when bin_samples()'s chunk buffers did not fit: half of the
// free memory plus what this context holds (other contexts' allocations
// count as used, so ranks sharing one GPU each size to what is left).
static size_t bin_samples_free(pt_ctx *c) {
    const size_t per = bin_bytes_per_sample(c);
    size_t free_b = 0, total_b = 0;
    if (!device_mem(c, free_b, total_b)) return size_t(1) << 27;
    const size_t held = c->bin_cap * size_t(c->n_lanes) * per;
    const size_t cap = std::max<size_t>(size_t(1) << 20, (free_b + held) / 2 / per);
    return std::min<size_t>(size_t(1) << 29, cap);
}

static void free_bin(pt_ctx *c) {
    for (auto &l : c->lane) {
        (void)hipFree(l.ray[0]);
        (void)hipFree(l.ray[1]);
        (void)hipFree(l.hq);
        (void)hipFree(l.mask_hi);
        (void)hipFree(l.key);
        (void)hipFree(l.idx);
        (void)hipFree(l.hist);
        (void)hipFree(l.offs);
        (void)hipFree(l.ctrl);
        (void)hipFree(l.hitn);
        const hipStream_t s = l.stream;
        l = pt_ctx::BinLane{};
        l.stream = s;
    }
    (void)hipFree(c->d_color);
    c->d_color = nullptr;
    (void)hipFree(c->d_btab);
    c->d_btab = nullptr;
    c->n_lanes = 0;
    c->bin_cap = c->ctrl_words = 0;
}

// ensure_bin's result when the buffers' allocation itself failed (out of
// device memory): the one failure launch_binned may answer with a smaller
// chunk.  Any other HIP error (e.g. an earlier kernel's fault reported by the
// synchronisation) keeps its message and ends the dispatch.
constexpr int kBinNoMemory = -1000;

// Buffers for `lanes` pipelines of `samples` samples each.
static int ensure_bin(pt_ctx *c, size_t samples, size_t passes, int lanes) {
    const size_t words = size_t(PT_CTRL_STRIDE) * (passes + 1);
    // (mask_hi, check[] bits 64..127, exists only for scenes with > 64 entries)
    const bool hi_ok = c->n_check <= 64 || (c->n_lanes > 0 && c->lane[0].mask_hi != nullptr);
    if (samples <= c->bin_cap && words <= c->ctrl_words && lanes <= c->n_lanes && hi_ok) return PT_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));  // lane 1 joins lane 0's stream before every dispatch ends
    samples = std::max(samples, c->bin_cap);
    lanes = std::max(lanes, c->n_lanes);
    free_bin(c);
    bool ok = hipMalloc(&c->d_color, size_t(lanes) * samples * sizeof(float4)) == hipSuccess &&
              hipMalloc(&c->d_btab, (PT_BINS + 1) * sizeof(unsigned long long)) == hipSuccess;  // (+ overflow count)
    for (int i = 0; ok && i < lanes; ++i) {
        pt_ctx::BinLane &l = c->lane[i];
        ok = hipMalloc(&l.ray[0], samples * sizeof(PtRay)) == hipSuccess &&
             hipMalloc(&l.ray[1], samples * sizeof(PtRay)) == hipSuccess &&
             hipMalloc(&l.hq, samples * sizeof(uint4)) == hipSuccess &&
             (c->n_check <= 64 || hipMalloc(&l.mask_hi, samples * sizeof(uint2)) == hipSuccess) &&
             hipMalloc(&l.key, samples * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc(&l.idx, samples * sizeof(uint32_t)) == hipSuccess &&
             (c->n_check <= 64 || hipMalloc(&l.hitn, samples * sizeof(float4)) == hipSuccess) &&
             hipMalloc(&l.hist, PT_BINS * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc(&l.offs, PT_BINS * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc(&l.ctrl, words * sizeof(uint32_t)) == hipSuccess;
    }
    if (!ok) {
        free_bin(c);
        (void)hipGetLastError();
        fail(c, PT_ERR_HIP, "out of device memory for the binned pipeline");
        return kBinNoMemory;
    }
    if (!c->fork_ev) HIPCHK(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
    c->lane[0].stream = c->stream;
    for (int i = 1; i < lanes; ++i) {
        if (!c->xstream[i]) HIPCHK(c, hipStreamCreateWithFlags(&c->xstream[i], hipStreamNonBlocking));
        if (!c->join_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming));
        c->lane[i].stream = c->xstream[i];
    }
    for (int i = 0; i < lanes; ++i) {
        HIPCHK(c, hipMemsetAsync(c->lane[i].hist, 0, PT_BINS * sizeof(uint32_t), c->stream));
        HIPCHK(c, hipMemsetAsync(c->lane[i].ctrl, 0, words * sizeof(uint32_t), c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->n_lanes = lanes;
    c->bin_cap = samples;
    c->ctrl_words = words;
    if (!c->cu_count) HIPCHK(c, hipDeviceGetAttribute(&c->cu_count, hipDeviceAttributeMultiprocessorCount, c->device));
    return PT_OK;
}

static hipError_t record_event(pt_ctx::EventLog &g, hipStream_t stream) {
    if (g.used == g.ev.size()) {
        hipEvent_t e;
        const hipError_t err = hipEventCreate(&e);
        if (err != hipSuccess) return err;
        g.ev.push_back(e);
    }
    return hipEventRecord(g.ev[g.used++], stream);
}

// Summed elapsed time of the log's (start, end) pairs; blocks for the last.
static hipError_t event_log_ms(pt_ctx::EventLog &g, double *sum) {
    *sum = 0.0;
    if (!g.used) return hipSuccess;
    hipError_t e = hipEventSynchronize(g.ev[g.used - 1]);
    for (size_t i = 0; e == hipSuccess && i + 1 < g.used; i += 2) {
        float ms = 0.0f;
        e = hipEventElapsedTime(&ms, g.ev[i], g.ev[i + 1]);
        *sum += ms;
    }
    return e;
}

// One dispatch chunk through the pass pipeline: frames are processed in
// sub-chunks of at most bin_samples() samples.
static int launch_binned(pt_ctx *c, PtLaunch &L, bool stats) {
    const uint32_t n_pix = uint32_t(L.n_tiles) * 64u;
    int32_t frame0 = L.frame0, lc0 = L.last_clear0;
    uint32_t spp = uint32_t(L.spp);
    if (L.debug != 0) {  // direct stores: only the last frame survives (as the other kernels)
        frame0 = int32_t(uint32_t(frame0) + spp - 1);
        lc0 = int32_t(uint32_t(lc0) + spp - 1);
        spp = 1;
    }
    if (!c->bin_samples && !c->bin_auto) c->bin_auto = bin_samples(c);  // (fixed from now on)
    const int passes = L.bounces + 1;
    uint32_t F = 0, FL = 0;
    int lanes = 0;
    auto size_chunk = [&]() {
        F = uint32_t(std::max<size_t>(1, std::min<size_t>(spp, bin_samples(c) / n_pix)));
        lanes = int(std::min<uint32_t>(uint32_t(c->bin_lanes), F));
        FL = (F + uint32_t(lanes) - 1) / uint32_t(lanes);  // frames per lane
    };
    size_chunk();
    int rc = ensure_bin(c, size_t(n_pix) * FL, size_t(passes), lanes);
    if (rc == kBinNoMemory && !c->bin_samples && !c->bin_fallback) {
        // the total-memory size does not fit (contexts sharing the GPU):
        // size to the free memory once, fixed from now on
        c->bin_fallback = true;
        c->bin_auto = bin_samples_free(c);
        c->err.clear();
        size_chunk();
        rc = ensure_bin(c, size_t(n_pix) * FL, size_t(passes), lanes);
    }
    if (rc == kBinNoMemory) rc = PT_ERR_HIP;  // (the message is in c->err)
    if (rc != PT_OK) return rc;
    if (!stats) c->last_chunks = (spp + F - 1) / F;
    const unsigned cu = unsigned(std::max(1, c->cu_count));
    auto item_grid = [&](size_t n) {
        return unsigned(std::max<size_t>(1, std::min<size_t>((n + PT_BIN_BLOCK - 1) / PT_BIN_BLOCK, 4 * cu)));
    };
    // scatter: 4 blocks per CU (8 / 16 measured equal), each one contiguous
    // run of PT_SCATTER_ITEMS-slot tiles
    auto scatter_grid = [&](size_t n) {
        const size_t tile = PT_BIN_BLOCK * PT_SCATTER_ITEMS;
        return unsigned(std::max<size_t>(1, std::min<size_t>((n + tile - 1) / tile, size_t(4) * cu)));
    };
    const PtJitModule *jm = jit_active(c);
    const bool jit = jm != nullptr;
    // the set table's overflow count covers the whole dispatch (the table
    // itself is cleared per chunk, below)
    const bool use_table = c->bin_table && c->n_check > uint32_t(PT_BIN_BITS) && c->n_check <= 64;
    if (use_table && stats) HIPCHK(c, hipMemsetAsync(c->d_btab + PT_BINS, 0, sizeof(unsigned long long), c->stream));
    if (!stats) c->btab_used = use_table;
    if (stats) c->btab_counted = use_table;
    // normal taps in the shade pass: march-only trace + tapping shade (scene kernels)
    const bool taps_shade = jit && c->shade_taps;
    hipFunction_t jf = jit ? (taps_shade ? (stats ? jm->trace_m_stats : jm->trace_m)
                                         : (stats ? jm->trace_stats : jm->trace))
                           : nullptr;
    int per_cu = 0;
    if (jit) HIPCHK(c, hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, jf, 64, 0));
    else per_cu = pt_bin_trace_blocks_per_cu(stats);
    // leave one wave slot per SIMD (4 per CU) to the other pipeline, so its
    // shade / scatter / scan blocks run beside the persistent trace waves
    // instead of waiting for a pass to drain: 28 of 32 with the 64-VGPR
    // (8-wave) build (+1.5 % over 24 of 28 at 72 VGPRs), 24 of 28 with the
    // 72-VGPR fallback (+1.5 % over 28 of 28)
    if (per_cu > 8) per_cu = std::min(per_cu - 4, 28);
    const unsigned trace_grid = cu * unsigned(std::max(1, per_cu));
    // the first pass's kernel may have been rebuilt at 7 waves on its own
    // (pt_jit_compile_source): the same one-slot-per-SIMD rule on its occupancy
    unsigned trace_g_grid = trace_grid;
    if (jit && jm->trace_g) {
        int g = 0;
        HIPCHK(c, hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&g, jm->trace_g, 64, 0));
        if (g > 8) g = std::min(g - 4, 28);
        if (g > 0 && g < per_cu) trace_g_grid = cu * unsigned(g);
    }
    // trace runs of at most 512 rays (256 / 768 / 1024 equal, 128 -7 %), a
    // refill once 2 lanes are free (1 / 4 equal)
    constexpr int run_max = 512, refill_min = 2;
    // two rounds of the tapping shade kernel's 7 resident blocks per CU
    // (measured +2 % over 8, whose last round ran on a quarter of the chip;
    // 8 / 16 at 8 waves -0.3 %); 8 for the table kernel
    const unsigned shade_cu = taps_shade ? 14u : 8u;
    const unsigned shade_grid =
        unsigned(std::max<size_t>(1, std::min<size_t>((c->bin_cap + PT_BIN_BLOCK - 1) / PT_BIN_BLOCK, size_t(shade_cu) * cu)));

    for (uint32_t done = 0; done < spp; done += F) {
        const uint32_t fr = std::min(F, spp - done);
        // the chunk's frames over the lanes: lane i renders fl[i] frames from
        // frame offset fo[i]; its colours land in the chunk's colour buffer
        // at that frame offset, so one fold mixes all of them in frame order
        const int nl = int(std::min<uint32_t>(uint32_t(lanes), fr));
        uint32_t fl[pt_ctx::kMaxLanes], fo[pt_ctx::kMaxLanes];
        for (int i = 0; i < nl; ++i) {
            fl[i] = fr / uint32_t(nl) + (uint32_t(i) < fr % uint32_t(nl) ? 1u : 0u);
            fo[i] = i == 0 ? 0u : fo[i - 1] + fl[i - 1];
        }
        // the table of check[] sets starts empty per chunk (bin_resolve: only
        // scenes whose sets do not fit the bin index use it)
        unsigned long long *btab = nullptr;
        if (use_table) {
            btab = c->d_btab;
            HIPCHK(c, hipMemsetAsync(btab, 0, PT_BINS * sizeof(unsigned long long), c->stream));
        }
        PtPass P[pt_ctx::kMaxLanes];
        for (int i = 0; i < nl; ++i) {
            const pt_ctx::BinLane &l = c->lane[i];
            PtPass &p = P[i];
            std::memset(&p, 0, sizeof p);
            p.L = L;
            p.L.frame0 = int32_t(uint32_t(frame0) + done + fo[i]);
            p.L.last_clear0 = int32_t(uint32_t(lc0) + done + fo[i]);
            p.L.spp = int32_t(fl[i]);
            p.rin = l.ray[0];
            p.rout = l.ray[1];
            p.hq = l.hq;
            p.mask_hi = l.mask_hi;
            p.key = l.key;
            p.idx = l.idx;
            p.hist = l.hist;
            p.offs = l.offs;
            p.color = c->d_color + size_t(fo[i]) * n_pix;
            p.hitn = l.hitn;
            p.ctrl = l.ctrl;
            p.n_src = nullptr;
            p.n_src_const = uint32_t(size_t(n_pix) * fl[i]);
            p.n_pix = int32_t(n_pix);
            p.frames = int32_t(fl[i]);
            p.wide = c->n_check > 64 ? 1 : 0;
            p.btab = btab;
            p.count_overflow = stats ? 1 : 0;
            p.run_max = run_max;
            p.refill_min = refill_min;
        }
        if (nl > 1) {  // lanes 1.. start after everything enqueued on the context stream so far
            HIPCHK(c, hipEventRecord(c->fork_ev, c->stream));
            for (int i = 1; i < nl; ++i) HIPCHK(c, hipStreamWaitEvent(c->lane[i].stream, c->fork_ev, 0));
        }
        // the first pass takes the primary rays in generation order (gen lists
        // them, the host sets the count; no histogram, scan or scatter: +1 %)
        // -- only when every local tile lies inside the image: then every
        // generated slot is live and the list is the identity order
        const bool full_tiles = L.width % PT_TILE == 0 && L.height % PT_TILE == 0 && L.debug == 0;
        for (int i = 0; i < nl && full_tiles; ++i) {
            P[i].gen_order = 1;
            // pass 0's control words = {count, run cursors 0}: stream-ordered
            // fills, no host buffer whose lifetime the copy would have to outlast
            HIPCHK(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->lane[i].ctrl), 0, PT_CTRL_STRIDE,
                                        c->lane[i].stream));
            HIPCHK(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->lane[i].ctrl), int(P[i].n_src_const), 1,
                                        c->lane[i].stream));
        }
        // no gen pass: the first trace pass makes its windows' camera rays
        // itself (scene kernels, generation order: +2.8 %); otherwise the
        // scene's gen kernel (straight-line bounds(): +1.4 % over the AOT one)
        if (!stats) c->gen_trace_used = c->gen_norec_used = 0;
        for (int i = 0; i < nl; ++i) {
            if (P[i].gen_order && jit && taps_shade && !stats && jm->trace_g) {
                P[i].gen_trace = 1;
                P[i].gen_norec = c->n_check <= 32 ? 1 : 0;  // (the check[] bits ride in the hit quad)
                c->gen_trace_used = 1;
                c->gen_norec_used = P[i].gen_norec;
            } else if (jit) {
                void *args[] = {&P[i]};
                HIPCHK(c, hipModuleLaunchKernel(stats ? jm->gen_stats : jm->gen, item_grid(size_t(P[i].n_src_const)), 1,
                                                1, PT_BIN_BLOCK, 1, 1, 0, c->lane[i].stream, args, nullptr));
            } else {
                pt_launch_bin(PtBinStage::Gen, P[i], stats, item_grid(size_t(P[i].n_src_const)), c->lane[i].stream);
                HIPCHK(c, hipGetLastError());
            }
        }
        // shade the hits of trace pass k (its hit quads and the rays it traced,
        // ray[k & 1]; or, taps in the trace pass, its hit records in
        // ray[(k + 1) & 1]): ended paths store their colour, the rest get
        // their next ray in ray[(k + 1) & 1], bounds() and bin
        auto shade = [&](int i, int k) -> int {
            PtPass S = P[i];
            S.bounce = k;
            S.rin = c->lane[i].ray[k & 1];
            S.rout = c->lane[i].ray[(k + 1) & 1];
            S.n_src = c->lane[i].ctrl + size_t(PT_CTRL_STRIDE) * k;
            if (!stats) HIPCHK(c, record_event(c->slog, c->lane[i].stream));
            if (taps_shade) {
                void *args[] = {&S};
                HIPCHK(c, hipModuleLaunchKernel(stats ? jm->shade_t_stats : jm->shade_t, shade_grid, 1, 1, PT_BIN_BLOCK,
                                                1, 1, 0, c->lane[i].stream, args, nullptr));
            } else {
                pt_launch_bin(PtBinStage::Shade, S, stats, shade_grid, c->lane[i].stream);
                HIPCHK(c, hipGetLastError());
            }
            if (!stats) HIPCHK(c, record_event(c->slog, c->lane[i].stream));
            return PT_OK;
        };
        for (int k = 0; k < passes; ++k) {
            for (int i = 0; i < nl; ++i) {
                // pass k: bin the rays of ray[k & 1] (gen's, or the shaded hits of pass k-1), trace them into the other
                const pt_ctx::BinLane &l = c->lane[i];
                PtPass &p = P[i];
                if (k > 0 && (rc = shade(i, k - 1)) != PT_OK) return rc;
                const bool gt = k == 0 && p.gen_trace;
                if (k > 0) p.gen_trace = p.gen_norec = 0;  // (shade pass 0 above still had them)
                p.bounce = k;
                p.rin = l.ray[k & 1];
                p.rout = l.ray[(k + 1) & 1];
                p.ctrl = l.ctrl + size_t(PT_CTRL_STRIDE) * k;
                p.n_src = k == 0 ? nullptr : l.ctrl + size_t(PT_CTRL_STRIDE) * (k - 1);
                if (k > 0 || !p.gen_order) {
                    pt_launch_bin(PtBinStage::Scan, p, stats, 1, l.stream);
                    pt_launch_bin(PtBinStage::Scatter, p, stats, scatter_grid(k == 0 ? p.n_src_const : c->bin_cap),
                                  l.stream);
                    HIPCHK(c, hipGetLastError());
                }
                if (!stats) HIPCHK(c, record_event(c->tlog, l.stream));
                if (jit) {
                    void *args[] = {&p};
                    HIPCHK(c, hipModuleLaunchKernel(gt ? jm->trace_g : jf, gt ? trace_g_grid : trace_grid, 1, 1, 64, 1,
                                                    1, 0, l.stream, args,
                                                    nullptr));
                } else {
                    pt_launch_bin(PtBinStage::Trace, p, stats, trace_grid, l.stream);
                    HIPCHK(c, hipGetLastError());
                }
                if (!stats) HIPCHK(c, record_event(c->tlog, l.stream));
            }
        }
        for (int i = 0; i < nl; ++i)  // the last bounce's hits end their paths
            if ((rc = shade(i, passes - 1)) != PT_OK) return rc;
        for (int i = 1; i < nl; ++i) {  // the fold (and everything after) waits for every lane
            HIPCHK(c, hipEventRecord(c->join_ev[i], c->lane[i].stream));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->join_ev[i], 0));
        }
        PtPass Fp = P[0];
        Fp.L.frame0 = int32_t(uint32_t(frame0) + done);
        Fp.L.last_clear0 = int32_t(uint32_t(lc0) + done);
        Fp.L.spp = int32_t(fr);
        Fp.color = c->d_color;
        Fp.frames = int32_t(fr);
        Fp.lanes = nl;  // (the colour regions' split: bin_fold_body)
        pt_launch_bin(PtBinStage::Fold, Fp, stats, unsigned((n_pix + PT_BIN_BLOCK - 1) / PT_BIN_BLOCK), c->stream);
        HIPCHK(c, hipGetLastError());
    }
    return PT_OK;
}

static bool use_binned(const PtLaunch &L) { return L.kernel == PT_KERNEL_BINNED && !pt_use_simple_kernel(L); }

// Launch one chunk: the scene-specialised wavefront kernel when loaded, else
// the ahead-of-time kernels (pt_kernel.hip).
static int launch(pt_ctx *c, PtLaunch &L, bool stats) {
    if (use_binned(L)) return launch_binned(c, L, stats);
    const PtJitModule *jm = jit_active(c);
    if (!pt_use_simple_kernel(L) && jm) {
        void *args[] = {&L};
        HIPCHK(c, hipModuleLaunchKernel(stats ? jm->render_stats : jm->render, unsigned(L.n_tiles), 1, 1,
                                        64, 1, 1, 0, c->stream, args, nullptr));
    } else {
        pt_launch_render(L, stats, c->stream);
        HIPCHK(c, hipGetLastError());
    }
    return PT_OK;
}

static int make_launch(pt_ctx *c, const pt_constants *k, const pt_settings *s, uint32_t spp, PtLaunch &L) {
    if (!c) return PT_ERR_INVALID;
    if (!k || !s) return fail(c, PT_ERR_INVALID, "null constants/settings");
    if (!c->have_program || !c->have_data) return fail(c, PT_ERR_STATE, "no program/data uploaded");
    if (s->bounces < 0) return fail(c, PT_ERR_INVALID, "negative bounces");
    std::memset(&L, 0, sizeof L);
    L.nodes = c->d_nodes;
    L.aabbs = c->d_aabbs;
    L.fast_bounds = c->fast_bounds ? 1 : 0;
    L.bound_k = c->bound_k;
    L.mats = c->d_mats;
    L.accum = c->accum;
    L.n_nodes = int32_t(c->ops.size());
    L.n_aabb = int32_t(c->aabbs.size());
    L.width = int32_t(c->width);
    L.height = int32_t(c->height);
    L.tiles_x = int32_t((c->width + PT_TILE - 1) / PT_TILE);
    const int64_t tiles = int64_t(L.tiles_x) * int64_t((c->height + PT_TILE - 1) / PT_TILE);
    L.n_tiles = int32_t(tiles > int64_t(c->rank) ? (tiles - int64_t(c->rank) + c->nranks - 1) / c->nranks : 0);
    L.rank = int32_t(c->rank);
    L.nranks = int32_t(c->nranks);
    L.frame0 = k->frame;
    L.last_clear0 = k->last_clear;
    L.spp = int32_t(spp);
    L.debug = s->debug;
    L.bounces = s->bounces;
    L.fov = s->fov;
    L.aspect = k->aspect;
    L.write = 1;
    L.kernel = c->kernel;
    if (L.kernel == PT_KERNEL_AUTO) {
        // small dispatches take the tile-resident wave kernel: one launch, no
        // pass sequence and no per-pass tails.  Crossover measured at about
        // samples x ops = 2^27 (scripts/kernel_crossover.py: C1 3x faster at
        // 65 K samples; the 32-node scene binned from ~4 M samples on)
        const double work = double(L.n_tiles) * 64.0 * double(spp) * double(std::max<size_t>(1, c->ops.size()));
        L.kernel = work < 134217728.0 ? PT_KERNEL_WAVEFRONT : PT_KERNEL_BINNED;
    }
    L.shade_batch = c->shade_batch;
    return PT_OK;
}

int pt_dispatch(pt_ctx *c, const pt_constants *k, const pt_settings *s, uint32_t spp) {
    PtLaunch L;
    int rc = make_launch(c, k, s, spp, L);
    if (rc != PT_OK) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    jit_tier_poll(c, false);  // switch to the values-baked kernel once it is built
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    c->tlog.used = c->slog.used = 0;
    if (spp > 0 && L.n_tiles > 0) {
        // bound a single launch's length; chunks continue frame/last_clear.
        // The binned pipeline takes every frame at once: it splits by its own
        // sample budget, and larger chunks mean fuller passes (at N GPUs each
        // rank owns 1/N of the pixels and renders N times the frames).
        const uint32_t chunk = use_binned(L) ? spp : 64;
        for (uint32_t done = 0; done < spp; done += chunk) {
            PtLaunch Lc = L;
            Lc.spp = int32_t(std::min(chunk, spp - done));
            Lc.frame0 = int32_t(uint32_t(L.frame0) + done);
            Lc.last_clear0 = int32_t(uint32_t(L.last_clear0) + done);
            if (L.debug != 0 && done + chunk < spp) continue;  // direct stores: only the last frame survives
            if ((rc = launch(c, Lc, false)) != PT_OK) return rc;
        }
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    return PT_OK;
}

int pt_dispatch_stats(pt_ctx *c, const pt_constants *k, const pt_settings *s, uint32_t spp,
                      uint64_t counters[PT_STAT_COUNT]) {
    static_assert(PT_STAT_COUNT >= PT_ST_COUNT, "stat count");
    PtLaunch L;
    int rc = make_launch(c, k, s, spp, L);
    if (rc != PT_OK) return rc;
    if (!counters) return fail(c, PT_ERR_INVALID, "null counters");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * 2 * PT_ST_COUNT, c->stream));
    L.stats = c->d_stats;
    L.write = 0;
    if (spp > 0 && L.n_tiles > 0)
        if ((rc = launch(c, L, true)) != PT_OK) return rc;
    unsigned long long host[2 * PT_ST_COUNT];  // [0, COUNT): everything else; [COUNT, 2 COUNT): shade-pass taps
    HIPCHK(c, hipMemcpyAsync(host, c->d_stats, sizeof host, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < PT_STAT_COUNT; ++i) counters[i] = i < PT_ST_COUNT ? host[i] + host[PT_ST_COUNT + i] : 0;
    for (int i = 0; i < PT_ST_COUNT; ++i) c->tap_stats[i] = host[PT_ST_COUNT + i];
    return PT_OK;
}

int pt_read_accum(pt_ctx *c, float *rgba, size_t bytes) {
    if (!c) return PT_ERR_INVALID;
    const size_t need = size_t(c->width) * c->height * 16;
    if (!rgba || bytes < need) return fail(c, PT_ERR_SIZE, "readback buffer too small");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(rgba, c->accum, need, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_write_accum(pt_ctx *c, const float *rgba, size_t bytes) {
    if (!c) return PT_ERR_INVALID;
    const size_t need = size_t(c->width) * c->height * 16;
    if (!rgba || bytes < need) return fail(c, PT_ERR_SIZE, "image buffer too small");
    HIPCHK(c, hipSetDevice(c->device));
    if (need) HIPCHK(c, hipMemcpyAsync(c->accum, rgba, need, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_display(pt_ctx *c, int format, void *out, size_t bytes) {
    if (!c) return PT_ERR_INVALID;
    if (format != PT_DISPLAY_RGBA32F && format != PT_DISPLAY_SRGB8) return fail(c, PT_ERR_INVALID, "bad display format");
    const size_t need = size_t(c->width) * c->height * (format == PT_DISPLAY_RGBA32F ? 16 : 4);
    if (!out || bytes < need) return fail(c, PT_ERR_SIZE, "display buffer too small");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure(c, &c->d_display, c->cap_display, std::max<size_t>(need, 16));
    if (rc != PT_OK) return rc;
    if (!c->dev0) {
        HIPCHK(c, hipEventCreate(&c->dev0));
        HIPCHK(c, hipEventCreate(&c->dev1));
    }
    HIPCHK(c, hipEventRecord(c->dev0, c->stream));
    pt_launch_display(c->accum, c->width, c->height, format, c->d_display, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->dev1, c->stream));
    c->display_timed = true;
    if (need) HIPCHK(c, hipMemcpyAsync(out, c->d_display, need, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_accum_device_ptr(pt_ctx *c, void **dev_ptr, size_t *bytes) {
    if (!c || !dev_ptr || !bytes) return PT_ERR_INVALID;
    *dev_ptr = c->accum;
    *bytes = size_t(c->width) * c->height * 16;
    return PT_OK;
}

int pt_get_size(const pt_ctx *c, uint32_t *w, uint32_t *h) {
    if (!c || !w || !h) return PT_ERR_INVALID;
    *w = c->width;
    *h = c->height;
    return PT_OK;
}

int pt_comm_get_unique_id(uint8_t id[PT_COMM_ID_BYTES]) {
    if (!id) return PT_ERR_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PT_ERR_RCCL;
    std::memcpy(id, u.internal, PT_COMM_ID_BYTES);
    return PT_OK;
}

int pt_comm_init(pt_ctx *c, uint32_t nranks, uint32_t rank, const uint8_t id[PT_COMM_ID_BYTES]) {
    if (!c || !id || nranks == 0 || rank >= nranks) return fail(c, PT_ERR_INVALID, "bad communicator arguments");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->comm) {
        ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, PT_COMM_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&c->comm, int(nranks), u, int(rank));
    if (r != ncclSuccess) return fail(c, PT_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    c->comm_nranks = nranks;
    return PT_OK;
}

int pt_comm_size(pt_ctx *c, uint32_t *nranks) {
    if (!c || !nranks) return PT_ERR_INVALID;
    if (!c->comm) return fail(c, PT_ERR_STATE, "pt_comm_init not called");
    int n = 0;
    ncclResult_t r = ncclCommCount(c->comm, &n);
    if (r != ncclSuccess) return fail(c, PT_ERR_RCCL, std::string("ncclCommCount: ") + ncclGetErrorString(r));
    *nranks = uint32_t(n);
    return PT_OK;
}

int pt_reduce_accum(pt_ctx *c, int root) {
    if (!c) return PT_ERR_INVALID;
    if (!c->comm) return fail(c, PT_ERR_STATE, "pt_comm_init not called");
    if (root < 0 || uint32_t(root) >= c->comm_nranks) return fail(c, PT_ERR_INVALID, "bad root");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t count = size_t(c->width) * c->height * 4;
    if (!c->reduced) HIPCHK(c, hipMalloc(&c->reduced, std::max<size_t>(count * 4, 16)));
    // non-owned texels are exactly 0 on every other rank, so the sum is the
    // bit-exact single-GPU image (x + 0 = x)
    ncclResult_t r = ncclReduce(c->accum, c->reduced, count, ncclFloat32, ncclSum, root, c->comm, c->stream);
    if (r != ncclSuccess) return fail(c, PT_ERR_RCCL, std::string("ncclReduce: ") + ncclGetErrorString(r));
    return PT_OK;
}

int pt_read_reduced(pt_ctx *c, float *rgba, size_t bytes) {
    if (!c) return PT_ERR_INVALID;
    if (!c->reduced) return fail(c, PT_ERR_STATE, "no reduced image");
    const size_t need = size_t(c->width) * c->height * 16;
    if (!rgba || bytes < need) return fail(c, PT_ERR_SIZE, "readback buffer too small");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(rgba, c->reduced, need, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_sync(pt_ctx *c) {
    if (!c) return PT_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_last_dispatch_ms(pt_ctx *c, float *ms) {
    if (!c || !ms) return PT_ERR_INVALID;
    if (!c->timed) return fail(c, PT_ERR_STATE, "no dispatch recorded");
    HIPCHK(c, hipEventSynchronize(c->ev1));
    HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    return PT_OK;
}

int pt_set_option(pt_ctx *c, const char *key, int value) {
    if (!c || !key) return PT_ERR_INVALID;
    if (!std::strcmp(key, "kernel")) {
        if (value < PT_KERNEL_AUTO || value > PT_KERNEL_BINNED) return fail(c, PT_ERR_INVALID, "bad kernel id");
        c->kernel = value;
        return PT_OK;
    }
    if (!std::strcmp(key, "jit")) {
        if (value != 0 && value != 1) return fail(c, PT_ERR_INVALID, "jit must be 0 or 1");
        c->jit = value;
        if (!value) {  // re-enabled on the next pt_set_data
            pt_jit_unload(c->jit_mod);
            pt_jit_unload(c->jit_tier);
            c->tier_want.clear();
        }
        return PT_OK;
    }
    if (!std::strcmp(key, "jit_bake")) {
        if (value < 0 || value > 2) return fail(c, PT_ERR_INVALID, "jit_bake must be 0, 1 or 2");
        c->jit_bake = value;  // takes effect at the next pt_set_data
        return PT_OK;
    }
    if (!std::strcmp(key, "jit_wait")) {  // block until a pending tier-up build is installed
        HIPCHK(c, hipSetDevice(c->device));
        jit_tier_poll(c, true);
        return PT_OK;
    }
    if (!std::strcmp(key, "bin_samples")) {
        if (value < 64) return fail(c, PT_ERR_INVALID, "bin_samples must be >= 64");
        c->bin_samples = value;
        return PT_OK;
    }
    if (!std::strcmp(key, "bin_lanes")) {
        if (value < 1 || value > pt_ctx::kMaxLanes) return fail(c, PT_ERR_INVALID, "bin_lanes must be in [1, 4]");
        c->bin_lanes = value;
        return PT_OK;
    }
    if (!std::strcmp(key, "bin_table")) {
        if (value < 0 || value > 1) return fail(c, PT_ERR_INVALID, "bin_table must be 0 or 1");
        c->bin_table = value;
        return PT_OK;
    }
    if (!std::strcmp(key, "shade_taps")) {
        if (value < 0 || value > 1) return fail(c, PT_ERR_INVALID, "shade_taps must be 0 or 1");
        c->shade_taps = value;
        return PT_OK;
    }
    if (!std::strcmp(key, "shade_batch")) {
        if (value < 1 || value > 64) return fail(c, PT_ERR_INVALID, "shade_batch must be in [1, 64]");
        c->shade_batch = value;
        return PT_OK;
    }
    return fail(c, PT_ERR_INVALID, std::string("unknown option ") + key);
}

int pt_get_option(pt_ctx *c, const char *key, double *value) {
    if (!c || !key || !value) return PT_ERR_INVALID;
    if (!std::strcmp(key, "jit_active")) *value = jit_active(c) ? 1.0 : 0.0;
    else if (!std::strcmp(key, "jit_tier_active")) *value = c->jit_tier.module ? 1.0 : 0.0;
    else if (!std::strcmp(key, "jit_tier_seconds")) *value = c->tier_seconds;
    else if (!std::strcmp(key, "jit_seconds")) *value = c->jit_seconds;
    else if (!std::strcmp(key, "jit_trace_waves") || !std::strcmp(key, "jit_shade_waves")) {
        // waves per SIMD the scene kernel in use can hold: 8 = the 8-wave build
        // (<= 64 VGPRs), 7 = the rebuild after a spill (pt_jit_compile_source)
        const PtJitModule *m = jit_active(c);
        const bool tr = key[4] == 't';
        const hipFunction_t f = m ? (tr ? m->trace_m : m->shade_t) : nullptr;
        const int threads = tr ? 64 : PT_BIN_BLOCK;
        int blocks = 0;
        if (f && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, f, threads, 0) != hipSuccess) blocks = 0;
        *value = double(blocks) * (threads / 64) / 4.0;  // (4 SIMDs per CU)
    }
    else if (!std::strcmp(key, "kernel")) *value = c->kernel;
    else if (!std::strcmp(key, "shade_batch")) *value = c->shade_batch;
    else if (!std::strcmp(key, "bin_samples")) *value = double(bin_samples(c));
    else if (!std::strcmp(key, "bin_chunks")) *value = double(c->last_chunks);  // of the last timed binned dispatch
    else if (!std::strcmp(key, "bin_fallback")) *value = c->bin_fallback ? 1.0 : 0.0;
    else if (!std::strcmp(key, "bin_sets") || !std::strcmp(key, "bin_overflow")) {
        // the table of check[] sets (-1: not in use): bin_sets, the distinct
        // sets the last chunk of the last dispatch claimed slots for;
        // bin_overflow, the lookups of the last instrumented dispatch
        // (pt_dispatch_stats) whose set found no slot within PT_BIN_PROBES
        // and shared its hash bin (pt_binned.h bin_resolve)
        *value = -1.0;
        const bool sets = key[4] == 's';
        if ((sets ? c->btab_used : c->btab_counted) && c->d_btab) {
            std::vector<unsigned long long> t(PT_BINS + 1);
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipMemcpy(t.data(), c->d_btab, t.size() * sizeof(t[0]), hipMemcpyDeviceToHost));
            if (sets) *value = double(std::count_if(t.begin(), t.end() - 1, [](unsigned long long v) { return v != 0ull; }));
            else *value = double(t.back());
        }
    }
    else if (!std::strcmp(key, "trace_launches")) *value = double(c->tlog.used / 2);
    else if (!std::strcmp(key, "shade_launches")) *value = double(c->slog.used / 2);
    else if (!std::strcmp(key, "display_ms")) {
        float ms = 0.0f;
        if (c->display_timed) HIPCHK(c, hipEventElapsedTime(&ms, c->dev0, c->dev1));
        *value = ms;
    }
    else if (!std::strcmp(key, "trace_ms")) HIPCHK(c, event_log_ms(c->tlog, value));  // summed over the trace passes
    else if (!std::strcmp(key, "shade_ms")) HIPCHK(c, event_log_ms(c->slog, value));  // summed over the shade passes
    else if (!std::strcmp(key, "bin_bytes")) *value = double(c->bin_cap) * double(c->n_lanes) * double(bin_bytes_per_sample(c));
    else if (!std::strcmp(key, "bin_lanes")) *value = double(c->bin_lanes);
    else if (!std::strcmp(key, "bin_table")) *value = double(c->bin_table);
    else if (!std::strcmp(key, "shade_taps")) *value = c->shade_taps ? 1.0 : 0.0;
    else if (!std::strcmp(key, "jit_cache")) {
        // where the scene kernel in use came from: 1 the shipped on-disk cache
        // (lib/jitcache), 0 this process's hipRTC, -1 none loaded
        *value = c->jit_tier.module ? c->tier_from : (c->jit_mod.module ? c->jit_from : -1);
    }
    else if (!std::strcmp(key, "gen_trace")) *value = double(c->gen_trace_used);
    else if (!std::strcmp(key, "gen_norec")) *value = double(c->gen_norec_used);
    else if (!std::strncmp(key, "tap_stat_", 9)) {  // tap_stat_<k>: counter k of the last stats run's shade-pass taps
        const int k = std::atoi(key + 9);
        if (k < 0 || k >= PT_ST_COUNT) return fail(c, PT_ERR_INVALID, "tap_stat index out of range");
        *value = double(c->tap_stats[k]);
    }
    else return fail(c, PT_ERR_INVALID, std::string("unknown option ") + key);
    return PT_OK;
}

const char *pt_jit_log(const pt_ctx *c) { return c ? c->jit_log.c_str() : ""; }

const char *pt_last_error(const pt_ctx *c) { return c ? c->err.c_str() : "null context"; }

void pt_destroy(pt_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->tier_job.valid()) c->tier_job.wait();
    pt_jit_unload(c->jit_mod);
    pt_jit_unload(c->jit_tier);
    (void)hipFree(c->accum);
    (void)hipFree(c->reduced);
    (void)hipFree(c->d_nodes);
    (void)hipFree(c->d_aabbs);
    (void)hipFree(c->d_mats);
    (void)hipFree(c->d_stats);
    free_bin(c);
    for (int i = 1; i < pt_ctx::kMaxLanes; ++i) {
        if (c->xstream[i]) (void)hipStreamDestroy(c->xstream[i]);
        if (c->join_ev[i]) (void)hipEventDestroy(c->join_ev[i]);
    }
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (hipEvent_t e : c->tlog.ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->slog.ev) (void)hipEventDestroy(e);
    (void)hipFree(c->d_display);
    if (c->dev0) (void)hipEventDestroy(c->dev0);
    if (c->dev1) (void)hipEventDestroy(c->dev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

}  // extern "C"
