// pt_device.h -- device-resident scene layout and launch parameters.
//
// The compiled program (pt_op list + data[]) is expanded on the host, once
// per pt_set_data, into three small read-only tables:
//   PtNode  one per op: opcode/combine/check + the op's derived constants
//           (1/s, pos*(1/s), per-axis cos/sin) -- exactly the values the
//           generated GLSL recomputes from data[] on every map() call
//           (data_structures.rs:45-55, shapes.glsl:34-68), hoisted.
//   PtAabb  one per `if (bool_hit(...))` of bounds(): its box min/max
//           (data_structures.rs:68-92, aabb.glsl:13-19), hoisted.
//   PtMat   material table; index 0 = MDEF (test_compute.glsl:63).
// Hoisting is bit-exact: the host evaluates the same f32 expressions with the
// same rounding (IEEE f32, no contraction) as the kernel would.
#pragma once

#ifndef __HIPCC_RTC__
#include <cstdint>
#endif

#include "pt_math.h"  // (hipRTC: provides the fixed-width typedefs)
#include "pt_abi.h"

#define PT_MAX_DEPTH 8      // union nesting supported by the interpreter
#define PT_MAX_CHECK 128    // check[] entries (two 64-bit lane masks)
#define PT_TILE 8           // one wave64 = one 8x8 pixel tile

enum : uint32_t {
    PT_NF_SCALE = 1u << 0,  // 1/s != 1
    PT_NF_POS = 1u << 1,    // pos*(1/s) != 0
    PT_NF_RX = 1u << 2,     // rotation about x is not the identity
    PT_NF_RY = 1u << 3,
    PT_NF_RZ = 1u << 4,
};

struct PtNode {  // 96 B
    int32_t op;
    int32_t shape;
    int32_t combine;
    int32_t check;
    int32_t mat;
    uint32_t flags;
    float inv;
    float m[3];
    float cx, sx, cy, sy, cz, sz;
    float size[3];
    float pad[5];
};
static_assert(sizeof(PtNode) == 96, "PtNode layout");

struct PtAabb {  // 32 B
    float bmin[3];
    float bmax[3];
    int32_t back;
    int32_t pad;
};
static_assert(sizeof(PtAabb) == 32, "PtAabb layout");

struct PtMat {  // 48 B
    float col[3];
    float spec;
    float spec_col[3];
    float rough2;    // roughness * roughness (test_compute.glsl:139)
    float emis[3];   // normalize(light) * brightness (test_compute.glsl:146)
    float pad;
};
static_assert(sizeof(PtMat) == 48, "PtMat layout");

// Work counters of the instrumented kernel variant (pt_dispatch_stats).
enum {
    PT_ST_SAMPLES = 0,
    PT_ST_SEGMENTS,
    PT_ST_MARCH,
    PT_ST_NORMAL_MAPS,
    PT_ST_SHADED,
    PT_ST_AABB,
    PT_ST_XFORM_UNION,
    PT_ST_XFORM_SHAPE,
    PT_ST_SDF_SPHERE,
    PT_ST_SDF_CUBE,
    PT_ST_SDF_TORUS,
    PT_ST_SDF_OCTA,
    PT_ST_COMB_UNION,
    PT_ST_COMB_SUB,
    PT_ST_COMB_ASSIGN,
    PT_ST_RR_BREAK,
    PT_ST_WAVE_MAPS,    // wave-level map() executions (one per wave per call)
    PT_ST_WAVE_SHAPES,  // wave-level shape evaluations (>= 1 lane passed check[])
    PT_ST_WAVE_ITERS,   // wavefront kernel loop iterations (per wave)
    PT_ST_LANE_IDLE,    // lanes without map work in an iteration (wavefront kernel)
    PT_ST_IDLE_SHADE,   //   ... of which waiting for a shading pass
    PT_ST_IDLE_FREE,    //   ... of which without a job (pool drained / ring full)
    PT_ST_CYC_REFILL,   // wave clock cycles (s_memtime) spent per phase: job refill + camera rays
    PT_ST_CYC_BOUNDS,   //   bounds() redistribution
    PT_ST_CYC_MAP,      //   map() + state update
    PT_ST_CYC_SHADE,    //   shading + fold
    PT_ST_CYC_TOTAL,    //   whole wave
    PT_ST_CULLED,       // lane shape evaluations dropped by the distance bound (counted in the kinds above too)
    PT_ST_WAVE_EVALS,   // wave-level shape evaluations that ran (WAVE_SHAPES minus whole-wave culls)
    PT_ST_BOUNDS_WAVES, // waves that ran bounds()' fast slab tests (first active lane counts)
    PT_ST_BOUNDS_EXACT, // of those, waves with an undecided lane, which redid every box exactly
    PT_ST_SHADED_FIRST, // hits shaded in the binned pipeline's shade pass 0 (the first segment's hits)
    PT_ST_COUNT
};

struct PtLaunch {
    const PtNode *nodes;
    const PtAabb *aabbs;
    const PtMat *mats;
    float *accum;            // [height][width][4]
    unsigned long long *stats;  // non-null only for the instrumented variant
    int32_t n_nodes;
    int32_t n_aabb;
    int32_t width;
    int32_t height;
    int32_t tiles_x;
    int32_t n_tiles;         // tiles owned by this rank
    int32_t rank;
    int32_t nranks;
    int32_t frame0;
    int32_t last_clear0;
    int32_t spp;
    int32_t debug;
    int32_t bounces;
    float fov;
    float aspect;
    int32_t write;           // 0: instrumented run, leave the image untouched
    int32_t kernel;          // PT_KERNEL_* (0 = choose)
    int32_t shade_batch;     // wavefront kernel: shade when >= this many lanes wait
    int32_t fast_bounds;     // every box coordinate passes pt_div_coord_ok (reciprocal slab divisions allowed)
    float bound_k;           // map() bound margin: the scene's transform-chain magnitude (NaN: no bound; pt_bound_k)
};

#define PT_KERNEL_AUTO 0
#define PT_KERNEL_SIMPLE 1     // one path per lane, reference loop structure
#define PT_KERNEL_WAVEFRONT 2  // per-lane state machine with job refill
#define PT_KERNEL_BINNED 3     // per-bounce passes over mask-binned rays (pt_binned.h)
#ifndef PT_RING
#define PT_RING 4              // wavefront kernel: in-flight samples per pixel (power of 2)
#endif
