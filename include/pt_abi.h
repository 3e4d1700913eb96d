/*
 * pt_abi.h -- C ABI of the MI355X-native SDF path-trace hot path.
 *
 * This is the drop-in boundary that replaces the wgpu objects owned by the
 * reference's `PathTracer` (src/path_tracer/path_tracer.rs:18-163), the
 * `data[]` storage buffer of `DataArray` (src/sdf_editor/primitives.rs:59-157)
 * and the GLSL text that `SDFEditor::compile` (src/sdf_editor/sdf_editor.rs:
 * 186-246) splices into the compute shader.  Plain C types only; every entry
 * point returns a status code (PT_OK = 0); `pt_last_error` explains failures.
 * Inputs are borrowed and copied before return; outputs are caller-owned.
 * Calls on one context are not re-entrant (the reference is single-threaded,
 * src/inbuilt/event_loop.rs:7-76).  See INTEGRATION.md for the Rust binding.
 */
#ifndef PT_ABI_H
#define PT_ABI_H

#ifndef __HIPCC_RTC__ /* also embedded in the hipRTC-compiled scene kernels */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 1

/* status codes */
#define PT_OK 0
#define PT_ERR_INVALID -1      /* bad argument / malformed program or scene */
#define PT_ERR_HIP -2          /* HIP runtime failure */
#define PT_ERR_UNSUPPORTED -3  /* e.g. Shapes::Plane (containers.rs:287,295 emits NotImplemented) */
#define PT_ERR_STATE -4        /* program/data missing, wrong call order */
#define PT_ERR_RCCL -5         /* collective failure */
#define PT_ERR_SIZE -6         /* caller buffer too small (required size written back) */

typedef struct pt_ctx pt_ctx;

/* == `Constants` UBO (path_tracer.rs:149-155, test_compute.glsl:6-11), 16 B */
typedef struct {
    float time;
    int32_t frame;
    float aspect;
    int32_t last_clear;
} pt_constants;

/* == `Settings` UBO (path_tracer.rs:157-163, test_compute.glsl:13-19), 20 B */
typedef struct {
    int32_t debug;   /* 0 path trace, 1 normals, 2 albedo, 3 bounce heat map */
    int32_t bounces;
    float scale;
    float fov;
    int32_t aabb;    /* unused by the kernel, as upstream */
} pt_settings;

/* ---------------------------------------------------------------------
 * Scene tree (the SDFEditor node graph, flattened) -> compiled program
 * --------------------------------------------------------------------- */
#define PT_NODE_UNION 0       /* containers.rs:8-15 */
#define PT_NODE_SPHERE 1      /* containers.rs:260 */
#define PT_NODE_CUBE 2        /* containers.rs:261 */
#define PT_NODE_TORUS 3       /* extension: BASELINE.json config 2 (absent upstream) */
#define PT_NODE_OCTAHEDRON 4  /* shapes.glsl:13-25 (deprecated editor format) */
#define PT_NODE_PLANE 5       /* containers.rs:262, unimplemented upstream -> PT_ERR_UNSUPPORTED */

#define PT_UNION_TYPE_UNION 0       /* containers.rs:244-252 */
#define PT_UNION_TYPE_SUBTRACTION 1

/* One Union or Shape.  A union's children are the later nodes whose `parent`
 * is its index, in array order; parent -1 = SDFEditor.header_unions. */
typedef struct {
    int32_t kind;
    int32_t parent;
    int32_t union_type;
    int32_t aabb;               /* Transform.aabb */
    float scale;                /* Transform.scale */
    float position[3];
    float rotation[3];
    float aabb_exaggeration;
    float size[3];              /* sphere [0]; cube xyz; torus (R, r); octahedron [0] */
    float material[18];         /* Material in Mat order (test_compute.glsl:45-59) */
} pt_scene_node;

#define PT_OP_UNION_BEGIN 0
#define PT_OP_SHAPE 1
#define PT_OP_UNION_END 2

#define PT_COMBINE_ASSIGN 0       /* UnionType::compile index 0 (containers.rs:245-247) */
#define PT_COMBINE_UNION 1        /* opUnion, shapes.glsl:72-74 */
#define PT_COMBINE_SUBTRACTION 2  /* opSubtraction, shapes.glsl:76-81 */

/* One statement of the generated `map()`; operands are data[] slot indices.
 * Replaces the GLSL text of Union::compile / Shape::compile. */
typedef struct {
    uint32_t opcode;
    uint32_t shape;          /* PT_NODE_* for SHAPE */
    uint32_t combine;        /* how the result joins the enclosing accumulator */
    int32_t check;           /* check[] index guarding a SHAPE, -1 = `if (true)` */
    uint32_t scale;
    uint32_t position[3];
    uint32_t rotation[3];
    uint32_t aabb_exaggeration;
    uint32_t size[3];
    uint32_t material[18];
} pt_op;

#define PT_SO_SCALAR 0  /* vec3(size[0])  sphere, octahedron */
#define PT_SO_VEC3 1    /* size.xyz       cube */
#define PT_SO_ONE 2     /* vec3(1.0)      (Plane; never reached) */
#define PT_SO_TORUS 3   /* extension: vec3(R + r, r, R + r) */

/* One `if (bool_hit(intersectAABB(...))) back[i] = true;` of the generated
 * `bounds()` (Shape::aabb_compile, containers.rs:442-463). */
typedef struct {
    int32_t back;
    uint32_t so_kind;
    uint32_t union_position[3];
    uint32_t union_scale;
    uint32_t shape_position[3];
    uint32_t shape_scale;
    uint32_t size[3];
    uint32_t aabb_exaggeration;
} pt_aabb;

/* Compile a scene tree exactly as SDFEditor::compile allocates data[] slots
 * and check[] indices (sdf_editor.rs:186-246).  Two-call pattern: any output
 * pointer may be NULL, sizes are always written; returns PT_ERR_SIZE if a
 * capacity is too small.  Host-only, no GPU needed.  Every Float gets its
 * own slot (the editor draws a fresh random hash per Float,
 * primitives.rs:12-17,220). */
int pt_compile_scene(const pt_scene_node *nodes, uint32_t n_nodes,
                     pt_op *ops, uint32_t ops_cap, uint32_t *n_ops,
                     pt_aabb *aabbs, uint32_t aabb_cap, uint32_t *n_aabb,
                     float *data, uint32_t data_cap, uint32_t *n_data,
                     uint32_t *n_check);

/* The identity of one Float: its serde `hash` (u128, primitives.rs:210).
 * DataArray::get_index (primitives.rs:117-129) gives Floats that share a hash
 * one data[] slot, holding the first one's value (cloned nodes and edited
 * JSON files share hashes).  {0, 0} = anonymous: always a fresh slot. */
typedef struct {
    uint64_t lo, hi;
} pt_float_key;
/* Keys per node: scale, position xyz, rotation xyz, aabb_exaggeration,
 * size[3], material[18] (a union uses the first 8). */
#define PT_NODE_FLOATS 29
/* pt_compile_scene with the Floats' hashes: keys[node * PT_NODE_FLOATS + k]
 * (NULL = all anonymous, the same as pt_compile_scene). */
int pt_compile_scene_keyed(const pt_scene_node *nodes, uint32_t n_nodes, const pt_float_key *keys,
                           pt_op *ops, uint32_t ops_cap, uint32_t *n_ops,
                           pt_aabb *aabbs, uint32_t aabb_cap, uint32_t *n_aabb,
                           float *data, uint32_t data_cap, uint32_t *n_data,
                           uint32_t *n_check);

/* ---------------------------------------------------------------------
 * Render context
 * --------------------------------------------------------------------- */
/* == StorageTexturePackage::new (structs.rs:113-160): RGBA32F image, zeroed.
 * Device memory is row-major, row y = 0 first, 16 B per texel. */
int pt_create(int hip_device, uint32_t width, uint32_t height, pt_ctx **out);
/* == StorageTexturePackage::remake + `last_clear = 0` (path_tracer.rs:101-106) */
int pt_resize_clear(pt_ctx *ctx, uint32_t width, uint32_t height);
/* == PathTracer::remake_pipeline(map) (path_tracer.rs:62-76): topology change */
int pt_set_program(pt_ctx *ctx, const pt_op *ops, uint32_t n_ops, const pt_aabb *aabbs, uint32_t n_aabb,
                   uint32_t n_check);
/* == DataArray::update (primitives.rs:131-151): value-only update, no recompile */
int pt_set_data(pt_ctx *ctx, const float *data, uint32_t n);
/* Multi-GPU tile ownership (new): 8x8 tile t is rendered iff t % nranks == rank.
 * Clears the image (non-owned texels stay exactly 0). */
int pt_set_tiles(pt_ctx *ctx, uint32_t rank, uint32_t nranks);
/* == `spp` successive (PathTracer::update, compute_pass) pairs: frame j uses
 * frame = c->frame + j and last_clear = c->last_clear + j (path_tracer.rs:
 * 110-111).  Asynchronous, ordered on the context's HIP stream. */
int pt_dispatch(pt_ctx *ctx, const pt_constants *c, const pt_settings *s, uint32_t spp);
/* == State::save_image readback (state.rs:237-303): blocking copy of the
 * local image (w*h*4 floats) into a caller buffer. */
int pt_read_accum(pt_ctx *ctx, float *rgba, size_t bytes);
/* Inverse of pt_read_accum (new): replace the local image with w*h*4 floats
 * from a caller buffer (resume a progressive render from a saved image, or
 * feed the display pass).  Blocking. */
int pt_write_accum(pt_ctx *ctx, const float *rgba, size_t bytes);
/* == the pixel transform of State::save_image (state.rs:277-289), host only:
 * `rgba` (w*h*4 floats, row 0 = y 0, as pt_read_accum returns it) to the
 * 8-bit RGBA of image.png, row 0 = top (rows flipped, :283): r, g, b =
 * (v.powf(1.0 / 2.2) * 255.0) as u8 with Rust's f32 1.0 / 2.2 and libm powf,
 * a = (v * 255.0) as u8; `as u8` saturates (NaN -> 0).  `out` holds w*h*4
 * bytes. */
int pt_save_rgba8(const float *rgba, uint32_t width, uint32_t height, uint8_t *out, size_t bytes);
/* Device pointer + size of the local image (for external collectives). */
int pt_accum_device_ptr(pt_ctx *ctx, void **dev_ptr, size_t *bytes);
int pt_get_size(const pt_ctx *ctx, uint32_t *width, uint32_t *height);

/* RCCL over xGMI (new).  The 128-byte id is produced on one rank and
 * broadcast by the caller's own channel (e.g. torch.distributed). */
#define PT_COMM_ID_BYTES 128
int pt_comm_get_unique_id(uint8_t id[PT_COMM_ID_BYTES]);
int pt_comm_init(pt_ctx *ctx, uint32_t nranks, uint32_t rank, const uint8_t id[PT_COMM_ID_BYTES]);
/* Ranks of the context's communicator as RCCL reports them (ncclCommCount):
 * the check that an N-GPU run reduced over N ranks.  PT_ERR_STATE before
 * pt_comm_init. */
int pt_comm_size(pt_ctx *ctx, uint32_t *nranks);
/* Sum of every rank's image into this context's result image on `root`
 * (out of place: the local accumulation keeps progressing). */
int pt_reduce_accum(pt_ctx *ctx, int root);
int pt_read_reduced(pt_ctx *ctx, float *rgba, size_t bytes);

int pt_sync(pt_ctx *ctx);
/* Device time (HIP events on the context stream) of the kernels of the last
 * pt_dispatch, in ms; blocks until they finished. */
int pt_last_dispatch_ms(pt_ctx *ctx, float *ms);
/* Instrumented re-run of one dispatch (does not touch the image): per-event
 * work counters for algorithmic-flop accounting, in the order
 * of compute_path_tracer_amd/_native.py STAT_NAMES. */
#define PT_STAT_COUNT 32
int pt_dispatch_stats(pt_ctx *ctx, const pt_constants *c, const pt_settings *s, uint32_t spp,
                      uint64_t counters[PT_STAT_COUNT]);
/* Display pass (replaces RenderTexturePipeline::render_pass,
 * render_texture_pipeline.rs:77-110 + render_texture_shader.wgsl:23-94):
 * ACESFilm + LinearToSRGB of the accumulation image.
 *   PT_DISPLAY_RGBA32F: fs_main's vec4 per texel, texel order (row 0 =
 *     bottom), w*h*16 bytes;
 *   PT_DISPLAY_SRGB8: the 8-bit RGBA the sRGB swapchain (setup.rs:53-59)
 *     stores -- encoded a second time, the reference's double-sRGB -- in
 *     screen order (row 0 = top), w*h*4 bytes.
 * Blocking; the output buffer is caller-owned (host memory). */
#define PT_DISPLAY_RGBA32F 0
#define PT_DISPLAY_SRGB8 1
int pt_display(pt_ctx *ctx, int format, void *out, size_t bytes);
/* Tuning knobs: "kernel" (0 auto = 3, 1 simple one-path-per-lane, 2 tile-
 * resident wavefront state machine, 3 mask-binned passes: per bounce, the
 * rays of a chunk of frames are grouped by their bounds() check set before
 * they are marched), "shade_batch" (state-machine kernels: lanes that must
 * wait before a shading pass runs, 1..64), "bin_samples" (binned kernel:
 * samples per chunk, >= 64; device memory = 168 B per sample, 192 B for
 * scenes with > 64 check[] entries; default 2^29 samples, at most half of
 * the device's total memory -- or, when that does not fit beside other
 * contexts on the same GPU, half of what this context could hold -- fixed at
 * the context's first binned dispatch), "bin_lanes"
 * (binned kernel: 1..4 pipelines, each on its own stream, over which a
 * chunk's frames are split, so one's memory-bound passes overlap another's
 * trace pass), "bin_table" (binned kernel, scenes with 13..64 check[]
 * entries: 1, the default, bins each set in a slot of its own from a table
 * of the sets seen; 0: hashed bins, which two sets share now and then), "jit" (1:
 * per-scene hipRTC build of the state-machine kernels, compiled at
 * pt_set_data when the topology or an identity flag changed -- the analogue
 * of remake_pipeline; 0: op-list interpreter), "jit_bake" (0: node values
 * read from the table; 1: baked into the kernel as literals, recompiled on
 * every value edit; 2, the default: tier-up -- the table kernel runs at
 * once, and a values-baked build compiled on a worker thread replaces it
 * while the values stay unchanged) and "jit_wait" (block until a pending
 * tier-up build is installed).  Results are bit-identical for every value. */
int pt_set_option(pt_ctx *ctx, const char *key, int value);
/* Read back: "jit_active" (1 when the scene-specialised kernel is loaded),
 * "jit_seconds" (last hipRTC compile time), "jit_tier_active" /
 * "jit_tier_seconds" (values-baked build in use / its compile time),
 * "kernel", "shade_batch",
 * "bin_samples", "bin_lanes", "bin_table", "bin_bytes" (device memory held by the binned
 * pipeline), "bin_chunks" (chunks of the last binned dispatch), "bin_fallback"
 * (1: the chunk size came from the free memory), "trace_ms" / "trace_launches" (device time and count of the last
 * dispatch's binned trace passes, HIP events on each pipeline's stream),
 * "shade_ms" / "shade_launches" (the same for its shade passes), "display_ms"
 * (device time of the last pt_display's kernel), "gen_trace" / "gen_norec"
 * (the last timed binned dispatch's first pass made its own camera rays /
 * and stored no ray records for shade pass 0). */
int pt_get_option(pt_ctx *ctx, const char *key, double *value);
/* Log of the last failed scene-kernel build ("" if none). */
const char *pt_jit_log(const pt_ctx *ctx);
/* Build the scene-specialised kernel for (program, data) with hipRTC without
 * a device (validation / cache warm-up); *code_bytes = code object size. */
int pt_jit_compile(const pt_op *ops, uint32_t n_ops, const pt_aabb *aabbs, uint32_t n_aabb, const float *data,
                   uint32_t n_data, char *log, size_t log_cap, size_t *code_bytes);
/* The scene kernel source pt_jit_compile would build for (program, data),
 * without compiling it (the counterpart of the reference's spliced-shader dump
 * shader_out/test_compute.glsl, glsl_preprocessor.rs:5-15).  baked != 0: node
 * values as literals (the tier-up build).  Host only; two-call pattern, *len
 * includes the terminating NUL. */
int pt_scene_kernel_source(const pt_op *ops, uint32_t n_ops, const pt_aabb *aabbs, uint32_t n_aabb,
                           const float *data, uint32_t n_data, int baked, char *out, size_t cap, size_t *len);
const char *pt_last_error(const pt_ctx *ctx);
void pt_destroy(pt_ctx *ctx);
int pt_abi_version(void);

/* Device arithmetic probes for the semantics contract (tests only):
 * out[i] = op(a[i], b[i]) computed by the kernels' own device functions. */
#define PT_MATH_MAX 0
#define PT_MATH_MIN 1
#define PT_MATH_SQRT 2   /* the kernels' fast correctly rounded sqrt */
#define PT_MATH_SQRTF 3  /* the compiler's IEEE sqrtf */
#define PT_MATH_SIN 4
#define PT_MATH_COS 5
#define PT_MATH_DIV 6
#define PT_MATH_FMA 7    /* fmaf(a, b, 1) */
int pt_device_math(int hip_device, int op, const float *a, const float *b, float *out, uint32_t n);
/* The kernels' sqrt vs IEEE sqrtf over all 2^32 inputs (NaN payloads aside). */
int pt_check_sqrt_exhaustive(int hip_device, uint64_t *mismatches, uint32_t *first_bad);
/* bounds()' reciprocal division (q = a*y, r = fma(-q,b,a), fma(r,y,q) with
 * y = 1/b) vs IEEE a / b for every a = 1.(a0..a0+na-1), b = 1.(b0..b0+nb-1)
 * significand pair (na, nb <= 2^23); first_bad = b bits << 32 | a bits. */
int pt_check_div_exhaustive(int hip_device, uint32_t a0, uint32_t na, uint32_t b0, uint32_t nb,
                            uint64_t *mismatches, uint64_t *first_bad);
/* The same on n random operands drawn inside the bounds() guards (a = x - o
 * of two guarded coordinates, guarded divisor); a zero quotient may differ in
 * sign only. */
int pt_check_div_random(int hip_device, uint32_t seed, uint32_t n, uint64_t *mismatches, uint64_t *first_bad);
/* The margin-decided slab test of bounds() on n random
 * guarded (box, ray) pairs; mode 1 puts the ray through a box edge (near
 * ties).  counts[0]: decided pairs whose answer differs from the IEEE slab
 * test, [1]: undecided pairs whose exact fallback differs, [2]: undecided
 * pairs, [3]: pairs drawn outside the guards (skipped). */
int pt_check_box_random(int hip_device, uint32_t seed, uint32_t n, int mode, uint64_t *counts);
/* Self-test: pt_div_k(a, b, RN(1/b)) (the baked scene kernels' division by a
 * scale constant, |b| in [2^-4, 2^4]) against the IEEE a / b, bit for bit,
 * for the na patterns a0 .. a0 + na - 1 (na a multiple of 256). */
int pt_check_div_k(int hip_device, float b, uint32_t a0, uint32_t na, uint64_t *mismatches, uint64_t *first_bad);
/* Calibration probes for rocprofv3's FETCH_SIZE / WRITE_SIZE on the
 * pipeline's access shapes (pt_probe.hip): 2^log2n items (16..26) of, in
 * order, a 64 B record gather, a 16 B coalesced read, a 16 B scattered store
 * and a 64 B record store; ms[k] = device time, bytes[k] = bytes moved. */
int pt_traffic_probe(int hip_device, uint32_t log2n, float ms[4], uint64_t bytes[4]);

#ifdef __cplusplus
}
#endif
#endif
