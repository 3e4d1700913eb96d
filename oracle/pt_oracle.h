/*
 * pt_oracle.h -- CPU restatement of the reference path-trace hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * path in compute_path_tracer_amd/csrc and the CPU baseline leg of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product path never links, calls or falls back to it.
 *
 * What it restates (file:line in zachdedoo13/compute_path_tracer @ 2024-10-08):
 *   - the compute kernel  assets/shaders/path_tracer/test_compute.glsl:26-246
 *   - rng.glsl:1-36, funcs.glsl:1-35, shapes.glsl:1-81, aabb.glsl:1-33
 *   - the scene -> GLSL code generator whose OUTPUT is part of the hot path:
 *       src/sdf_editor/sdf_editor.rs:186-246   (map()/bounds() skeleton)
 *       src/sdf_editor/containers.rs:143-202,244-252,404-463
 *       src/sdf_editor/data_structures.rs:45-96,178-194
 *       src/sdf_editor/primitives.rs:53-56,117-129 (data[] slot allocation)
 *   - the per-frame counters   src/path_tracer/path_tracer.rs:97-118
 * The scene is taken as the editor TREE (not as a compiled op list), so the
 * oracle allocates data[] slots and walks the tree itself, independently of
 * the product's scene compiler.
 *
 * Parity status: the reference (Rust + wgpu + naga GLSL) cannot be built or
 * run in this environment and ships no tests or golden outputs for this path,
 * so floating-point parity with the real GLSL-on-driver is UNPINNED.  Pinned:
 * the data[] slot / check[] topology against the one captured compiler output
 * (assets/shaders/path_tracer/shader_out/test_compute.glsl:185-392), and the
 * integer RNG.  Builtins whose precision the GLSL spec leaves to the driver
 * are fixed by the semantics contract in DESIGN.md section 3 (IEEE f32,
 * correctly rounded + - * / sqrt, no FMA contraction, GLSL-spec min/max,
 * pto_sin/pto_cos polynomial below).
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Editor node kinds.  UNION = containers.rs:8-15; SPHERE/CUBE/PLANE =
 * containers.rs:259-264; OCTAHEDRON = shapes.glsl:13-25 (deprecated editor);
 * TORUS = build extension (BASELINE.json config 2; absent upstream). */
enum { PTO_UNION = 0, PTO_SPHERE = 1, PTO_CUBE = 2, PTO_TORUS = 3, PTO_OCTAHEDRON = 4, PTO_PLANE = 5 };
enum { PTO_TYPE_UNION = 0, PTO_TYPE_SUBTRACTION = 1 };

/* One editor node (Union or Shape), flattened.  Children of a union are the
 * nodes whose parent is that union, in array order (unions and shapes keep
 * their own relative order, as Union.children_unions / children_shapes). */
typedef struct {
    int32_t kind;
    int32_t parent;       /* -1: SDFEditor.header_unions */
    int32_t union_type;   /* unions only */
    int32_t aabb;         /* Transform.aabb */
    float scale;
    float pos[3];
    float rot[3];
    float aabb_ex;
    float size[3];        /* sphere: [0]; cube: xyz; torus: R, r; octahedron: [0] */
    float mat[18];        /* Mat order, test_compute.glsl:45-59 */
} pto_node;

typedef struct { float time; int32_t frame; float aspect; int32_t last_clear; } pto_constants;
typedef struct { int32_t debug; int32_t bounces; float scale; float fov; int32_t aabb; } pto_settings;

/* Work counters (algorithmic-flop accounting). */
typedef struct {
    uint64_t samples;          /* camera paths */
    uint64_t segments;         /* bounds()+CastRay() pairs */
    uint64_t march_steps;      /* map() calls inside CastRay */
    uint64_t normal_maps;      /* map() calls inside calc_normal */
    uint64_t shaded;           /* segments that reached shading */
    uint64_t aabb_tests;       /* slab tests executed */
    uint64_t xform_union;      /* union transforms evaluated */
    uint64_t xform_shape;      /* shape transforms evaluated (check passed) */
    uint64_t sdf[6];           /* per kind, index = PTO_* */
    uint64_t comb_union;       /* opUnion */
    uint64_t comb_sub;         /* opSubtraction */
    uint64_t comb_assign;
    uint64_t rr_break;
} pto_counters;

typedef struct pto_scene pto_scene;

/* Compile the tree: allocate data[] slots exactly like SDFEditor::compile.
 * Returns 0, or -1 on an invalid tree, -2 for Shapes::Plane (NotImplemented). */
int  pto_scene_build(const pto_node *nodes, int n, pto_scene **out);
/* With the Floats' u128 hashes, keys[(node * 29 + k) * 2 + {0: lo, 1: hi}]
 * in the node's slot order (8 transform, 3 size, 18 material); {0, 0} =
 * anonymous.  Shared hashes share a data[] slot (primitives.rs:117-129). */
int  pto_scene_build_keyed(const pto_node *nodes, int n, const uint64_t *keys, pto_scene **out);
void pto_scene_free(pto_scene *s);
int  pto_scene_n_data(const pto_scene *s);
int  pto_scene_n_check(const pto_scene *s);
void pto_scene_get_data(const pto_scene *s, float *out);
int  pto_scene_set_data(pto_scene *s, const float *data, int n);   /* value-only refresh */
/* Slot table per node: 8 transform slots + size[3] + mat[18] (-1 = none) and
 * the check index used by map() (-1 = `if (true)`), bounds() index. */
void pto_scene_node_slots(const pto_scene *s, int node, int32_t *slots29, int32_t *check, int32_t *bounds_idx);

/* Kernel pieces (for KATs). */
uint32_t pto_wang_hash(uint32_t *state);
float    pto_random01(uint32_t *state);
uint32_t pto_gen_rng(int32_t x, int32_t y, int32_t frame, int32_t w, int32_t h);
float    pto_sin(float x);
float    pto_cos(float x);
float    pto_map(const pto_scene *s, const float p[3], const uint8_t *check, int32_t *shape);
void     pto_bounds(const pto_scene *s, const float ro[3], const float rd[3], uint8_t *check, float debug[3]);

/* Render `spp` successive frames into image[h][w][4] (row y=0 first), frame
 * j using constants.frame + j and last_clear + j (path_tracer.rs:110-111).
 * Only tiles t (8x8, row-major over ceil(w/8)) with t % nranks == rank are
 * touched.  Rows with (y % row_stride) != 0 are skipped (CPU baseline sample).
 * nthreads <= 0: one thread. counters may be NULL. */
void pto_render(const pto_scene *s, float *image, int w, int h,
                const pto_constants *c, const pto_settings *st, int spp,
                int rank, int nranks, int row_stride, int nthreads,
                pto_counters *counters);

/* Display pass, render_texture_shader.wgsl:23-94 (+ the sRGB swapchain,
 * setup.rs:53-59), under DESIGN.md's display contract: pow in double with
 * fixed series and fma, rounded once to f32.  fmt 0: fs_main's RGBA32F per
 * texel (texel order); fmt 1: 8-bit RGBA as the sRGB surface stores it,
 * screen order (row 0 = top = texel row h-1). */
void pto_display(const float *image, int w, int h, int fmt, void *out);
float pto_pow_pos(float x, float y);

/* Analysis aid: log every path segment (ray, check mask, march steps) of
 * subsequent single-threaded renders into buf (counters must be requested). */
typedef struct { float ro[3], rd[3]; uint64_t mask[2]; int32_t seg, steps, hit, pad; } pto_segment;
void pto_set_segment_log(pto_segment *buf, int cap);
int pto_segment_log_count(void);

#ifdef __cplusplus
}
#endif
#endif
