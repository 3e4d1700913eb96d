/*
 * abi_harness.c -- a compiled C caller of include/pt_abi.h (VERDICT r04 item
 * 6; SURVEY.md 7 step 3's "C++ host harness" beside the ctypes driver).
 *
 * Built by the tests with `gcc -std=c11 -Wall -Werror -pedantic` against
 * compute_path_tracer_amd/lib/libpt.so.  It is what the reference's Rust host
 * (path_tracer.rs:28-146, primitives.rs:131-151) would do through the
 * INTEGRATION.md `extern "C"` block, in C:
 *
 *   layout            the struct sizes and field offsets, also fixed at
 *                     compile time by the _Static_asserts below (the Rust
 *                     #[repr(C)] block of INTEGRATION.md 2 lays them out the
 *                     same way); prints them for the test to compare with
 *                     ctypes
 *   compile           pt_compile_scene of BASELINE config 1's scene (the
 *                     editor's default Union + Sphere(1.0), brightness 1,
 *                     sdf_editor.rs:20-33) with the two-call pattern; prints
 *                     the program (no GPU needed)
 *   render FIXTURE    GPU: pt_create -> pt_set_program -> pt_set_data ->
 *                     pt_dispatch (32x32, 2 spp, 1 bounce, frame 1) ->
 *                     pt_read_accum, compared bit for bit with the committed
 *                     oracle image FIXTURE (.npy, float32 [32][32][4])
 *
 * Exit status 0 on success; anything else prints the reason on stderr.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pt_abi.h"

/* == Constants (path_tracer.rs:149-155), Settings (:157-163) */
_Static_assert(sizeof(pt_constants) == 16, "pt_constants is 16 B");
_Static_assert(offsetof(pt_constants, time) == 0 && offsetof(pt_constants, frame) == 4 &&
                   offsetof(pt_constants, aspect) == 8 && offsetof(pt_constants, last_clear) == 12,
               "pt_constants fields");
_Static_assert(sizeof(pt_settings) == 20, "pt_settings is 20 B");
_Static_assert(offsetof(pt_settings, debug) == 0 && offsetof(pt_settings, bounces) == 4 &&
                   offsetof(pt_settings, scale) == 8 && offsetof(pt_settings, fov) == 12 &&
                   offsetof(pt_settings, aabb) == 16,
               "pt_settings fields");
/* the flattened SDFEditor node and the generated map() statement: 132 B */
_Static_assert(sizeof(pt_scene_node) == 132, "pt_scene_node is 132 B");
_Static_assert(offsetof(pt_scene_node, kind) == 0 && offsetof(pt_scene_node, parent) == 4 &&
                   offsetof(pt_scene_node, union_type) == 8 && offsetof(pt_scene_node, aabb) == 12 &&
                   offsetof(pt_scene_node, scale) == 16 && offsetof(pt_scene_node, position) == 20 &&
                   offsetof(pt_scene_node, rotation) == 32 && offsetof(pt_scene_node, aabb_exaggeration) == 44 &&
                   offsetof(pt_scene_node, size) == 48 && offsetof(pt_scene_node, material) == 60,
               "pt_scene_node fields");
_Static_assert(sizeof(pt_op) == 132, "pt_op is 132 B");
_Static_assert(offsetof(pt_op, opcode) == 0 && offsetof(pt_op, shape) == 4 && offsetof(pt_op, combine) == 8 &&
                   offsetof(pt_op, check) == 12 && offsetof(pt_op, scale) == 16 && offsetof(pt_op, position) == 20 &&
                   offsetof(pt_op, rotation) == 32 && offsetof(pt_op, aabb_exaggeration) == 44 &&
                   offsetof(pt_op, size) == 48 && offsetof(pt_op, material) == 60,
               "pt_op fields");
/* one bounds() statement: 56 B */
_Static_assert(sizeof(pt_aabb) == 56, "pt_aabb is 56 B");
_Static_assert(offsetof(pt_aabb, back) == 0 && offsetof(pt_aabb, so_kind) == 4 &&
                   offsetof(pt_aabb, union_position) == 8 && offsetof(pt_aabb, union_scale) == 20 &&
                   offsetof(pt_aabb, shape_position) == 24 && offsetof(pt_aabb, shape_scale) == 36 &&
                   offsetof(pt_aabb, size) == 40 && offsetof(pt_aabb, aabb_exaggeration) == 52,
               "pt_aabb fields");
_Static_assert(sizeof(pt_float_key) == 16 && offsetof(pt_float_key, hi) == 8, "pt_float_key is u128 lo, hi");

#define FIELD(T, f) printf("  \"%s.%s\": [%u, %u],\n", #T, #f, (unsigned)offsetof(T, f), (unsigned)sizeof(((T *)0)->f))

static int layout(void) {
    printf("{\n");
    FIELD(pt_constants, time);
    FIELD(pt_constants, frame);
    FIELD(pt_constants, aspect);
    FIELD(pt_constants, last_clear);
    FIELD(pt_settings, debug);
    FIELD(pt_settings, bounces);
    FIELD(pt_settings, scale);
    FIELD(pt_settings, fov);
    FIELD(pt_settings, aabb);
    FIELD(pt_scene_node, kind);
    FIELD(pt_scene_node, parent);
    FIELD(pt_scene_node, union_type);
    FIELD(pt_scene_node, aabb);
    FIELD(pt_scene_node, scale);
    FIELD(pt_scene_node, position);
    FIELD(pt_scene_node, rotation);
    FIELD(pt_scene_node, aabb_exaggeration);
    FIELD(pt_scene_node, size);
    FIELD(pt_scene_node, material);
    FIELD(pt_op, opcode);
    FIELD(pt_op, shape);
    FIELD(pt_op, combine);
    FIELD(pt_op, check);
    FIELD(pt_op, scale);
    FIELD(pt_op, position);
    FIELD(pt_op, rotation);
    FIELD(pt_op, aabb_exaggeration);
    FIELD(pt_op, size);
    FIELD(pt_op, material);
    FIELD(pt_aabb, back);
    FIELD(pt_aabb, so_kind);
    FIELD(pt_aabb, union_position);
    FIELD(pt_aabb, union_scale);
    FIELD(pt_aabb, shape_position);
    FIELD(pt_aabb, shape_scale);
    FIELD(pt_aabb, size);
    FIELD(pt_aabb, aabb_exaggeration);
    FIELD(pt_float_key, lo);
    FIELD(pt_float_key, hi);
    printf("  \"sizes\": [%u, %u, %u, %u, %u, %u]\n}\n", (unsigned)sizeof(pt_constants),
           (unsigned)sizeof(pt_settings), (unsigned)sizeof(pt_scene_node), (unsigned)sizeof(pt_op),
           (unsigned)sizeof(pt_aabb), (unsigned)sizeof(pt_float_key));
    return 0;
}

/* BASELINE config 1: SDFEditor::new's default scene (sdf_editor.rs:20-33):
 * one Union, one Sphere of radius 1.0, AABB on with exaggeration 1.3
 * (data_structures.rs Transform defaults), the default material with
 * brightness 1 (so the image is not black). */
static void c1_scene(pt_scene_node n[2]) {
    memset(n, 0, 2 * sizeof n[0]);
    n[0].kind = PT_NODE_UNION;
    n[0].parent = -1;
    n[0].union_type = PT_UNION_TYPE_UNION;
    n[0].aabb = 1;
    n[0].scale = 1.0f;
    n[0].aabb_exaggeration = 1.3f;
    n[1] = n[0];
    n[1].kind = PT_NODE_SPHERE;
    n[1].parent = 0;
    n[1].size[0] = 1.0f;
    /* Mat order (test_compute.glsl:45-59): col3, brightness, light3, spec,
     * spec_col3, roughness, IOR, refract_chance, refract_roughness, refract_col3 */
    {
        static const float mat[18] = {1, 1, 1, 1, 1, 1, 1, 0, 1, 1, 1, 0, 0, 0, 0, 1, 1, 1};
        memcpy(n[1].material, mat, sizeof mat);
    }
}

typedef struct {
    pt_op *ops;
    pt_aabb *aabbs;
    float *data;
    uint32_t n_ops, n_aabb, n_data, n_check;
} program;

static int compile_c1(program *p) {
    pt_scene_node nodes[2];
    c1_scene(nodes);
    memset(p, 0, sizeof *p);
    /* call 1: sizes only (every output pointer NULL) */
    int rc = pt_compile_scene(nodes, 2, NULL, 0, &p->n_ops, NULL, 0, &p->n_aabb, NULL, 0, &p->n_data, &p->n_check);
    if (rc != PT_OK) {
        fprintf(stderr, "pt_compile_scene (sizes): %d\n", rc);
        return 1;
    }
    p->ops = calloc(p->n_ops ? p->n_ops : 1, sizeof *p->ops);
    p->aabbs = calloc(p->n_aabb ? p->n_aabb : 1, sizeof *p->aabbs);
    p->data = calloc(p->n_data ? p->n_data : 1, sizeof *p->data);
    if (!p->ops || !p->aabbs || !p->data) return 1;
    /* a capacity one short must be refused with PT_ERR_SIZE */
    if (p->n_data > 0) {
        uint32_t a = 0, b = 0, d = 0, k = 0;
        rc = pt_compile_scene(nodes, 2, p->ops, p->n_ops, &a, p->aabbs, p->n_aabb, &b, p->data, p->n_data - 1, &d, &k);
        if (rc != PT_ERR_SIZE || d != p->n_data) {
            fprintf(stderr, "short data[] capacity: rc %d, n_data %u\n", rc, d);
            return 1;
        }
    }
    /* call 2: the program */
    rc = pt_compile_scene(nodes, 2, p->ops, p->n_ops, &p->n_ops, p->aabbs, p->n_aabb, &p->n_aabb, p->data, p->n_data,
                          &p->n_data, &p->n_check);
    if (rc != PT_OK) {
        fprintf(stderr, "pt_compile_scene: %d\n", rc);
        return 1;
    }
    return 0;
}

static uint32_t bits(float f) {
    uint32_t u;
    memcpy(&u, &f, sizeof u);
    return u;
}

static int compile_print(void) {
    program p;
    if (compile_c1(&p)) return 1;
    printf("{\"n_ops\": %u, \"n_aabb\": %u, \"n_data\": %u, \"n_check\": %u, \"data_bits\": [", p.n_ops, p.n_aabb,
           p.n_data, p.n_check);
    for (uint32_t i = 0; i < p.n_data; ++i) printf("%s%u", i ? ", " : "", (unsigned)bits(p.data[i]));
    printf("], \"ops\": [");
    for (uint32_t i = 0; i < p.n_ops; ++i) {
        const pt_op *o = &p.ops[i];
        printf("%s[%u, %u, %u, %d, %u, %u, %u]", i ? ", " : "", (unsigned)o->opcode, (unsigned)o->shape,
               (unsigned)o->combine, (int)o->check, (unsigned)o->scale, (unsigned)o->size[0],
               (unsigned)o->material[0]);
    }
    printf("], \"aabbs\": [");
    for (uint32_t i = 0; i < p.n_aabb; ++i) {
        const pt_aabb *a = &p.aabbs[i];
        printf("%s[%d, %u, %u, %u, %u]", i ? ", " : "", (int)a->back, (unsigned)a->so_kind, (unsigned)a->union_scale,
               (unsigned)a->shape_scale, (unsigned)a->aabb_exaggeration);
    }
    printf("]}\n");
    free(p.ops);
    free(p.aabbs);
    free(p.data);
    return 0;
}

/* float32 [h][w][4] from a version-1 .npy file (little-endian '<f4', C order) */
static float *load_npy(const char *path, size_t want_floats, const char *shape) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        fprintf(stderr, "cannot open %s\n", path);
        return NULL;
    }
    unsigned char head[10];
    float *out = NULL;
    if (fread(head, 1, 10, f) == 10 && memcmp(head, "\x93NUMPY", 6) == 0 && head[6] == 1) {
        const size_t hlen = (size_t)head[8] | ((size_t)head[9] << 8);
        char *dict = calloc(hlen + 1, 1);
        if (dict && fread(dict, 1, hlen, f) == hlen && strstr(dict, "'<f4'") && strstr(dict, shape) &&
            strstr(dict, "'fortran_order': False")) {
            out = malloc(want_floats * sizeof(float));
            if (out && fread(out, sizeof(float), want_floats, f) != want_floats) {
                free(out);
                out = NULL;
            }
        }
        free(dict);
    }
    fclose(f);
    if (!out) fprintf(stderr, "%s: not a float32 %s .npy\n", path, shape);
    return out;
}

#define CHK(call)                                                                                  \
    do {                                                                                           \
        const int rc_ = (call);                                                                    \
        if (rc_ != PT_OK) {                                                                        \
            fprintf(stderr, "%s: %d (%s)\n", #call, rc_, ctx ? pt_last_error(ctx) : "no context"); \
            goto done;                                                                             \
        }                                                                                          \
    } while (0)

static int render(const char *fixture) {
    enum { W = 32, H = 32, SPP = 2, BOUNCES = 1 };
    const size_t nf = (size_t)W * H * 4;
    int status = 1;
    pt_ctx *ctx = NULL;
    program p;
    float *img = NULL, *want = load_npy(fixture, nf, "(32, 32, 4)");
    if (!want || compile_c1(&p)) return 1;
    img = malloc(nf * sizeof(float));
    if (!img) goto done;
    {
        /* State::new -> PathTracer::new (path_tracer.rs:28-60) + the
         * editor's first compile and data upload (sdf_editor.rs:35-47) */
        const pt_constants c = {0.0f, 1, (float)W / (float)H, 1}; /* frame 1, last_clear 1: the first update() */
        const pt_settings s = {0, BOUNCES, 1.0f, 1.0f, 0};
        CHK(pt_create(0, W, H, &ctx));
        CHK(pt_set_program(ctx, p.ops, p.n_ops, p.aabbs, p.n_aabb, p.n_check));
        CHK(pt_set_data(ctx, p.data, p.n_data));
        /* SPP frames = SPP x (update, compute_pass) (path_tracer.rs:97-146) */
        CHK(pt_dispatch(ctx, &c, &s, SPP));
        CHK(pt_read_accum(ctx, img, nf * sizeof(float)));
        {
            size_t bad = 0, first = 0;
            for (size_t i = 0; i < nf; ++i)
                if (bits(img[i]) != bits(want[i]) && bad++ == 0) first = i;
            double mean = 0.0;
            for (size_t i = 0; i < nf; i += 4) mean += img[i] + img[i + 1] + img[i + 2];
            printf("{\"floats\": %zu, \"mismatched\": %zu, \"mean_rgb\": %.6f}\n", nf, bad, mean / (3.0 * W * H));
            if (bad) {
                fprintf(stderr, "%zu floats differ from %s (first at %zu: %.9g vs %.9g)\n", bad, fixture, first,
                        img[first], want[first]);
                goto done;
            }
            if (!(mean > 0.0)) {
                fprintf(stderr, "black image\n");
                goto done;
            }
        }
        /* a bad argument comes back as a status code, not a crash */
        if (pt_read_accum(ctx, img, 16) != PT_ERR_SIZE) {
            fprintf(stderr, "pt_read_accum accepted a short buffer\n");
            goto done;
        }
        status = 0;
    }
done:
    if (ctx) pt_destroy(ctx);
    free(img);
    free(want);
    free(p.ops);
    free(p.aabbs);
    free(p.data);
    return status;
}

int main(int argc, char **argv) {
    if (pt_abi_version() != PT_ABI_VERSION) {
        fprintf(stderr, "ABI version %d, header %d\n", pt_abi_version(), PT_ABI_VERSION);
        return 1;
    }
    if (argc >= 2 && strcmp(argv[1], "layout") == 0) return layout();
    if (argc >= 2 && strcmp(argv[1], "compile") == 0) return compile_print();
    if (argc >= 3 && strcmp(argv[1], "render") == 0) return render(argv[2]);
    fprintf(stderr, "usage: %s layout | compile | render FIXTURE.npy\n", argv[0]);
    return 2;
}
