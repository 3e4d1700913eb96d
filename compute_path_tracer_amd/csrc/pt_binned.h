// pt_binned.h -- the mask-binned wavefront schedule (PT_KERNEL_BINNED).
//
// Same per-sample arithmetic as the reference loop (pt_path.h), different
// grouping of work.  The tile-resident wavefront kernel (pt_wave.h) keeps a
// lane's path on that lane, so after the first bounce the 64 lanes of a wave
// march rays whose check[] sets (bounds(), test_compute.glsl:101) differ and
// the wave pays for the union of their shapes.  Here every bounce is one pass
// over all live paths of a chunk of frames:
//
//   gen     camera rays of every (pixel, frame) + their bounds() mask
//   bin     histogram of mask bins -> prefix sum -> scatter of 4-byte ray
//           slots into bin order
//   trace   persistent waves take runs of the binned slots; the slots of the
//           next 64-ray window are prefetched one window ahead, the rays
//           (64 B records, mask included) gathered into staging registers
//           and handed to free lanes, which march and calc_normal them; a
//           miss stores the path's colour, a hit writes a hit record to the
//           other ray buffer at its binned position
//   shade   shading + Russian roulette of every hit record, then bounds()
//           mask + bin of each continuing ray (next pass)
//   fold    each pixel mixes its frames' colours in frame order
//
// The host splits a chunk's frames over two such pipelines on two streams
// (pt_runtime.hip launch_binned), so their passes overlap.
//
// Paths are independent and the fold runs in frame order, so the schedule
// changes nothing in the image: it is bit-identical to the other kernels.
#pragma once

#include "pt_path.h"

#ifndef PT_BIN_BITS
#define PT_BIN_BITS 12
#endif
#define PT_BINS (1 << PT_BIN_BITS)
#define PT_BIN_NONE 0xffffffffu
#define PT_AUX_MISS 0xffffffffu  // trace -> shade: PtRay q2.w of a position whose segment missed
#define PT_BIN_BLOCK 256  // threads per block of the gen / bounds / scatter kernels
// A pass's control words (PtPass.ctrl): [0] = its ray count, and the trace
// pass's run cursors, one per share of the pass (PT_RUN_SHARDS, one per XCD),
// each on its own 128-byte line.
#ifndef PT_RUN_SHARDS
#define PT_RUN_SHARDS 8
#endif
#define PT_CTRL_CURSOR(k) (32u * (1u + uint32_t(k)))
#define PT_CTRL_STRIDE (32u * (1u + uint32_t(PT_RUN_SHARDS)))
#ifndef PT_SCATTER_ITEMS
#define PT_SCATTER_ITEMS 16
#endif

// A path between two segments (ray) or, taps in the trace pass, at the hit
// of its segment (hit record), 64 B = four 16 B quads:
//   q0 = (ro.x, ro.y, ro.z, rd.x)        ro: origin, or the hit point
//   q1 = (rd.y, rd.z, thr.x, thr.y)
//   q2 = (thr.z, rng, sid, aux)          sid: sample slot = frame * n_pix + local
//                                        pixel; aux: a ray's own slot (its index
//                                        in its buffer), a hit record's material
//                                        index, or PT_AUX_MISS (a miss writes
//                                        only this quad)
//   q3 = ray: check[] bits 0..63 of the segment to trace (64..127: PtPass.mask_hi)
//        hit record: (calc_normal's differences, 0)
// With the taps in the shade pass (the scene kernels) the trace pass writes
// no record: a hit or a miss is one 16 B hit quad (PtPass.hq) at its binned
// position, {t, material or PT_AUX_MISS, the taps' map() bound, the ray's
// slot}, and the shade pass reads the traced ray itself from its slot -- the
// trace pass does not change it -- and recomputes the hit point ro + rd * t
// with calc_point's f32 steps.  (check[] bits 64..127 of a hit: PtPass.hitn.zw.)
// The path's radiance (path_trace's `ret`) is not carried: it lives in the
// sample's colour slot (zeroed by gen), which the shade pass updates when an
// emission is added and which is final when the path ends.
struct PtRay {
    uint4 q[4];
};

struct PtPass {
    PtLaunch L;             // scene tables, image, frame0 / last_clear0 of this chunk
    PtRay *rin;             // this pass's rays, by slot (gen: the rays being binned; shade: the traced rays)
    PtRay *rout;            // trace with taps: its hit records; shade: the next pass's rays (both by binned
                            // position)
    uint4 *hq;              // trace -> shade (taps in the shade pass): a hit quad per binned position
    uint2 *mask_hi;         // check[] bits 64..127 per rin slot (scenes with > 64 entries)
    uint32_t *key;          // bin per rin slot (PT_BIN_NONE: no live ray)
    uint32_t *idx;          // rin slots in bin order
    uint32_t *hist;         // [PT_BINS] counts, zero outside gen/bounds -> scan
    uint32_t *offs;         // [PT_BINS] scatter cursors
    uint32_t *ctrl;         // this pass: [0] binned rays, [PT_CTRL_CURSOR(k)] trace run cursors
    const uint32_t *n_src;  // rin slots (bounds / scatter), null: n_src_const
    float4 *color;          // [frames][n_pix] sample colours
    float4 *hitn;           // trace -> shade: check[] bits 64..127 of a hit (.zw; scenes with > 64 entries)
    unsigned long long *btab;  // [PT_BINS] check[] set + 1 per bin (0: free), null: hashed bins (bin_resolve);
                               // [PT_BINS]: sets that found no slot (the dispatch's overflow count)
    int32_t lanes;          // fold: pipelines that split the chunk's frames (colour regions, bin_fold_body)
    uint32_t n_src_const;
    int32_t bounce;         // segment index of this pass (path_trace's loop counter i)
    int32_t n_pix;          // local pixel slots: n_tiles * 64
    int32_t frames;         // frames in this chunk
    int32_t wide;           // check[] has more than 64 entries
    int32_t run_max;        // trace: longest run of binned rays a wave takes at once (multiple of 64)
    int32_t refill_min;     // trace: refill when at least this many lanes are free (or none map)
    int32_t gen_order;      // gen: list the slots in generation order (idx; the host sets ctrl[0]) for the
                            // first trace pass instead of binning them (the gen pass: a 64-ray window = one
                            // 8x8 tile; gen_trace: one pixel over 64 frames, gen_sample)
    int32_t gen_trace;      // first pass without a gen pass (scene kernels, generation order): the trace
                            // pass makes each window's camera rays and bounds() itself, a miss zeroes its
                            // colour slot, and the shade pass stores (not adds) the first segment's emission
    int32_t count_overflow; // bin_resolve counts the sets that find no slot (btab[PT_BINS]; instrumented runs)
    int32_t gen_norec;      // gen_trace, check[] of <= 32 entries: the first pass writes no ray records -- its
                            // hit quads carry the ray's check[] bits in .w (the slot is the position) -- and
                            // shade pass 0 makes each traced camera ray again (camera_ray: the same bits)
};

namespace pt {

__device__ __forceinline__ uint32_t bin_hash(const uint4 &m) {
    const uint32_t h = (m.x * 0x9E3779B1u) ^ (m.y * 0x85EBCA77u) ^ (m.z * 0xC2B2AE3Du) ^ (m.w * 0x27D4EB2Fu);
    return (h ^ (h >> 15)) * 0x2C1B3C6Du >> (32 - PT_BIN_BITS);
}

// The bin of a check[] set.  Scenes with at most PT_BIN_BITS entries: the set
// itself.  Wider scenes: a hash would put two sets in one bin now and then,
// and a trace window of that bin then evaluates the union of both sets'
// shapes (C3: ~4900 distinct sets seen; a 64-ray window of a hashed bin admits
// ~2.6 boxes where its own set has ~1.8).  So with P.btab
// (scenes of 13..64 entries) the bin is the set's slot in a table of sets,
// open addressing from the hash: the first lane to see a set claims a free
// slot with a CAS, every later one finds it.  Only the schedule depends on
// the table (the host clears it per dispatch); a set that finds no slot
// within PT_BIN_PROBES shares its hash bin as before.
#ifndef PT_BIN_PROBES
#define PT_BIN_PROBES 8
#endif
// In two steps, so a pass can issue the first probe's load before it stores
// the ray and compare after: vmcnt counts stores as well as loads (gfx9), so
// a load issued behind the ray's stores would wait for them too (the shade
// pass: +10 points of its wave time at s_waitcnt, 3.21).
struct BinProbe {
    uint32_t h;              // the hash bin: the first slot
    unsigned long long e;    // the set + 1 (0: not in the table)
    unsigned long long v;    // the first slot's content
};
__device__ __forceinline__ BinProbe bin_probe(const PtPass &P, const uint4 &m) {
    BinProbe b;
    b.h = bin_hash(m);
    b.e = 0ull;
    b.v = 0ull;
    if (P.btab) {
        b.e = ((unsigned long long)m.y << 32 | m.x) + 1ull;  // (0: a free slot)
        // (a plain load: a slot only ever goes from 0 to its set, so a stale
        // 0 just sends the lane to the CAS, which returns the slot's set)
        if (b.e != 0ull) b.v = P.btab[b.h];
    }
    return b;
}
__device__ __forceinline__ uint32_t bin_resolve(const PtPass &P, const uint4 &m, BinProbe b) {
    if (!P.btab) {
        if ((m.y | m.z | m.w) == 0u && m.x < uint32_t(PT_BINS)) return m.x;  // small scenes: the exact set
        return b.h;
    }
    // (the set already in its hash slot, nearly every lane after a pass's
    // first waves, returns before the claim below, so the claim's wait for
    // its CAS -- a vmcnt(0), the ray's stores included -- runs only in waves
    // with a lane that claims or probes on)
    if (b.e == 0ull || b.v == b.e) return b.h;
    uint32_t s = b.h;
    unsigned long long v = b.v;
    for (int k = 0;;) {
        if (v == 0ull) v = atomicCAS(P.btab + s, 0ull, b.e);
        if (v == 0ull || v == b.e) return s;
        if (++k == PT_BIN_PROBES) {  // no slot for this set: it shares its hash bin
            // (counted by the instrumented dispatch only: one word that every
            // overflowing lane adds to would be a hot atomic in the timed one)
            if (P.count_overflow) atomicAdd(P.btab + PT_BINS, 1ull);
            return b.h;
        }
        s = (s + 1u) & uint32_t(PT_BINS - 1);
        v = P.btab[s];
    }
}

// bounds() of one ray, one thread: every box's slab test (scalar box loads).
// Rays (and scenes, L.fast_bounds) inside the pt_div_*_ok guards divide via
// per-ray reciprocals; the rest take the IEEE divisions.  Same bits either way.
template <bool ST>
__device__ __forceinline__ uint4 bounds_mask(const PtLaunch &L, const pt_f3 &ro, const pt_f3 &rd, Stats<ST> &st) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    const caabb_ptr boxes = (caabb_ptr)L.aabbs;
    const bool fast = L.fast_bounds != 0 && pt_div_coord_ok(ro.x) && pt_div_coord_ok(ro.y) &&
                      pt_div_coord_ok(ro.z) && pt_div_dir_ok(rd.x) && pt_div_dir_ok(rd.y) && pt_div_dir_ok(rd.z);
    if (fast) {
        if constexpr (ST)
            if (first_active_lane()) st.add(PT_ST_BOUNDS_WAVES);
        const float yx = 1.0f / rd.x, yy = 1.0f / rd.y, yz = 1.0f / rd.z;
        // slab values from the reciprocal products; a wave with an undecided
        // comparison redoes every box exactly (ray_box_ulp)
        uint32_t gapu = 0xffffffffu;
#pragma unroll 4  // scalar box loads issued ahead of their slab tests
        for (int b = 0; b < L.n_aabb; ++b) {
            const PtAabb bx = boxes[b];
            if (ray_box_ulp<false>(bx, ro.x, ro.y, ro.z, yx, yy, yz, gapu)) w[bx.back >> 5] |= 1u << (bx.back & 31);
        }
        if (__builtin_expect(__ballot(!(gapu > PT_ULP_MARGIN)) != 0ull, 0)) {
            if constexpr (ST)
                if (first_active_lane()) st.add(PT_ST_BOUNDS_EXACT);
            uint32_t v[4] = {0u, 0u, 0u, 0u};
            for (int b = 0; b < L.n_aabb; ++b) {
                const PtAabb bx = boxes[b];
                if (ray_box_rcp(bx, ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, yx, yy, yz))
                    v[bx.back >> 5] |= 1u << (bx.back & 31);
            }
            if (!(gapu > PT_ULP_MARGIN))
                for (int k = 0; k < 4; ++k) w[k] = v[k];
        }
    } else {
        for (int b = 0; b < L.n_aabb; ++b) {
            const PtAabb bx = boxes[b];
            if (ray_box(bx, ro.x, ro.y, ro.z, rd.x, rd.y, rd.z)) w[bx.back >> 5] |= 1u << (bx.back & 31);
        }
    }
    st.add(PT_ST_SEGMENTS);
    st.add(PT_ST_AABB, uint32_t(L.n_aabb));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// check[] wider than 64 bits, per map type: -1 = decided at run time
// (PtPass.wide); the scene kernels specialise it with their scene's answer,
// so a narrow scene's kernels carry no high mask words at all
template <class Map>
struct MapWide {
    static constexpr int v = -1;
};
template <class Map>
__device__ __forceinline__ bool wide_of(const PtPass &P) {
    if constexpr (MapWide<Map>::v >= 0) return MapWide<Map>::v != 0;
    else return P.wide != 0;
}

// material table entries a map type's shade pass stages in LDS (0: none;
// the scene kernels specialise it with their table's size, pt_jit.cpp)
template <class Map>
struct MapMats {
    static constexpr int n = 0;
};

// bounds() of the shade pass, per map type: the generic box loop; the
// scene kernels specialise it (pt_jit.cpp: straight-line slab tests with
// constant check[] bits, boxes baked as literals in the tier-up build).
template <class Map>
struct MapBounds {
    template <bool ST>
    static __device__ __forceinline__ uint4 mask(const PtLaunch &L, const pt_f3 &ro, const pt_f3 &rd, Stats<ST> &st) {
        return bounds_mask<ST>(L, ro, rd, st);
    }
    // the same with box k's slab test skipped where bit k of `skip` is set
    // (primary_box_skip: every lane of the wave provably misses box k); the
    // generic loop ignores the hint
    template <bool ST>
    static __device__ __forceinline__ uint4 mask_skip(const PtLaunch &L, const pt_f3 &ro, const pt_f3 &rd, uint64_t skip,
                                                      Stats<ST> &st) {
        (void)skip;
        return bounds_mask<ST>(L, ro, rd, st);
    }
};

// The boxes that no lane of a wave can hit, for the first pass's camera rays
// (DESIGN.md 3.20): bit k set = box k's fast-path slab test would report a
// decided miss in every lane, so bounds() may skip it.  The rays of a window
// (one 8x8 tile of one frame) share the camera's origin o and have nearly
// the same direction, and a box is tested against the wave's whole bundle at
// once, one box per lane: with y_a = RN(1/d_a) of every lane inside
// [ylo_a, yhi_a] (one sign) and C = RN(b - o) a constant, each lane's slab
// value RN(C * y_a) lies between the products at the interval's ends (RN is
// monotone, so is the product in y for a fixed C).  Hence every lane's
// tnear' >= L (the largest over the axes of the least corner product) and
// tfar' <= U (the least of the largest).  U <= 0: tfar' <= 0 in every lane,
// and the IEEE tfar has tfar''s sign (3.14): a miss.  L, U > 0 with
// bits(L) - bits(U) > PT_ULP_MARGIN: every lane's slab gap exceeds the
// margin, so its fast-path result is decided (3.19) and is a miss.  Either
// way the lane's bit is 0 and the box does not change whether the lane takes
// the exact fallback (its gap is above the margin).  Every lane of the wave
// must be active; lanes outside the fast path's guards do not count (they
// take the IEEE loop).  Returns 0 (skip nothing) unless the fast-path lanes
// share one origin, the scene's boxes pass the guards and there are <= 64.
__device__ __forceinline__ uint64_t primary_box_skip(const PtLaunch &L, const pt_f3 &ro, const pt_f3 &rd) {
    const int nb = L.n_aabb;
    if (L.fast_bounds == 0 || nb <= 0 || nb > 64) return 0ull;
    // the row-broadcast scans read every lane: with a partial EXEC the
    // inactive lanes' stale values could make a box look missed
    if (__builtin_amdgcn_read_exec() != ~0ull) return 0ull;
    const bool fast = pt_div_coord_ok(ro.x) && pt_div_coord_ok(ro.y) && pt_div_coord_ok(ro.z) &&
                      pt_div_dir_ok(rd.x) && pt_div_dir_ok(rd.y) && pt_div_dir_ok(rd.z);
    const uint64_t fm = __ballot(fast);
    if (fm == 0ull) return 0ull;
    // the origin of the first fast lane, and no fast lane with another one
    const int l0 = __builtin_ctzll(fm);
    const float ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ro.x), l0));
    const float oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ro.y), l0));
    const float oz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ro.z), l0));
    if (__ballot(fast && (__float_as_uint(ro.x) != __float_as_uint(ox) || __float_as_uint(ro.y) != __float_as_uint(oy) ||
                          __float_as_uint(ro.z) != __float_as_uint(oz))) != 0ull)
        return 0ull;
    const float inf = __builtin_inff();
    const uint32_t lane = threadIdx.x & 63u;
    const bool mine = lane < uint32_t(nb);  // lane k tests box k against the whole bundle
    // (the offset through an empty asm: a per-lane address the compiler
    // hoisted out of the persistent loop took two registers and spilled)
    static_assert(sizeof(PtAabb) == 32, "box stride");
    uint32_t off;
    __asm__ volatile("v_lshlrev_b32 %0, 5, %1" : "=v"(off) : "v"(lane));
    const float *box = reinterpret_cast<const float *>(reinterpret_cast<const char *>(L.aabbs) + off);
    float lo = -inf, hi = inf;
    // one axis at a time (few registers live): the lanes' y = the reciprocal
    // bounds() itself forms (the same correctly rounded division), its wave
    // range, and box k's corner products; an axis whose lanes' y straddle
    // zero gives no finite bound and is left out
    auto axis = [&](int a, float d, float o) {
        const float y = 1.0f / d;
        const float ylo = wave_min_f32(fast ? y : inf), yhi = wave_max_f32(fast ? y : -inf);
        if (mine && (ylo > 0.0f || yhi < 0.0f)) {
            const float c1 = box[a] - o, c2 = box[3 + a] - o;  // PtAabb: bmin[3], bmax[3]
            const float p1 = c1 * ylo, p2 = c1 * yhi, p3 = c2 * ylo, p4 = c2 * yhi;
            lo = pt_gmax(lo, pt_gmin(pt_gmin(p1, p2), pt_gmin(p3, p4)));
            hi = pt_gmin(hi, pt_gmax(pt_gmax(p1, p2), pt_gmax(p3, p4)));
        }
    };
    axis(0, rd.x, ox);
    axis(1, rd.y, oy);
    axis(2, rd.z, oz);
    const bool skip = mine && (hi <= 0.0f ||
                               (lo > 0.0f && hi > 0.0f && __float_as_uint(lo) > __float_as_uint(hi) + PT_ULP_MARGIN));
    return __ballot(skip);
}

__device__ __forceinline__ void store_ray(PtRay *r, const pt_f3 &ro, const pt_f3 &rd, const pt_f3 &thr, uint32_t rng,
                                          uint32_t sid, uint32_t aux, const uint4 &q3) {
    r->q[0] = make_uint4(__float_as_uint(ro.x), __float_as_uint(ro.y), __float_as_uint(ro.z), __float_as_uint(rd.x));
    r->q[1] = make_uint4(__float_as_uint(rd.y), __float_as_uint(rd.z), __float_as_uint(thr.x), __float_as_uint(thr.y));
    r->q[2] = make_uint4(__float_as_uint(thr.z), rng, sid, aux);
    r->q[3] = q3;
}

__device__ __forceinline__ void hist_zero(uint32_t *lh) {
    for (int b = int(threadIdx.x); b < PT_BINS; b += int(blockDim.x)) lh[b] = 0u;
    __syncthreads();
}
__device__ __forceinline__ void hist_flush(const uint32_t *lh, uint32_t *hist) {
    __syncthreads();
    for (int b = int(threadIdx.x); b < PT_BINS; b += int(blockDim.x))
        if (lh[b] != 0u) atomicAdd(&hist[b], lh[b]);
}
// local pixel slot -> image coordinates (cyclic tile ownership, as pt_wave.h)
__device__ __forceinline__ void pixel_of(int rank, int nranks, int tiles_x, uint32_t pl, int &x, int &y) {
    const int k = int(pl >> 6), p = int(pl & 63u);
    const int g = rank + k * nranks;
    x = (g % tiles_x) * PT_TILE + (p & 7);
    y = (g / tiles_x) * PT_TILE + (p >> 3);
}
__device__ __forceinline__ void pixel_of(const PtLaunch &L, uint32_t pl, int &x, int &y) {
    pixel_of(L.rank, L.nranks, L.tiles_x, pl, x, y);
}
// The first pass's position p -> its sample (frame f, local pixel pl), frame
// fastest: a 64-ray window is one pixel's camera rays of 64 frames (with 64
// or more frames in the chunk), whose directions differ only by the
// sub-pixel jitter -- the narrowest bundle for the box skip (3.20) and the
// most coherent march.  The sample's colour slot stays f * n_pix + pl.
__device__ __forceinline__ void gen_sample(uint32_t frames, uint32_t p, uint32_t &f, uint32_t &pl) {
    pl = p / frames;
    f = p - pl * frames;
}
// A sample's colour slot in its pipeline's region: [pixel][frame], so the
// first pass's position is its sample's slot (gen_sample) and a pixel's
// frames lie in one run for the fold.
__device__ __forceinline__ uint32_t colour_slot(uint32_t frames, uint32_t f, uint32_t pl) { return pl * frames + f; }

// gen: camera ray + bounds() of every (frame, pixel) of the chunk
// (MapBounds<Map>: the generic box loop, or the scene kernels' straight-line
// slab tests).
template <class Map, bool ST>
__device__ __forceinline__ void bin_gen_body(const PtPass &P) {
    __shared__ uint32_t lh[PT_BINS];
    hist_zero(lh);
    Stats<ST> st;
    st.init();
    const PtLaunch &L = P.L;
    const uint32_t npix = uint32_t(P.n_pix), n = npix * uint32_t(P.frames);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t f = i / npix, pl = i - f * npix;
        int x, y;
        pixel_of(L, pl, x, y);
        const bool live = x < L.width && y < L.height;
        // the first pass's list in generation order (the host takes this path
        // only when every tile is full, so every slot is live)
        if (P.gen_order) P.idx[i] = i;
        if (!live) {
            if (!P.gen_order) P.key[i] = PT_BIN_NONE;
            continue;
        }
        uint32_t rng;
        pt_f3 ro, rd;
        camera_ray(x, y, int32_t(uint32_t(L.frame0) + f), L.width, L.height, L.aspect, L.fov, rng, ro, rd);
        st.add(PT_ST_SAMPLES);
        const uint4 m = MapBounds<Map>::template mask<ST>(L, ro, rd, st);
        const BinProbe bp = P.gen_order ? BinProbe{0u, 0ull, 0ull} : bin_probe(P, m);  // (before the stores)
        const uint32_t sid = colour_slot(uint32_t(P.frames), f, pl);
        store_ray(P.rin + i, ro, rd, pt_f3{1.0f, 1.0f, 1.0f}, rng, sid, i, make_uint4(m.x, m.y, 0u, 0u));
        P.color[sid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // the path's radiance (ret) starts at 0
        if (wide_of<Map>(P)) P.mask_hi[i] = make_uint2(m.z, m.w);
        if (!P.gen_order) {
            const uint32_t b = bin_resolve(P, m, bp);
            P.key[i] = b;
            atomicAdd(&lh[b], 1u);
        }
    }
    if (!P.gen_order) hist_flush(lh, P.hist);
    flush_stats<ST>(L, st);
}

// shade: every hit the last trace pass wrote (positions marked HIT) is
// shaded -- material, new direction, emission, throughput, Russian roulette
// (pt_path.h shade_lane, the same f32 steps and rng draws) -- and a path that
// goes on gets its next segment's bounds() mask and bin.  Shading is taken
// out of the trace pass, where it ran on a fraction of the lanes of a wave;
// here, one thread per hit, it fills the VALU time this memory-latency-bound
// pass had idle.
//
// TAPS = false (PtPass taps_in_shade, scene kernels only): the trace pass
// stopped at the hit and wrote its hit quad; this pass reads the traced ray
// from the quad's slot, recomputes the hit point, and evaluates
// calc_normal's six taps itself (test_compute.glsl:57-66) with Map = JitMapB:
// all lanes of a wave tap together, and the per-hit map() bound (pt_path.h
// tap_bound, carried in the quad) lets each tap drop every shape that
// provably lies farther away.  TAPS = true: the hit records
// of P.rout, shaded and replaced in place by the next rays.
template <class Map, bool ST, bool TAPS>
__device__ __forceinline__ void bin_shade_body(const PtPass &P) {
    __shared__ uint32_t lh[PT_BINS];
    // the scene kernels' material table (MapMats<Map>::n entries) staged in
    // LDS: a hit's material is then one LDS read, not three dependent global
    // round trips after the taps
    constexpr int NM = MapMats<Map>::n;
    __shared__ PtMat lm[NM > 0 ? NM : 1];
    const PtMat *mats = P.L.mats;
    if constexpr (NM > 0) {
        const uint4 *src = reinterpret_cast<const uint4 *>(P.L.mats);
        uint4 *dst = reinterpret_cast<uint4 *>(lm);
        for (int k = int(threadIdx.x); k < NM * int(sizeof(PtMat) / 16); k += int(blockDim.x)) dst[k] = src[k];
        mats = lm;
    }
    hist_zero(lh);  // (its barrier also publishes lm)
    Stats<ST> st;
    st.init();
    Stats<ST> stt;  // the normal taps' work (TAPS = false)
    stt.init();
    const PtLaunch &L = P.L;
    const uint32_t n = P.n_src ? *P.n_src : P.n_src_const;
    // q0..q3: the traced ray (TAPS = false; hq its hit quad) or the hit
    // record (TAPS = true)
    auto shade_one = [&](uint32_t i, const uint4 &q0, const uint4 &q1, const uint4 &q2, const uint4 &q3,
                         const uint2 &hi, const uint4 &hq) {
        pt_f3 ro{__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z)};
        pt_f3 rd{__uint_as_float(q0.w), __uint_as_float(q1.x), __uint_as_float(q1.y)};
        pt_f3 thr{__uint_as_float(q1.z), __uint_as_float(q1.w), __uint_as_float(q2.x)};
        pt_f3 ret{0.0f, 0.0f, 0.0f};  // this segment's emission (added to the colour slot below)
        uint32_t rng = q2.y;
        const uint32_t sid = q2.z;
        const int mat = int(TAPS ? q2.w : hq.y);
        int seg = P.bounce;
        // taps in the trace pass: q3 = calc_normal's differences
        float dv0 = __uint_as_float(q3.x), dv1 = __uint_as_float(q3.y), dv2 = __uint_as_float(q3.z);
        if constexpr (!TAPS) {
            // the hit point: calc_point's f32 steps with the trace's t
            // (pt_path.h after_map), so the same bits
            const float t = __uint_as_float(hq.x);
            ro = pt_f3{ro.x + rd.x * t, ro.y + rd.y * t, ro.z + rd.z * t};
            // (the taps' counters go to their own half of the stats buffer:
            // pt_dispatch_stats sums both, bench.py splits the flops by pass)
            // the ray's check[] bits 0..63 (q3.xy) and 64..127 (hi)
            Check ck{uint64_t(q3.x) | (uint64_t(q3.y) << 32), uint64_t(hi.x) | (uint64_t(hi.y) << 32)};
            const float bnd = __uint_as_float(hq.z);
            // bnd widened by the taps' spread (two taps are at most 2e apart,
            // plus their coordinates' rounding): the first tap's tests against
            // it leave in `live` every shape any tap may need
            const float bndw = bnd + (0x1.a3ap-13f + 0x1p-20f * (fabsf(ro.x) + fabsf(ro.y) + fabsf(ro.z)));
            uint64_t live = 0ull;
            float dp = 0.0f;
#pragma unroll 1
            for (int k = 0; k < 6; ++k) {
                float qx, qy, qz;
                map_point(ST_NORMAL, k, ro, rd, 0.0f, qx, qy, qz);
                if constexpr (ST)
                    if (first_active_lane()) stt.add(PT_ST_WAVE_MAPS);
                const Hit h = k == 0 ? Map::template first<ST>(L, qx, qy, qz, ck, bnd, bndw, live, stt)
                                     : Map::template rest<ST>(L, qx, qy, qz, ck, bnd, bndw, live, stt);
                if (k == 0) ck.alo = Map::alive(live);  // (the other taps' wave-level live test)
                if ((k & 1) == 0) {
                    dp = h.d;  // d(p + e)
                } else {
                    const float dd = dp - h.d;
                    if (k == 1) dv0 = dd;
                    else if (k == 3) dv1 = dd;
                    else dv2 = dd;
                }
            }
            stt.add(PT_ST_NORMAL_MAPS, 6);
        }
        const bool done = shade_lane<ST>(mats, L.bounces, mat, dv0, dv1, dv2, 0, rng, ro, rd, thr, ret, seg, st);
        if (P.bounce == 0) st.add(PT_ST_SHADED_FIRST);
        // ret += emission * throughput (test_compute.glsl:148) on the colour
        // slot: 0 + e, added to the slot, equals the slot plus e (a slot
        // never holds -0), and a zero e changes no slot, so only emitting
        // segments touch it
        if (P.gen_trace) {  // first segment, no gen pass: the slot was never zeroed; 0 + e = e
            P.color[sid] = make_float4(ret.x, ret.y, ret.z, 0.0f);
        } else if (ret.x != 0.0f || ret.y != 0.0f || ret.z != 0.0f) {
            float4 c = P.color[sid];
            c.x += ret.x;
            c.y += ret.y;
            c.z += ret.z;
            P.color[sid] = c;
        }
        if (done) {
            if (L.debug == 3) {  // bounce-count view: the colour is the segment count, not the radiance
                const pt_f3 col = final_color(L.debug, seg, L.bounces, ret);
                P.color[sid] = make_float4(col.x, col.y, col.z, 0.0f);
            }
            P.key[i] = PT_BIN_NONE;
            return;
        }
        const uint4 m = MapBounds<Map>::template mask<ST>(L, ro, rd, st);
        const BinProbe bp = bin_probe(P, m);  // (before the stores: bin_probe)
        store_ray(P.rout + i, ro, rd, thr, rng, sid, i, make_uint4(m.x, m.y, 0u, 0u));
        if (wide_of<Map>(P)) P.mask_hi[i] = make_uint2(m.z, m.w);
        const uint32_t k = bin_resolve(P, m, bp);
        P.key[i] = k;
        atomicAdd(&lh[k], 1u);
    };
    // One thread per binned position.  TAPS = false: its hit quad, then the
    // traced ray from the quad's slot; TAPS = true: its hit record (a miss
    // marks its record's q2).
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if constexpr (TAPS) {
            const uint4 q0 = P.rout[i].q[0], q1 = P.rout[i].q[1], q2 = P.rout[i].q[2], q3 = P.rout[i].q[3];
            if (q2.w == PT_AUX_MISS) P.key[i] = PT_BIN_NONE;  // the path ended in the trace pass
            else shade_one(i, q0, q1, q2, q3, make_uint2(0u, 0u), q3);
        } else {
            uint4 hq = P.hq[i];
            // (the whole quad in one load before the miss test: left alone,
            // the compiler loads .yz, tests, then loads .xw inside the
            // branch -- a second round trip before the ray's gather)
            __asm__ volatile("" : "+v"(hq.x), "+v"(hq.y), "+v"(hq.z), "+v"(hq.w));
            if (hq.y == PT_AUX_MISS) {
                P.key[i] = PT_BIN_NONE;  // the path ended in the trace pass
                continue;
            }
            uint4 q0, q1, q2, q3;
            if (P.gen_norec) {
                // shade pass 0 without ray records: the traced camera ray of
                // sample i (its slot is its position) made again, as the first
                // pass made it (bin_trace_body stage), check[] bits from the quad
                // (the launch's scalars through an empty asm: left alone, the
                // compiler hoists what depends only on them -- the integer
                // divisions' reciprocals, float(height), fov * fov -- out of the
                // loop into registers held across the whole body, where they
                // spill)
                uint32_t npix = uint32_t(P.n_pix), nf = uint32_t(P.frames);
                int rk = L.rank, nr = L.nranks, tx = L.tiles_x, cw = L.width, chh = L.height;
                float ca = L.aspect, cf = L.fov;
                __asm__ volatile("" : "+s"(npix), "+s"(nf), "+s"(rk), "+s"(nr), "+s"(tx), "+s"(cw), "+s"(chh),
                                 "+s"(ca), "+s"(cf));
                uint32_t f, pl;
                gen_sample(nf, i, f, pl);
                int x, y;
                pixel_of(rk, nr, tx, pl, x, y);
                uint32_t rg;
                pt_f3 o, d;
                camera_ray(x, y, int32_t(uint32_t(L.frame0) + f), cw, chh, ca, cf, rg, o, d);
                q0 = make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), __float_as_uint(d.x));
                q1 = make_uint4(__float_as_uint(d.y), __float_as_uint(d.z), __float_as_uint(1.0f), __float_as_uint(1.0f));
                q2 = make_uint4(__float_as_uint(1.0f), rg, colour_slot(nf, f, pl), i);
                q3 = make_uint4(hq.w, 0u, 0u, 0u);
            } else {
                const PtRay *r = P.rin + hq.w;
                q0 = r->q[0];
                q1 = r->q[1];
                q2 = r->q[2];
                q3 = r->q[3];
            }
            uint2 hi = make_uint2(0u, 0u);
            if (wide_of<Map>(P)) {
                const float4 nd = P.hitn[i];
                hi = make_uint2(__float_as_uint(nd.z), __float_as_uint(nd.w));
            }
            shade_one(i, q0, q1, q2, q3, hi, hq);
        }
    }
    hist_flush(lh, P.hist);
    flush_stats<ST>(L, st);
    if constexpr (!TAPS) flush_stats<ST>(L, stt, PT_ST_COUNT);
}

// scan: exclusive prefix of the histogram; clears the histogram and this
// pass's cursors.  One wave (PT_SCAN_THREADS lanes, PT_BINS / 64 bins each,
// no LDS): it fits on a CU beside the other pipeline's persistent trace
// waves (28 of 32 slots), where a 1024-thread block waited for that trace
// pass to drain (1.26 ms per launch with two pipelines, 5 us alone).
#define PT_SCAN_THREADS 64
__device__ __forceinline__ void bin_scan_body(const PtPass &P) {
    constexpr int PER = PT_BINS / PT_SCAN_THREADS;
    const int t = int(threadIdx.x);
    uint4 *h4 = reinterpret_cast<uint4 *>(P.hist + t * PER);
    uint4 *o4 = reinterpret_cast<uint4 *>(P.offs + t * PER);
    uint32_t sum = 0u;
#pragma unroll
    for (int j = 0; j < PER / 4; ++j) {
        const uint4 v = h4[j];
        sum += v.x + v.y + v.z + v.w;
    }
    uint32_t inc = sum;  // inclusive prefix over the wave's lanes
#pragma unroll
    for (int off = 1; off < PT_SCAN_THREADS; off <<= 1) {
        const uint32_t x = uint32_t(__shfl_up(int(inc), off, PT_SCAN_THREADS));
        if (t >= off) inc += x;
    }
    uint32_t run = inc - sum;
#pragma unroll
    for (int j = 0; j < PER / 4; ++j) {
        const uint4 v = h4[j];
        uint4 o;
        o.x = run;
        run += v.x;
        o.y = run;
        run += v.y;
        o.z = run;
        run += v.z;
        o.w = run;
        run += v.w;
        o4[j] = o;
        h4[j] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (t == PT_SCAN_THREADS - 1) P.ctrl[0] = inc;
    if (t < PT_RUN_SHARDS) P.ctrl[PT_CTRL_CURSOR(t)] = 0u;
}

// scatter: ray slots into bin order.  Per block tile, the slots of one bin
// take consecutive places (LDS ranks) after one global reservation.
__device__ __forceinline__ void bin_scatter_body(const PtPass &P) {
    __shared__ uint32_t cnt[PT_BINS];
    const uint32_t n = P.n_src ? *P.n_src : P.n_src_const;
    // One contiguous run of the slots per block: count its bins in LDS,
    // reserve each bin's places with one global atomic for the whole run
    // (not one per 4096-slot tile), then read the keys again and hand out
    // the places with LDS cursors.
    const uint32_t per = ((n + gridDim.x - 1u) / gridDim.x + PT_BIN_BLOCK - 1u) & ~uint32_t(PT_BIN_BLOCK - 1);
    const uint32_t b0 = min(n, blockIdx.x * per), b1 = min(n, b0 + per);
    // (eight keys in flight per thread: the loads are issued before the LDS
    // atomics that use them)
    constexpr uint32_t U = 8u;
    hist_zero(cnt);
    for (uint32_t e0 = b0 + threadIdx.x; e0 < b1; e0 += U * PT_BIN_BLOCK) {
        uint32_t k[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            const uint32_t e = e0 + j * PT_BIN_BLOCK;
            k[j] = e < b1 ? P.key[e] : PT_BIN_NONE;
        }
#pragma unroll
        for (uint32_t j = 0; j < U; ++j)
            if (k[j] != PT_BIN_NONE) atomicAdd(&cnt[k[j]], 1u);
    }
    __syncthreads();
    for (int b = int(threadIdx.x); b < PT_BINS; b += PT_BIN_BLOCK) {
        const uint32_t c = cnt[b];
        if (c != 0u) cnt[b] = atomicAdd(&P.offs[b], c);
    }
    __syncthreads();
    for (uint32_t e0 = b0 + threadIdx.x; e0 < b1; e0 += U * PT_BIN_BLOCK) {
        uint32_t k[U];
#pragma unroll
        for (uint32_t j = 0; j < U; ++j) {
            const uint32_t e = e0 + j * PT_BIN_BLOCK;
            k[j] = e < b1 ? P.key[e] : PT_BIN_NONE;
        }
#pragma unroll
        for (uint32_t j = 0; j < U; ++j)
            if (k[j] != PT_BIN_NONE) P.idx[atomicAdd(&cnt[k[j]], 1u)] = e0 + j * PT_BIN_BLOCK;
    }
}

// trace: one wave per block, persistent.  The wave takes runs of the binned
// slots (so its lanes share their check[] set).  Windows of 64: the slots of
// the next window are loaded one window ahead, the current window's rays are
// gathered into staging registers and handed to free lanes by cross-lane
// moves.  Lanes run the MARCH -> NORMAL -> SHADE state machine of pt_path.h;
// a shaded path either ends (colour stored, end marker written) or writes
// its next ray to rout at its binned position.
//
// TAPS = false: a lane stops at the hit and writes its 16 B hit quad for the
// shade pass (PtPass.hq), which reads the ray itself from its slot and
// evaluates the normal taps (bin_shade_body).
//
// GEN (PtPass gen_trace, the first pass in position order): a window's
// rays are not loaded but made here, lane j the camera ray and bounds() mask
// of the sample at position wbase + j (gen_sample: frame-fastest, so a
// window is one pixel over 64 frames) -- what gen would have written
// (bin_gen_body), with all 64 lanes at once, and, for scenes of more than 32
// check[] entries, stored to its slot for the shade pass -- so the chunk
// needs no gen pass.
template <class Map, bool ST, bool TAPS = true, bool GEN = false>
__device__ __forceinline__ void bin_trace_body(const PtPass &P) {
    // the staged window, once its loads have landed: [part][lane], so a
    // refill reads a ray with 4 ds_read_b128 instead of 16 cross-lane moves
    __shared__ uint4 W[MapWide<Map>::v == 0 ? 4 : 5][64];  // (W[4]: check[] bits 64..127)
    const PtLaunch &L = P.L;
    const int lane = int(threadIdx.x);
    Stats<ST> st;
    st.init();
    const uint64_t t_start = st.clk();
    const uint32_t n = P.ctrl[0];
    // Run length: about 8 runs per wave, 64..run_max rays, whole windows.
    // (Measured: fixed 256-ray runs beat both longer runs and guided sizes
    // that shrink towards the end of the pass.)
    const uint32_t rmax = uint32_t(P.run_max);
    uint32_t R = n / (gridDim.x * 8u);
    R = R < 64u ? 64u : (R > rmax ? rmax : (R + 63u) & ~63u);
    // Run cursors: one per share of the pass (PT_RUN_SHARDS contiguous
    // shares, whole windows).  A wave takes runs from the share of its
    // workgroup's XCD (blockIdx % 8: workgroups go to the XCDs round-robin)
    // and, once that share is used up, from the next ones.  One device-scope
    // atomic word saturates at ~88 dequeues per us (MI355X_MICROARCH.md,
    // "dequeue"): the first pass of a C2 render asks for ~2.6e5 runs in ~3 ms.
    uint32_t shard = blockIdx.x % PT_RUN_SHARDS, tried = 0u;
    auto shard_lo = [&](uint32_t k) -> uint32_t {
        return k >= PT_RUN_SHARDS ? n : uint32_t((uint64_t(n >> 6) * k / PT_RUN_SHARDS) << 6);
    };
    // (lane 0) reserve a run of `len` positions: its start, and its end in
    // `end`; start == end == n once every share is used up
    auto take = [&](uint32_t len, uint32_t &end) -> uint32_t {
        while (tried < PT_RUN_SHARDS) {
            const uint32_t lo = shard_lo(shard), hi = shard_lo(shard + 1u);
            const uint32_t b = lo + atomicAdd(&P.ctrl[PT_CTRL_CURSOR(shard)], len);
            if (b < hi) {
                end = b + len < hi ? b + len : hi;
                return b;
            }
            shard = (shard + 1u) % PT_RUN_SHARDS;
            ++tried;
        }
        end = n;
        return n;
    };

    // runs [run_cur, run_end); the next run is reserved one run ahead
    uint32_t nxt = 0u, nxt_end = 0u;
    if (lane == 0) nxt = take(R, nxt_end);
    uint32_t run_cur = uint32_t(__builtin_amdgcn_readfirstlane(int(nxt)));
    uint32_t run_end = uint32_t(__builtin_amdgcn_readfirstlane(int(nxt_end)));
    if (lane == 0 && run_cur < n) nxt = take(R, nxt_end);
    auto next_window = [&](uint32_t &b, uint32_t &c) {
        if (run_cur >= run_end) {
            run_cur = uint32_t(__builtin_amdgcn_readfirstlane(int(nxt)));
            run_end = uint32_t(__builtin_amdgcn_readfirstlane(int(nxt_end)));
            if (lane == 0 && run_cur < n) nxt = take(R, nxt_end);
        }
        b = run_cur;
        c = run_end - run_cur < 64u ? run_end - run_cur : 64u;
        run_cur += c;
    };
    // next window: its slots, one per lane
    uint32_t nb = 0u, nc = 0u, nslot = 0u;
    next_window(nb, nc);
    if (!GEN && uint32_t(lane) < nc) nslot = P.idx[nb + uint32_t(lane)];
    // staged window: lane j holds the ray of binned position wbase + j
    uint32_t wbase = 0u, wcnt = 0u, wtake = 0u;
    float4 s0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s1 = s0, s2 = s0;
    uint4 s3 = make_uint4(0u, 0u, 0u, 0u);
    uint2 sh = make_uint2(0u, 0u);
    bool in_lds = false;  // the staged window has been copied to W
    auto stage = [&]() {
        wbase = nb;
        wcnt = nc;
        wtake = 0u;
        in_lds = false;
        if (GEN && uint32_t(lane) < wcnt) {
            const uint32_t i = wbase + uint32_t(lane), npix = uint32_t(P.n_pix);
            uint32_t f, pl;
            gen_sample(uint32_t(P.frames), i, f, pl);
            const uint32_t sid = colour_slot(uint32_t(P.frames), f, pl);  // (= i)
            (void)npix;
            int x, y;
            pixel_of(L, pl, x, y);
            uint32_t rg;
            pt_f3 o, d;
            // (fov through an empty asm: normalize's fov * fov, hoisted out of
            // the persistent loop, held a register there and spilled)
            float fov = L.fov;
            __asm__ volatile("" : "+v"(fov));
            camera_ray(x, y, int32_t(uint32_t(L.frame0) + f), L.width, L.height, L.aspect, fov, rg, o, d);
            st.add(PT_ST_SAMPLES);
            // the boxes no camera ray of the window can hit (every lane of a
            // full window is here, as the skip's wave reductions need)
            const uint64_t skip = wcnt == 64u ? primary_box_skip(L, o, d) : 0ull;
            const uint4 m = MapBounds<Map>::template mask_skip<ST>(L, o, d, skip, st);
            s0 = make_float4(o.x, o.y, o.z, d.x);
            s1 = make_float4(d.y, d.z, 1.0f, 1.0f);
            s2 = make_float4(1.0f, __uint_as_float(rg), __uint_as_float(sid), __uint_as_float(i));  // (aux: its slot)
            s3 = make_uint4(m.x, m.y, 0u, 0u);
            sh = make_uint2(m.z, m.w);
        } else if (uint32_t(lane) < wcnt) {
            const uint32_t slot = nslot;
            const uint4 *v = reinterpret_cast<const uint4 *>(P.rin + slot);
            const uint4 a = v[0], b = v[1], c = v[2];
            s0 = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
            s1 = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
            s2 = make_float4(__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z), __uint_as_float(c.w));
            s3 = v[3];
            if (wide_of<Map>(P)) sh = P.mask_hi[slot];
        }
        if (wcnt != 0u) {
            next_window(nb, nc);
            if (!GEN && uint32_t(lane) < nc) nslot = P.idx[nb + uint32_t(lane)];
        }
    };
    stage();

    int state = ST_FREE;
    uint32_t rng = 0u, sid = 0u, pos = 0u, slot = 0u;
    pt_f3 ro{0.0f, 0.0f, 0.0f}, rd{0.0f, 0.0f, 1.0f};
    pt_f3 thr{1.0f, 1.0f, 1.0f};
    int step = 0, mat = 0;  // (a lane's segment index is this pass's P.bounce)
    float t = 0.0f;
    float dv0 = 0.0f, dv1 = 0.0f, dv2 = 0.0f;
    Check ck{0ull, 0ull};

    auto hand_on = [&]() {
        if (state == ST_SHADE) {
            if (step < 0) {
                if (L.debug == 3) {  // bounce-count view
                    const pt_f3 c = final_color(L.debug, P.bounce, L.bounces, pt_f3{0.0f, 0.0f, 0.0f});
                    P.color[sid] = make_float4(c.x, c.y, c.z, 0.0f);
                }
                if constexpr (TAPS) P.rout[pos].q[2] = make_uint4(0u, 0u, sid, PT_AUX_MISS);
                else P.hq[pos] = make_uint4(0u, PT_AUX_MISS, 0u, slot);
                if constexpr (GEN) P.color[sid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // (no gen pass zeroed it)
            } else {
                if constexpr (TAPS) {  // hit record: hit point + normal differences
                    store_ray(P.rout + pos, ro, rd, thr, rng, sid, uint32_t(mat),
                              make_uint4(__float_as_uint(dv0), __float_as_uint(dv1), __float_as_uint(dv2), 0u));
                } else {  // hit quad: t, material, tap bound, slot (bin_shade_body)
                    P.hq[pos] = make_uint4(__float_as_uint(t), uint32_t(mat), __float_as_uint(dv0),
                                           GEN && P.gen_norec ? uint32_t(ck.lo) : slot);
                    if (wide_of<Map>(P))
                        P.hitn[pos] = make_float4(0.0f, 0.0f, __uint_as_float(uint32_t(ck.hi)),
                                                  __uint_as_float(uint32_t(ck.hi >> 32)));
                }
            }
            state = ST_FREE;
        }
    };

    // park the staged window in LDS (waits for its loads) and form the
    // wave's check[] union (Check.alo/ahi) for the scene kernels: the masks of
    // the lanes still mapping and of the whole window, so it also covers every
    // lane this window's refills start
    auto park = [&]() {
        const bool mapping_now = state == ST_MARCH || (TAPS && state == ST_NORMAL);
        const bool in_win = uint32_t(lane) < wcnt;
        ck.alo = wave_or_u64((mapping_now ? ck.lo : 0ull) |
                             (in_win ? (uint64_t(s3.x) | (uint64_t(s3.y) << 32)) : 0ull));
        ck.ahi = wide_of<Map>(P) ? wave_or_u64((mapping_now ? ck.hi : 0ull) |
                                      (in_win ? (uint64_t(sh.x) | (uint64_t(sh.y) << 32)) : 0ull))
                        : 0ull;
        W[0][lane] = make_uint4(__float_as_uint(s0.x), __float_as_uint(s0.y), __float_as_uint(s0.z),
                                __float_as_uint(s0.w));
        W[1][lane] = make_uint4(__float_as_uint(s1.x), __float_as_uint(s1.y), __float_as_uint(s1.z),
                                __float_as_uint(s1.w));
        W[2][lane] = make_uint4(__float_as_uint(s2.x), __float_as_uint(s2.y), __float_as_uint(s2.z),
                                __float_as_uint(s2.w));
        W[3][lane] = s3;
        if constexpr (MapWide<Map>::v != 0)
            if (wide_of<Map>(P)) W[4][lane] = make_uint4(sh.x, sh.y, 0u, 0u);
        if constexpr (GEN) {
            // the window's camera rays at their slots for the shade pass: 64
            // lanes, 64 contiguous records (whole lines) -- unless shade pass
            // 0 makes them again (gen_norec: 64 B per sample neither written
            // here nor gathered there)
            if (in_win && !P.gen_norec) {
                uint4 *r = reinterpret_cast<uint4 *>(P.rin + wbase + uint32_t(lane));
                r[0] = make_uint4(__float_as_uint(s0.x), __float_as_uint(s0.y), __float_as_uint(s0.z),
                                  __float_as_uint(s0.w));
                r[1] = make_uint4(__float_as_uint(s1.x), __float_as_uint(s1.y), __float_as_uint(s1.z),
                                  __float_as_uint(s1.w));
                r[2] = make_uint4(__float_as_uint(s2.x), __float_as_uint(s2.y), __float_as_uint(s2.z),
                                  __float_as_uint(s2.w));
                r[3] = s3;
                // (check[] bits 64..127 need no copy here: the shade pass
                // takes a hit's from its hitn entry, P.hitn)
            }
        }
        in_lds = true;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };

    for (;;) {
        uint64_t tm = st.clk();
        // ---- 1. refill free lanes from the staging window --------------
        const uint64_t freem = __ballot(state == ST_FREE);
        if (freem != 0ull && wcnt != 0u &&
            (__popcll(freem) >= P.refill_min || __ballot(state == ST_MARCH || state == ST_NORMAL) == 0ull)) {
            const uint32_t avail = wcnt - wtake, nf = uint32_t(__popcll(freem));
            const uint32_t take = nf < avail ? nf : avail;
            const int r = lane_rank(freem);
            const int src = int(wtake) + r;
            const bool got = state == ST_FREE && uint32_t(r) < take;
            if (!in_lds) park();  // first refill from this window
            float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f, b0 = 0.0f, b1 = 0.0f, b2 = 0.0f, b3 = 0.0f;
            float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
            uint32_t d0 = 0u, d1 = 0u, d2 = 0u, d3 = 0u, e0 = 0u, e1 = 0u;
            if (got) {
                const uint4 wa = W[0][src], wb = W[1][src], wc = W[2][src], wd = W[3][src];
                a0 = __uint_as_float(wa.x), a1 = __uint_as_float(wa.y), a2 = __uint_as_float(wa.z);
                a3 = __uint_as_float(wa.w);
                b0 = __uint_as_float(wb.x), b1 = __uint_as_float(wb.y), b2 = __uint_as_float(wb.z);
                b3 = __uint_as_float(wb.w);
                c0 = __uint_as_float(wc.x), c1 = __uint_as_float(wc.y), c2 = __uint_as_float(wc.z);
                c3 = __uint_as_float(wc.w);
                d0 = wd.x, d1 = wd.y, d2 = wd.z, d3 = wd.w;
                if constexpr (MapWide<Map>::v != 0) {
                    if (wide_of<Map>(P)) {
                        const uint4 we = W[4][src];
                        e0 = we.x;
                        e1 = we.y;
                    }
                }
            }
            if (got) {
                ro = pt_f3{a0, a1, a2};
                rd = pt_f3{a3, b0, b1};
                thr = pt_f3{b2, b3, c0};
                rng = __float_as_uint(c1);
                sid = __float_as_uint(c2);
                slot = __float_as_uint(c3);  // (a ray's aux: its slot)
                ck.lo = uint64_t(d0) | (uint64_t(d1) << 32);
                (void)d2;
                (void)d3;
                ck.hi = uint64_t(e0) | (uint64_t(e1) << 32);
                pos = wbase + uint32_t(src);
                t = 0.0f;
                step = 0;
                state = ST_MARCH;
            }
            wtake += take;
            if (wtake == wcnt) stage();  // wcnt = 0: no rays left for this wave
        }
        const bool more = wcnt != 0u;
        tm = st.lap(PT_ST_CYC_REFILL, tm);

        // ---- 2. one map() per marching / normal-tap lane ------------------
        // (TAPS = false: no lane is ever NORMAL here, the shade pass taps)
        const bool mapping = state == ST_MARCH || (TAPS && state == ST_NORMAL);
        st.add(PT_ST_LANE_IDLE, mapping ? 0u : 1u);
        st.add(PT_ST_IDLE_SHADE, state == ST_SHADE ? 1u : 0u);
        st.add(PT_ST_IDLE_FREE, state == ST_FREE ? 1u : 0u);
        if (lane == 0) st.add(PT_ST_WAVE_ITERS);
        if (__ballot(mapping) != 0ull) {
            if (lane == 0) st.add(PT_ST_WAVE_MAPS);
            if (mapping) {
                float qx, qy, qz;
                map_point(TAPS ? state : int(ST_MARCH), step, ro, rd, t, qx, qy, qz);
                uint64_t live = 0;  // (the taps' live mask: unused here)
                const Hit h = Map::template eval<ST>(L, qx, qy, qz, ck, __builtin_inff(), __builtin_inff(), live, st);
                after_map<ST, !TAPS>(h, state, step, t, ro, rd, mat, dv0, dv1, dv2, st);
                if constexpr (!TAPS) {
                    if (state == ST_NORMAL) {  // hit: the shade pass takes the taps
                        dv0 = tap_bound(h.d, qx, qy, qz, t, L.bound_k);
                        state = ST_SHADE;
                    }
                }
            }
        }
        tm = st.lap(PT_ST_CYC_MAP, tm);

        // ---- 3. hand finished segments on: a miss ends the path (its
        // colour slot already holds its radiance), a hit goes to the shade
        // pass as one 64 B record (PtRay)
        hand_on();
        tm = st.lap(PT_ST_CYC_SHADE, tm);
        if (!more && __ballot(state != ST_FREE) == 0ull) break;
    }
    (void)st.lap(PT_ST_CYC_TOTAL, t_start);
    flush_stats<ST>(L, st);
}

// fold: every pixel mixes its frames in order (test_compute.glsl:240-245).
#define PT_FOLD_SLICE 8  // frames per LDS slice of the fold
__device__ __forceinline__ void bin_fold_body(const PtPass &P) {
    // A block folds PT_BIN_BLOCK consecutive local pixels.  Each pipeline's
    // colour region holds its frames as [pixel][frame], so the block's
    // pixels' next PT_FOLD_SLICE frames are runs of PT_FOLD_SLICE float4 per
    // pixel: the block loads them together (8 threads per 128 B run) into
    // LDS, then each thread mixes its pixel's frames in frame order.
    __shared__ float4 tile[PT_BIN_BLOCK][PT_FOLD_SLICE + 1];  // (+1: no bank conflicts between rows)
    const PtLaunch &L = P.L;
    const uint32_t t = threadIdx.x, pl0 = blockIdx.x * PT_BIN_BLOCK, pl = pl0 + t;
    const uint32_t npix = uint32_t(P.n_pix), fr = uint32_t(P.frames);
    const uint32_t nl = uint32_t(P.lanes > 0 ? P.lanes : 1);
    int x = 0, y = 0;
    bool mine = pl < npix && L.write;
    if (mine) {
        pixel_of(L, pl, x, y);
        mine = x < L.width && y < L.height;
    }
    float4 *texel = mine ? reinterpret_cast<float4 *>(L.accum + (size_t(y) * size_t(L.width) + size_t(x)) * 4) : nullptr;
    if (L.debug != 0) {  // direct store of the chunk's (single) frame: one pipeline, one frame
        if (mine) {
            const float4 c = P.color[pl];
            *texel = make_float4(c.x, c.y, c.z, 1.0f);
        }
        return;
    }
    float ar = 0.0f, ag = 0.0f, ab = 0.0f;
    if (mine) {
        const float4 v = *texel;
        ar = v.x;
        ag = v.y;
        ab = v.z;
    }
    uint32_t f0 = 0u;  // the chunk frame of region j's first frame
    for (uint32_t j = 0u; j < nl; ++j) {
        const uint32_t fl = fr / nl + (j < fr % nl ? 1u : 0u);
        const float4 *reg = P.color + size_t(f0) * npix;
        for (uint32_t s0 = 0u; s0 < fl; s0 += PT_FOLD_SLICE) {
            const uint32_t sn = fl - s0 < PT_FOLD_SLICE ? fl - s0 : PT_FOLD_SLICE;
            __syncthreads();  // (the previous slice's reads are done)
            for (uint32_t e = t; e < PT_BIN_BLOCK * PT_FOLD_SLICE; e += PT_BIN_BLOCK) {
                const uint32_t q = e / PT_FOLD_SLICE, k = e % PT_FOLD_SLICE;
                if (k < sn && pl0 + q < npix) tile[q][k] = reg[size_t(pl0 + q) * fl + s0 + k];
            }
            __syncthreads();
            if (mine) {
                for (uint32_t k = 0u; k < sn; ++k) {
                    const float4 c = tile[t][k];
                    const int32_t lc = int32_t(uint32_t(L.last_clear0) + f0 + s0 + k);
                    const float w = 1.0f / float(lc + 1), omw = 1.0f - w;
                    ar = ar * omw + c.x * w;
                    ag = ag * omw + c.y * w;
                    ab = ab * omw + c.z * w;
                }
            }
        }
        f0 += fl;
    }
    if (mine) *texel = make_float4(ar, ag, ab, 1.0f);
}

}  // namespace pt
