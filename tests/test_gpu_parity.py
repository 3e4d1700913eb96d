"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (BASELINE.json north star): per-pixel RMS < 1e-5 over all pixels and
channels.  The semantics contract makes the two bit-exact, so
the tests also report the bit-exact texel fraction and require it to be 1
where no transcendental-free difference is expected.
"""
import ctypes

import numpy as np
import pytest

from compute_path_tracer_amd import _native as N
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.path_tracer import PathTracer
from compute_path_tracer_amd.sdf_editor import CompData
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5


KERNELS = {"simple": {"kernel": "simple", "jit": 0}, "wave": {"kernel": "wave", "jit": 0},
           "jit": {"kernel": "wave", "jit": 1, "jit_bake": 0}, "binned": {"kernel": "binned", "jit": 0},
           "binned_jit": {"kernel": "binned", "jit": 1, "jit_bake": 0},
           "binned_bake": {"kernel": "binned", "jit": 1, "jit_bake": 1},
           "binned_tier": {"kernel": "binned", "jit": 1, "jit_bake": 2},
           # normal taps in the trace pass instead of the shade pass
           "binned_trace_taps": {"kernel": "binned", "jit": 1, "jit_bake": 2, "shade_taps": 0}}
ALL = ["simple", "wave", "jit", "binned", "binned_jit", "binned_bake", "binned_tier", "binned_trace_taps"]


def _tier_up(pt, opts):
    """jit_bake 2: wait for the values-baked build, so the test runs on it."""
    if opts.get("jit_bake") == 2:
        pt.set_option("jit_wait", 1)
        assert pt.get_option("jit_tier_active") == 1.0, pt.jit_log()


def _render_pair(ed, w, h, spp, bounces, debug=0, frame=1, last_clear=1, fov=1.0, aspect=None, kernel="jit",
                 shade_batch=None, bin_samples=None, bin_lanes=None, extra=None):
    prog = ed.compile(CompData())
    st = N.Settings(debug=debug, bounces=bounces, scale=1.0, fov=fov, aabb=0)
    opts = dict(KERNELS[kernel])
    opts.update(extra or {})
    if shade_batch:
        opts["shade_batch"] = shade_batch
    if bin_samples:
        opts["bin_samples"] = bin_samples
    if bin_lanes:
        opts["bin_lanes"] = bin_lanes
    pt = PathTracer(w, h, prog, settings=st, options=opts)
    if opts["jit"]:
        assert pt.get_option("jit_active") == 1.0, pt.jit_log()
    _tier_up(pt, opts)
    a = float(np.float32(w) / np.float32(h)) if aspect is None else aspect
    pt.dispatch(N.Constants(time=0.0, frame=frame, aspect=a, last_clear=last_clear), spp)
    gpu = pt.read_image()
    pt.close()
    ref = O.OracleScene(ed.rows()).render(w, h, O.Constants(0.0, frame, a, last_clear),
                                          O.Settings(debug, bounces, 1.0, fov, 0), spp)
    return gpu, ref


def _report(gpu, ref):
    d = gpu.astype(np.float64) - ref.astype(np.float64)
    both_nan = np.isnan(gpu) & np.isnan(ref)
    d[both_nan] = 0.0
    rms = float(np.sqrt(np.mean(d ** 2)))
    exact = float(np.mean((gpu.view(np.uint32) == ref.view(np.uint32)) | both_nan))
    return rms, exact


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("name,w,h,spp,bounces", [
    ("c1", 256, 256, 1, 1),        # BASELINE config 1 in full
    ("c2", 96, 64, 4, 4),
    ("c3", 96, 54, 2, 8),
    ("nested", 64, 64, 3, 6),
    ("wide", 48, 32, 2, 6),        # 124 check[] entries: the high mask words
    ("c3_noaabb", 40, 24, 2, 8),   # no bounds() boxes: every mask empty, one bin
    ("cull", 64, 40, 3, 6),        # distance-bound culling near its threshold, rule on/off per union
    ("tiny", 64, 40, 3, 4),        # unions of scale 1e-3: culled first shapes in open space (MAXHIT * s = 10)
    ("farbox", 64, 40, 3, 4),      # a box coordinate beyond the reciprocal guard: IEEE-division bounds()
])
def test_parity_path_trace(gpu, name, w, h, spp, bounces, kernel):
    gpu_img, ref = _render_pair(scenes.SCENES[name](), w, h, spp, bounces, kernel=kernel)
    rms, exact = _report(gpu_img, ref)
    print(f"{kernel} {name}: rms={rms:.3e} bit-exact={exact:.5f} mean={ref[..., :3].mean():.5f}")
    assert ref[..., :3].mean() > 0
    assert rms < RMS_TOL
    assert exact == 1.0


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("debug", [1, 2, 3])
def test_parity_debug_views(gpu, debug, kernel):
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 80, 45, 2, 8, debug=debug, kernel=kernel)
    rms, exact = _report(gpu_img, ref)
    assert rms < RMS_TOL and exact == 1.0


@pytest.mark.parametrize("kernel", ["wave", "jit", "binned", "binned_jit"])
@pytest.mark.parametrize("shade_batch", [1, 7, 64])
def test_wave_kernel_schedule_invariance(gpu, shade_batch, kernel):
    """Shading batch size changes the schedule only, never the result; spp
    above the LDS ring size exercises the in-order fold."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 40, 24, 19, 8, kernel=kernel, shade_batch=shade_batch)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0, (shade_batch, rms)


@pytest.mark.parametrize("kernel", ["binned_jit", "binned_tier"])
@pytest.mark.parametrize("fov", [0.02, 1.0, 5.0])
def test_first_pass_box_skip_edges(gpu, kernel, fov):
    """The first pass's wave-level box skip at its edges:
    72x40 puts windows across the image centre (uv = 0, so a window's rd.x
    or rd.y changes sign and that axis gives no bound), and a narrow and a
    wide field of view (fov is rd.z before normalising: at 0.02 a window's
    rays are nearly parallel to the image plane's axes, at 5 nearly along
    z).  Bit-exact against the oracle on C3's 24 boxes."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 72, 40, 2, 3, fov=fov, kernel=kernel)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0 and rms == 0.0, (rms, exact)


@pytest.mark.parametrize("kernel", ["jit", "binned_jit"])
def test_long_dispatch_chunks(gpu, kernel):
    """spp > 64 is split into several launches that continue frame/last_clear."""
    gpu_img, ref = _render_pair(scenes.c1_default(), 16, 16, 70, 1, kernel=kernel)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0


@pytest.mark.parametrize("bin_samples", [64, 1000, 4096, 1 << 20])
def test_binned_sub_chunks(gpu, bin_samples):
    """The binned pipeline splits a dispatch into sub-chunks of frames that fit
    its sample budget (one frame when the budget is below the pixel count);
    the fold continues last_clear across them."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 40, 24, 11, 8, kernel="binned_jit", bin_samples=bin_samples)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0, rms


@pytest.mark.parametrize("bin_lanes", [1, 2, 3, 4])
@pytest.mark.parametrize("spp,bin_samples", [(1, None), (2, None), (11, None), (11, 3000), (7, 64)])
def test_binned_lanes(gpu, bin_lanes, spp, bin_samples):
    """A chunk's frames split over one to four pipelines on separate streams
    (ragged splits, one-frame chunks, several chunks) fold to the same image."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 40, 24, spp, 8, kernel="binned_tier", bin_samples=bin_samples,
                                bin_lanes=bin_lanes)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0, rms


@pytest.mark.parametrize("kernel", ["binned", "binned_jit", "binned_tier"])
@pytest.mark.parametrize("bin_table", [0, 1])
@pytest.mark.parametrize("name,spp,bin_lanes", [("c3", 4, 2), ("c3", 3, 3), ("cull", 3, 1), ("c3_noaabb", 2, 2)])
def test_bin_table_schedule_only(gpu, kernel, bin_table, name, spp, bin_lanes):
    """Bins from the table of check[] sets (pt_binned.h bin_of, DESIGN.md
    3.21) or from the hash: the schedule changes, the image does not.  C3
    (24 boxes) and `cull` use the table, with one to three pipelines sharing
    it; C3 without boxes has one set."""
    gpu_img, ref = _render_pair(scenes.SCENES[name](), 96, 54, spp, 8, kernel=kernel, bin_lanes=bin_lanes,
                                extra={"bin_table": bin_table})
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0 and rms == 0.0, (rms, exact)


@pytest.mark.parametrize("kernel", ["binned_jit", "binned_tier"])
@pytest.mark.parametrize("bin_lanes", [1, 2])
def test_first_pass_without_records(gpu, kernel, bin_lanes):
    """Whole tiles, so the first pass makes its own camera rays (gen_trace);
    C3's 24 check[] entries, so it stores no ray records and shade pass 0
    makes them again, with one and two pipelines:
    bit-exact against the oracle."""
    ed = scenes.c3_graph32()
    prog = ed.compile(CompData())
    w, h, spp = 64, 48, 6
    opts = dict(KERNELS[kernel], bin_lanes=bin_lanes)
    pt = PathTracer(w, h, prog, settings=N.Settings(debug=0, bounces=8, scale=1.0, fov=1.0, aabb=0), options=opts)
    _tier_up(pt, opts)
    a = float(np.float32(w) / np.float32(h))
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=a, last_clear=1), spp)
    gpu_img = pt.read_image()
    assert pt.get_option("gen_trace") == 1.0 and pt.get_option("gen_norec") == 1.0
    pt.close()
    ref = O.OracleScene(ed.rows()).render(w, h, O.Constants(0.0, 1, a, 1), O.Settings(0, 8, 1.0, 1.0, 0), spp)
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0 and rms == 0.0, (rms, exact)


@pytest.mark.parametrize("kernel", ["jit", "binned_jit"])
def test_empty_scene_is_black(gpu, kernel):
    gpu_img, ref = _render_pair(scenes.empty(), 40, 24, 2, 4, kernel=kernel)
    assert np.all(gpu_img[..., :3] == 0) and np.all(gpu_img[..., 3] == 1)
    assert np.array_equal(gpu_img, ref)


@pytest.mark.parametrize("kernel", ["jit", "binned_jit"])
def test_ragged_and_edge_sizes(gpu, kernel):
    for (w, h) in [(1, 1), (7, 3), (9, 17), (65, 1)]:
        gpu_img, ref = _render_pair(scenes.c2_sphere_box_torus(), w, h, 2, 3, kernel=kernel)
        rms, exact = _report(gpu_img, ref)
        assert exact == 1.0, (w, h)


def test_progressive_equals_batched(gpu):
    """spp successive 1-spp frames == one spp dispatch (path_tracer.rs:110-111)."""
    ed = scenes.c2_sphere_box_torus()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=4, scale=1.0, fov=1.0, aabb=0)
    a = PathTracer(48, 32, prog, settings=st)
    b = PathTracer(48, 32, prog, settings=st)
    for _ in range(5):
        a.update()
        a.compute_pass()
    b.update()
    b.constants.frame -= 1
    b.constants.last_clear -= 1
    b.render(5)
    ia, ib = a.read_image(), b.read_image()
    ref = O.OracleScene(ed.rows()).render(48, 32, O.Constants(0.0, 1, float(np.float32(48) / np.float32(32)), 1),
                                          O.Settings(0, 4, 1.0, 1.0, 0), 5)
    bad_a = (ia.view(np.uint32) != ref.view(np.uint32)).any(-1)
    bad_b = (ib.view(np.uint32) != ref.view(np.uint32)).any(-1)
    assert not bad_a.any() and not bad_b.any(), (np.argwhere(bad_a)[:8].tolist(), np.argwhere(bad_b)[:8].tolist())
    assert a.constants.frame == b.constants.frame == 5


@pytest.mark.parametrize("kernel", ["jit", "binned_jit"])
def test_tiles_union_is_full_image(gpu, kernel):
    ed = scenes.c3_graph32()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=8, scale=1.0, fov=1.0, aabb=0)
    c = N.Constants(time=0.0, frame=3, aspect=float(np.float32(72) / np.float32(40)), last_clear=1)
    full = PathTracer(72, 40, prog, settings=st)
    full.dispatch(c, 2)
    ref = full.read_image()
    acc = np.zeros_like(ref)
    for r in range(3):
        p = PathTracer(72, 40, prog, settings=st, options=KERNELS[kernel])
        p.set_tiles(r, 3)
        p.dispatch(c, 2)
        acc += p.read_image()
        p.close()
    assert np.array_equal(acc.view(np.uint32), ref.view(np.uint32))


def test_jit_recompiles_only_on_flag_change(gpu):
    """Value edits reuse the scene kernel; an identity flag flip (rotation 0 ->
    non-zero) rebuilds it; results stay exact throughout."""
    ed = scenes.c2_sphere_box_torus()
    cd = CompData()
    prog = ed.compile(cd)
    st = N.Settings(debug=0, bounces=3, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(40, 30, prog, settings=st, options={"jit": 1})
    assert pt.get_option("jit_active") == 1.0
    sph = ed.header_unions[0].children_shapes[1]
    sph.transform.position.x.set(-0.3)  # value only
    ed.data_update(cd)
    pt.set_data(cd.data_array.as_array())
    assert pt.get_option("jit_active") == 1.0
    sph.transform.rotation.y.set(0.7)  # rotation about y becomes non-identity
    ed.data_update(cd)
    pt.set_data(cd.data_array.as_array())
    assert pt.get_option("jit_active") == 1.0
    c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(40) / np.float32(30)), last_clear=1)
    pt.dispatch(c, 2)
    gpu_img = pt.read_image()
    ref = O.OracleScene(ed.rows()).render(40, 30, O.Constants(0.0, 1, c.aspect, 1), O.Settings(0, 3, 1.0, 1.0, 0), 2)
    assert np.array_equal(gpu_img.view(np.uint32), ref.view(np.uint32))


def test_value_update_without_recompile(gpu):
    ed = scenes.c2_sphere_box_torus()
    cd = CompData()
    prog = ed.compile(cd)
    st = N.Settings(debug=0, bounces=3, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(40, 30, prog, settings=st)
    sph = ed.header_unions[0].children_shapes[1]
    sph.transform.position.x.set(-0.3)
    ed.data_update(cd)
    pt.set_data(cd.data_array.as_array())
    c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(40) / np.float32(30)), last_clear=1)
    pt.dispatch(c, 2)
    gpu_img = pt.read_image()
    ref = O.OracleScene(ed.rows()).render(40, 30, O.Constants(0.0, 1, c.aspect, 1), O.Settings(0, 3, 1.0, 1.0, 0), 2)
    assert np.array_equal(gpu_img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("kernel", ALL)
def test_work_counters_match_oracle(gpu, kernel):
    ed = scenes.c3_graph32()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=8, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(64, 40, prog, settings=st, options=KERNELS[kernel])
    _tier_up(pt, KERNELS[kernel])
    a = float(np.float32(64) / np.float32(40))
    got = pt.stats(N.Constants(time=0.0, frame=1, aspect=a, last_clear=1), 2)
    _, ct = O.OracleScene(ed.rows()).render(64, 40, O.Constants(0.0, 1, a, 1), O.Settings(0, 8, 1.0, 1.0, 0), 2,
                                            counters=True)
    for k in ("samples", "segments", "march_steps", "normal_maps", "shaded", "aabb_tests", "xform_union",
              "xform_shape", "sdf_sphere", "sdf_cube", "sdf_octahedron", "comb_union", "comb_sub", "comb_assign",
              "rr_break"):
        assert got[k] == ct[k], (k, got[k], ct[k])
    # where the normal taps ran: the shade pass (scene kernels, shade_taps on)
    # reports them in its own share, which bench.py keeps out of the trace
    # pass's flops
    taps = pt.tap_stats()
    if KERNELS[kernel]["kernel"] == "binned" and KERNELS[kernel]["jit"] and pt.get_option("shade_taps") == 1.0:
        assert taps["normal_maps"] == ct["normal_maps"] and taps["march_steps"] == 0
        assert 0 < taps["xform_shape"] < got["xform_shape"]
    else:
        assert all(v == 0 for v in taps.values()), taps
    pt.close()


def _oracle_tiles(ed, w, h, spp, bounces, tiles):
    """The oracle's render of each 8x8 tile alone (rank = tile, nranks =
    #tiles), tiles in parallel (ctypes drops the GIL in pto_render)."""
    from concurrent.futures import ThreadPoolExecutor

    tx, ntiles = (w + 7) // 8, ((w + 7) // 8) * ((h + 7) // 8)
    aspect = float(np.float32(w) / np.float32(h))
    osc = O.OracleScene(ed.rows())

    def one(t):
        ref = osc.render(w, h, O.Constants(0.0, 1, aspect, 1), O.Settings(0, bounces, 1.0, 1.0, 0), spp, rank=t,
                         nranks=ntiles, threads=1)
        y0, x0 = (t // tx) * 8, (t % tx) * 8
        return ref[y0:y0 + 8, x0:x0 + 8].copy()

    with ThreadPoolExecutor(max_workers=16) as ex:
        return dict(zip(tiles, ex.map(one, tiles)))


# BASELINE configs at their full size and spp (C5: 2^31 samples, four 2^29
# chunks; C4: the 8-GPU image on one GPU)
FULL_CONFIGS = ["c2", "c3", "c5", "c4"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", FULL_CONFIGS)
def test_full_size_tiles_match_oracle(gpu, name):
    """BASELINE configs at full resolution and full spp: 8 random 8x8 tiles,
    plus the tiles holding a non-finite texel (normalize of a zero vector
    upstream; at most 16), against the oracle rendering just that tile."""
    scene, w, h, spp, bounces = scenes.CONFIGS[name]
    ed = scenes.SCENES[scene]()
    st = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(w, h, ed.compile(CompData()), settings=st)
    pt.set_option("jit_wait", 1)
    aspect = float(np.float32(w) / np.float32(h))
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)
    img = pt.read_image()
    chunk = pt.get_option("bin_samples")
    pt.close()
    if name == "c5":
        assert w * h * spp > 2 * chunk  # the multi-chunk path at full size
    tx, ntiles = (w + 7) // 8, ((w + 7) // 8) * ((h + 7) // 8)
    bad = sorted({(int(y) // 8) * tx + int(x) // 8 for y, x in np.argwhere(~np.isfinite(img[..., :3]).all(-1))})
    print(f"{name}: {len(bad)} tiles with non-finite texels, mean {np.nanmean(img[..., :3]):.5f}")
    tiles = sorted(set(np.random.default_rng(11).choice(ntiles, 8, replace=False).tolist()) | set(bad[:16]))
    for t, ref in _oracle_tiles(ed, w, h, spp, bounces, tiles).items():
        y0, x0 = (t // tx) * 8, (t % tx) * 8
        a = img[y0:y0 + 8, x0:x0 + 8]
        assert np.array_equal(a.view(np.uint32), ref.view(np.uint32)), t


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("bounces", [0, 16, 32])
def test_parity_bounce_range(gpu, bounces, kernel):
    """The Settings slider range (path_tracer.rs:160, 0..=32): segments
    i = 0..=bounces (test_compute.glsl:99), so 1, 17 and 33 passes of the
    binned pipeline, deep Russian roulette and ping-pong buffers."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 48, 32, 3, bounces, kernel=kernel)
    rms, exact = _report(gpu_img, ref)
    assert ref[..., :3].mean() > 0
    assert rms < RMS_TOL and exact == 1.0, (rms, exact)


@pytest.mark.parametrize("kernel", ALL)
@pytest.mark.parametrize("bounces", [0, 32])
def test_bounce_heat_map_edges(gpu, bounces, kernel):
    """debug 3 stores i / bounces (test_compute.glsl:163): at bounces 0 that
    is 0 / 0 = NaN for a miss and 1 / 0 = +inf for a hit; bit patterns must
    match the oracle, NaNs included."""
    gpu_img, ref = _render_pair(scenes.c3_graph32(), 40, 24, 2, bounces, debug=3, kernel=kernel)
    assert np.array_equal(gpu_img.view(np.uint32), ref.view(np.uint32))
    if bounces == 0:
        assert np.isnan(ref[..., 0]).any() and np.isinf(ref[..., 0]).any()


@pytest.mark.timeout(600)
def test_tile_split_2160p_eight_ranks(gpu):
    """C4's split: eight contexts in one process, each owning
    the 8x8 tiles t % 8 == rank of the 3840x2160 image; their images summed
    on the host equal the one-context render bit for bit (non-owned texels
    are exactly 0)."""
    scene, w, h, _, bounces = scenes.CONFIGS["c4"]
    ed = scenes.SCENES[scene]()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
    c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(w) / np.float32(h)), last_clear=1)
    spp = 16
    full = PathTracer(w, h, prog, settings=st)
    full.dispatch(c, spp)
    want = full.read_image()
    full.close()
    acc = np.zeros_like(want)
    owned = np.zeros(want.shape[:2], np.int32)
    for r in range(8):
        p = PathTracer(w, h, prog, settings=st)
        p.set_tiles(r, 8)
        p.dispatch(c, spp)
        part = p.read_image()
        p.close()
        nz = (part.view(np.uint32) != 0).any(-1)
        owned += nz
        acc += part
    assert owned.max() == 1  # every texel rendered by at most one rank
    assert np.array_equal(acc.view(np.uint32), want.view(np.uint32))


def test_rccl_single_rank_reduce_and_errors(gpu):
    """pt_comm_init / pt_reduce_accum / pt_read_reduced through RCCL on one
    GPU (a 1-rank communicator: the reduce is a copy), plus their argument
    and state errors."""
    L = N.lib()
    ed = scenes.c2_sphere_box_torus()
    st = N.Settings(debug=0, bounces=3, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(40, 24, ed.compile(CompData()), settings=st)
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=float(np.float32(40) / np.float32(24)), last_clear=1), 3)
    with pytest.raises(N.NativeError) as e:
        pt.reduce(0)  # before pt_comm_init
    assert e.value.code == N.PT_ERR_STATE
    with pytest.raises(N.NativeError) as e:
        pt.read_reduced()
    assert e.value.code == N.PT_ERR_STATE
    with pytest.raises(N.NativeError) as e:
        pt.comm_size()
    assert e.value.code == N.PT_ERR_STATE
    uid = PathTracer.comm_unique_id()
    assert len(uid) == N.PT_COMM_ID_BYTES
    with pytest.raises(N.NativeError) as e:
        pt.comm_init(1, 1, uid)  # rank >= nranks
    assert e.value.code == N.PT_ERR_INVALID
    pt.comm_init(1, 0, uid)
    assert pt.comm_size() == 1  # (ncclCommCount: what bench.py reports as rccl_ranks)
    for root in (-1, 1):
        with pytest.raises(N.NativeError) as e:
            pt.reduce(root)
        assert e.value.code == N.PT_ERR_INVALID
    pt.reduce(0)
    got = pt.read_reduced()
    assert np.array_equal(got.view(np.uint32), pt.read_image().view(np.uint32))
    small = np.zeros(4, np.float32)
    assert L.pt_read_reduced(pt._ctx, small.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 16) == N.PT_ERR_SIZE
    pt.close()


def test_jit_tier_up_follows_value_edits(gpu):
    """jit_bake 2: the table kernel serves at once; the values-baked build
    takes over after jit_wait; a value edit drops it (stale literals) until
    the rebuilt one is waited for.  Every image stays exact."""
    ed = scenes.c2_sphere_box_torus()
    cd = CompData()
    prog = ed.compile(cd)
    st = N.Settings(debug=0, bounces=3, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(40, 30, prog, settings=st, options={"kernel": "binned", "jit": 1, "jit_bake": 2})
    c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(40) / np.float32(30)), last_clear=1)

    def check():
        pt.clear()
        pt.dispatch(c, 2)
        ref = O.OracleScene(ed.rows()).render(40, 30, O.Constants(0.0, 1, c.aspect, 1), O.Settings(0, 3, 1.0, 1.0, 0),
                                              2)
        assert np.array_equal(pt.read_image().view(np.uint32), ref.view(np.uint32))

    check()
    pt.set_option("jit_wait", 1)
    assert pt.get_option("jit_tier_active") == 1.0  # (jit_tier_seconds is 0 on a process-cache hit)
    check()
    sph = ed.header_unions[0].children_shapes[1]
    sph.transform.position.x.set(-0.25)  # value only: the baked build is stale
    ed.data_update(cd)
    pt.set_data(cd.data_array.as_array())
    assert pt.get_option("jit_tier_active") == 0.0
    check()
    pt.set_option("jit_wait", 1)
    assert pt.get_option("jit_tier_active") == 1.0
    check()
    pt.close()


def test_deprecated_map_scene(gpu):
    """The reference's saved map (assets/maps/test.json fixture) through the
    default kernel, against the oracle."""
    import os

    from compute_path_tracer_amd.scenes import deprecated_map

    ed = deprecated_map(os.path.join(os.path.dirname(__file__), "golden", "maps_test.json"))
    gpu_img, ref = _render_pair(ed, 64, 40, 3, 6, kernel="binned_tier")
    rms, exact = _report(gpu_img, ref)
    assert exact == 1.0, rms


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_shipped_scene_kernels_in_a_torch_process(gpu, name):
    """This process imported torch before the library (conftest's GPU probe),
    so it holds torch's bundled hipRTC; the BASELINE scenes' kernels still
    come from lib/jitcache, built by build() with this image's hipRTC
    (DESIGN.md 5): the 8-wave build runs, for the table kernel and
    the values-baked tier-up alike, and renders the oracle's image."""
    import sys

    assert "torch" in sys.modules
    ed = scenes.SCENES[name]()
    prog = ed.compile(CompData())
    st = N.Settings(debug=0, bounces=3, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(48, 32, prog, settings=st, options={"kernel": "binned", "jit": 1, "jit_bake": 2})
    assert pt.get_option("jit_trace_waves") == 8 and pt.get_option("jit_shade_waves") == 8
    assert pt.get_option("jit_seconds") < 1.0  # (a cache hit, not a 5-25 s compile)
    pt.set_option("jit_wait", 1)
    assert pt.get_option("jit_tier_active") == 1.0
    assert pt.get_option("jit_trace_waves") == 8 and pt.get_option("jit_shade_waves") == 8
    a = float(np.float32(48) / np.float32(32))
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=a, last_clear=1), 2)
    gpu_img = pt.read_image()
    pt.close()
    ref = O.OracleScene(ed.rows()).render(48, 32, O.Constants(0.0, 1, a, 1), O.Settings(0, 3, 1.0, 1.0, 0), 2)
    assert np.array_equal(gpu_img.view(np.uint32), ref.view(np.uint32))
