"""bench.py's algorithmic accounting, host side: the per-kernel
flop split covers the whole pipeline exactly once, and the pipeline-bytes
model adds up.  Counters from the oracle's instrumented render of a small
C3 frame (the same events the GPU's stats kernels count)."""
import numpy as np
import pytest

import bench
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd.sdf_editor import CompData
from oracle import oracle as O


@pytest.fixture(scope="module")
def counters():
    ed = scenes.c3_graph32()
    prog = ed.compile(CompData())
    w, h = 48, 32
    _, ct = O.OracleScene(ed.rows()).render(w, h, O.Constants(0.0, 1, float(np.float32(w) / np.float32(h)), 1),
                                            O.Settings(0, 8, 1.0, 1.0, 0), 2, counters=True)
    return prog, ct, w * h


def _taps_share(ct: dict) -> dict:
    """A stand-in for the stats run's shade-pass tap half: every calc_normal
    map() of the oracle (the counters split it out on the GPU)."""
    taps = {k: 0 for k in ct}
    taps["normal_maps"] = ct["normal_maps"]
    return taps


@pytest.mark.parametrize("gen_trace", [True, False])
def test_flop_split_covers_the_pipeline_once(counters, gen_trace):
    prog, ct, _ = counters
    st = dict(ct, wave_maps=0, wave_shapes=0)
    taps = _taps_share(ct)
    total = bench.algorithmic_flops(st)
    trace = bench.trace_flops(st, taps, prog.n_aabb, gen_trace)
    shade = bench.shade_flops(st, taps, prog.n_aabb)
    gen = 0.0 if gen_trace else (bench.W_CAMERA + bench.W_AABB * prog.n_aabb) * st["samples"]
    fold = bench.W_ACCUM * st["samples"]
    assert trace > 0 and shade > 0
    assert trace + shade + gen + fold == pytest.approx(total, rel=0, abs=1e-3)
    # the primary rays' bounds() are never the shade pass's: one test per box
    # of each primary segment
    assert st["aabb_tests"] >= st["samples"] * prog.n_aabb
    if gen_trace:  # the first trace pass carries the camera rays and primary bounds()
        assert trace - bench.trace_flops(st, taps, prog.n_aabb, False) == pytest.approx(
            (bench.W_CAMERA + bench.W_AABB * prog.n_aabb) * st["samples"])


def test_pipeline_bytes_add_up(counters):
    _, ct, pixels = counters
    # (the oracle does not count first-segment hits; a stand-in below the samples)
    ct = dict(ct, shaded_first=ct["samples"] * 3 // 4)
    for gen_trace, gen_norec in ((True, False), (False, False), (True, True)):
        parts = bench.pipeline_bytes(ct, pixels, gen_trace=gen_trace, gen_norec=gen_norec)
        assert parts["total"] == pytest.approx(sum(v for k, v in parts.items() if k not in ("total", "trace_m", "trace_first")))
        assert parts["trace_m"] + parts["trace_first"] == pytest.approx(parts["trace"])
        assert parts["fold"] == 16.0 * ct["samples"] + 32.0 * pixels
    # no records in the first pass: 64 B per sample (trace) and per first-segment hit (shade) fewer
    rec = bench.pipeline_bytes(ct, pixels, gen_trace=True)
    norec = bench.pipeline_bytes(ct, pixels, gen_trace=True, gen_norec=True)
    assert rec["trace"] - norec["trace"] == pytest.approx(64.0 * ct["samples"])
    assert rec["shade"] - norec["shade"] == pytest.approx(64.0 * ct["shaded_first"])


def test_hw_view_and_cpu_info():
    hw = bench.hw_view({"valu_issue_frac_of_peak": 0.5, "valu_lane_utilization": 0.8, "salu_per_valu": 0.3})
    assert hw["valu_lane_slots_busy"] == pytest.approx(0.4)
    info = bench.cpu_info()
    assert info["os_cpu_count"] >= 1 and info["affinity"] >= 1 and info["model"]
    assert 1 <= bench.default_cpu_threads() <= info["affinity"]
    assert bench.default_cpu_threads() == bench.usable_cpus(info)  # every usable CPU: pthreads, not OpenMP
    assert bench.usable_cpus(dict(info, affinity=256, quota=16.0)) == 16
    assert bench.usable_cpus(dict(info, affinity=8, quota=None)) == 8


def test_resolve_world():
    """--gpus N without a launcher starts N ranks; under a launcher it must
    agree with WORLD_SIZE (a silent 1-GPU run claimed N)."""
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(8, {}) == (8, True)
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "3"], 8, 29501)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-3:] == ["--gpus", "8", "--steps", "3"][-3:]


def test_gpus_mismatch_exits_before_the_gpu():
    """A launcher's WORLD_SIZE that disagrees with --gpus ends bench.py with a
    non-zero status before it imports the library or touches a GPU."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "8"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not any(l.startswith("{") for l in r.stdout.splitlines())


def test_executed_flops_drop_only_culled_work(counters):
    """roofline.frac's executed flops: each pass's algorithmic flops less its
    culled evaluations, each culled one still paying its test; without culls
    the two agree."""
    prog, ct, _ = counters
    st = dict(ct, wave_maps=0, wave_shapes=0)
    taps = _taps_share(ct)
    alg = (bench.trace_flops(st, taps, prog.n_aabb, True), bench.shade_flops(st, taps, prog.n_aabb))
    assert bench.executed_split(dict(st, culled=0), taps, prog.n_aabb, True) == pytest.approx(alg)
    st_c = dict(st, culled=st["xform_shape"] // 2)
    ex = bench.executed_split(st_c, taps, prog.n_aabb, True)
    assert ex[0] < alg[0] and ex[1] == pytest.approx(alg[1])
    per = bench.W_XFORM + bench.W_FINALISE + 1 - bench.W_CULL_TEST
    assert alg[0] - ex[0] >= st_c["culled"] * per  # (plus the mean SDF weight)


def _kernel_source(prog, data, baked: int) -> str:
    import ctypes

    from compute_path_tracer_amd import _native as N

    d = np.ascontiguousarray(data, np.float32)
    args = (prog.ops, prog.n_ops, prog.aabbs, prog.n_aabb, d.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(d),
            baked)
    n = ctypes.c_size_t()
    assert N.lib().pt_scene_kernel_source(*args, None, 0, ctypes.byref(n)) == N.PT_OK
    buf = ctypes.create_string_buffer(n.value)
    assert N.lib().pt_scene_kernel_source(*args, buf, n.value, ctypes.byref(n)) == N.PT_OK
    return buf.value.decode()


@pytest.mark.parametrize("scene", ["c1", "c2", "c3"])
def test_value_edit_leg_rebuilds_only_the_baked_kernel(scene):
    """bench.value_edit_leg's one-ulp edit: the table
    scene kernel's source is unchanged (no recompile: what an editing
    session renders meanwhile) and the values-baked source differs (its
    rebuild is what tier_up_s times -- a source no cache holds)."""
    from compute_path_tracer_amd import scenes
    from compute_path_tracer_amd.sdf_editor import CompData

    prog = scenes.SCENES[scene]().compile(CompData())
    for ulps in (1, 4095):
        k, edited = bench.edited_data(prog, ulps)
        assert k == bench.edit_slot(prog) and edited[k] > prog.data[k]
        assert np.count_nonzero(edited != prog.data) == 1
        assert _kernel_source(prog, prog.data, 0) == _kernel_source(prog, edited, 0)
        assert _kernel_source(prog, prog.data, 1) != _kernel_source(prog, edited, 1)
