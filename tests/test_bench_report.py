"""bench.py's JSON line on the CPU: report() driven by a stand-in context
with the oracle's counters of a small C3 frame, so the driver's contract
(metric, value, unit, n_gpus, ... roofline {bound, achieved, peak, unit,
frac, traffic}) and the round-4 roofline views are checked without a GPU."""
import json
import os
import sys

import numpy as np
import pytest

import bench
from compute_path_tracer_amd import scenes
from compute_path_tracer_amd._native import STAT_NAMES
from compute_path_tracer_amd.sdf_editor import CompData
from oracle import oracle as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


class _Ctx:
    """Answers pt.get_option like a binned two-pipeline scene-kernel run."""

    size = (48, 32)

    def get_option(self, key):
        return {"jit_active": 1, "gen_trace": 1, "gen_norec": 1, "shade_taps": 1, "bin_lanes": 2, "jit_tier_active": 1,
                "jit_trace_waves": 8, "jit_shade_waves": 8, "jit_cache": 1, "display_ms": 0.01}.get(key, 0.0)

    def display(self, srgb8=False):
        return np.zeros((32, 48, 4), np.uint8)


class _Args:
    steps, warmup, config, no_cpu_baseline, cpu_threads = 4, 1, "c3", True, 0


W, H, SPP = 48, 32, 2


@pytest.fixture(scope="module")
def frame():
    ed = scenes.c3_graph32()
    prog = ed.compile(CompData())
    _, ct = O.OracleScene(ed.rows()).render(W, H, O.Constants(0.0, 1, float(np.float32(W) / np.float32(H)), 1),
                                            O.Settings(0, 8, 1.0, 1.0, 0), SPP, counters=True)
    # the GPU stats run's keys (the oracle counts the algorithmic events; the
    # schedule counters are the wavefront's own): a quarter of shape
    # evaluations culled, half of them in the taps
    st = {k: 0 for k in STAT_NAMES}
    st.update(ct, culled=ct["xform_shape"] // 4, wave_maps=ct["march_steps"] // 64, wave_shapes=ct["xform_shape"] // 64,
              wave_evals=ct["xform_shape"] // 96)
    taps = {k: 0 for k in st}
    taps.update(normal_maps=st["normal_maps"], xform_shape=st["xform_shape"] // 4, culled=st["culled"] // 2,
                wave_maps=1, wave_shapes=1, wave_evals=1)
    return ed, prog, st, taps


def _report(frame):
    ed, prog, st, taps = frame
    solo = {"frames": 1, "st": st, "taps": taps, "dispatch_ms": 2.0, "trace_ms": 1.5, "trace_n": 9,
            "shade_ms": 0.5, "shade_n": 9}
    # timed steps: dispatch 3 ms, 18 trace launches in 2 ms, 18 shade launches in 1 ms
    out = bench.report(_Args, _Ctx(), st, taps, prog, "c3", W, H, 8, SPP, SPP, 1, "weak", 1.0, 3.0, [3.0],
                       [2.0], [18], [1.0], [18], 0.0, ed, None, solo)
    return json.loads(json.dumps(out))


@pytest.fixture(scope="module")
def line(frame):
    _, prog, st, taps = frame
    return _report(frame), st, taps, prog


def test_contract_fields(line):
    out = line[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["metric"] == bench.METRIC and out["n_gpus"] == 1 and out["dtype"] == "f32"
    r = out["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["peak"] == bench.PEAK_F32_TFLOPS and r["unit"] == "TFLOP/s"
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)


def test_roofline_views(line):
    out, st, taps, prog = line
    r = out["roofline"]
    ex_t, ex_s = bench.executed_split(st, taps, prog.n_aabb, True)
    # headline: executed trace flops over the solo run's trace time
    assert r["achieved"] == pytest.approx(ex_t / 1.5e-3 / 1e12, abs=5e-4)  # rounded to 3 places
    assert r["shade"]["achieved"] == pytest.approx(ex_s / 0.5e-3 / 1e12, abs=5e-4)
    assert r["solo_launches"] == 9 and r["timing"].startswith("one pipeline alone")
    # overlapped: the same executed flops over the timed steps' times; the sum is fracs_sum
    ov = r["overlapped"]
    assert ov["trace_frac"] == pytest.approx(ex_t / 2.0e-3 / 1e12 / bench.PEAK_F32_TFLOPS, abs=1e-4)
    assert r["fracs_sum"] == pytest.approx(ov["trace_frac"] + ov["shade_frac"], abs=2e-4)
    # reference-equivalent: algorithmic flops (>= executed) over the same times
    assert r["reference_equivalent_frac"] >= ov["trace_frac"]


def test_no_profile_no_traffic(line):
    """The test frame's workload has no committed PMC summary: traffic null."""
    r = line[0]["roofline"]
    assert r["traffic"] is None and r["traffic_source"] is None and "hw" not in r


def test_profiled_traffic_scaled_to_the_launch(frame, tmp_path, monkeypatch):
    """A one-pipeline PMC summary of the same workload supplies per-launch
    HBM bytes; a launch of this two-pipeline run carries half its frames."""
    out0 = _report(frame)
    cfg = {k: out0["config"][k] for k in ("width", "height", "bounces", "spp_per_step", "workload")}
    pmc = {"bench_config": dict(cfg, pipelines=1),
           "per_kernel": {"pt_bin_trace_m_jit": {"hbm_bytes_per_launch": 1000.0, "valu_issue_frac_of_peak": 0.8,
                                                 "valu_lane_utilization": 0.5},
                          "pt_bin_trace_g_jit": {"hbm_bytes_per_launch": 4000.0},
                          "pt_bin_shade_t_jit": {"hbm_bytes_per_launch": 600.0}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "zz_pmc.json").write_text(json.dumps(pmc))
    (tmp_path / "profiles" / "zz_l2_pmc.json").write_text(json.dumps(dict(pmc, bench_config=dict(cfg, pipelines=2))))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = _report(frame)["roofline"]
    _, _, st, _ = frame
    pipe = bench.pipeline_bytes(st, W * H, gen_trace=True, gen_norec=True)
    assert r["traffic_source"].startswith(os.path.join("profiles", "zz_pmc.json"))  # not the 2-pipeline one
    assert r["traffic"] == 500
    assert r["traffic_algorithmic"] == round(pipe["trace_m"] / 16)  # 18 trace launches less 2 first passes
    assert r["traffic_first_pass"] == {"kernel": "pt_bin_trace_g_jit", "measured": 2000,
                                       "algorithmic": round(pipe["trace_first"] / 2)}
    assert r["shade"]["traffic"] == 300
    assert r["hw"]["valu_lane_slots_busy"] == pytest.approx(0.4)


def test_march_traffic_halves_the_scattered_quad_writes(frame, tmp_path, monkeypatch):
    """The march pass's only stores are 16 B hit quads at scattered
    positions, which WRITE_SIZE counts twice (r04q_calib_traffic.json):
    roofline.traffic = FETCH_SIZE + WRITE_SIZE / 2, the raw sum kept beside
    it; and with two chunks per dispatch there are two first
    passes per pipeline."""
    out0 = _report(frame)
    cfg = {k: out0["config"][k] for k in ("width", "height", "bounces", "spp_per_step", "workload")}
    pmc = {"bench_config": dict(cfg, pipelines=1),
           "per_kernel": {"pt_bin_trace_m_jit": {"hbm_bytes_per_launch": 1400.0, "fetch_bytes_per_launch": 1000.0,
                                                 "write_bytes_per_launch": 400.0},
                          "pt_bin_trace_g_jit": {"hbm_bytes_per_launch": 4000.0}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "zz_pmc.json").write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    ed, prog, st, taps = frame
    solo = {"frames": 1, "st": st, "taps": taps, "dispatch_ms": 2.0, "trace_ms": 1.5, "trace_n": 9,
            "shade_ms": 0.5, "shade_n": 9}
    out = bench.report(_Args, _Ctx(), st, taps, prog, "c3", W, H, 8, SPP, SPP, 1, "weak", 1.0, 3.0, [3.0],
                       [2.0], [18], [1.0], [18], 0.0, ed, None, solo, [2])
    r = json.loads(json.dumps(out))["roofline"]
    assert r["traffic"] == 600 and r["traffic_uncorrected"] == 700  # (1000 + 200, 1400) x 1/2 pipelines
    assert "WRITE_SIZE / 2" in r["traffic_source"]
    pipe = bench.pipeline_bytes(st, W * H, gen_trace=True, gen_norec=True)
    assert r["traffic_algorithmic"] == round(pipe["trace_m"] / 14)  # 18 launches less 2 x 2 first passes
    assert r["traffic_first_pass"]["algorithmic"] == round(pipe["trace_first"] / 4)
    assert out["config"]["chunks_per_dispatch"] == 2.0


def test_launch_split(tmp_path):
    """summarize_profile.launch_split: the last n launches of each pass are
    bench.py's solo dispatch, the rest its timed steps."""
    import summarize_profile as S

    kt = tmp_path / "kt"
    kt.mkdir()
    rows = ["\"Kernel_Name\",\"Start_Timestamp\",\"End_Timestamp\""]
    t = 0
    for name, ns in ([("pt_bin_trace_g_jit", 3000), ("pt_bin_shade_t_jit", 1000)] * 3 +
                     [("pt_bin_trace_m_jit", 2000), ("pt_bin_shade_t_jit", 500)] * 2):
        rows.append(f"\"{name}\",{t},{t + ns}")
        t += ns + 10
    (kt / "kt_kernel_trace.csv").write_text("\n".join(rows) + "\n")
    ls = S.launch_split(str(tmp_path), 2)
    assert ls["trace_solo_ms"] == pytest.approx(2e-3)
    assert ls["shade_solo_ms"] == pytest.approx(0.5e-3)
    assert ls["trace_timed_ms"] == pytest.approx(3e-3)
    assert ls["shade_timed_ms"] == pytest.approx(1e-3)


def test_measured_view_pmc_and_calibration(frame, tmp_path, monkeypatch):
    """roofline.measured: the PMC FP32 flops of the
    solo trace launches (8 march launches + 1 first pass, per-launch figures
    of a one-pipeline profile halved for this two-pipeline run's launch size)
    over their time, the no-FMA ceiling, and the counted events at a
    calibration's executed weights (frac_executed_calibrated, by_event)."""
    out0 = _report(frame)
    cfg = {k: out0["config"][k] for k in ("width", "height", "bounces", "spp_per_step", "workload")}
    pmc = {"bench_config": dict(cfg, pipelines=1),
           "per_kernel": {"pt_bin_trace_m_jit": {"hbm_bytes_per_launch": 1.0, "fp32_flops_per_launch": 4.0e9,
                                                 "valu_issue_frac_of_peak": 0.8, "valu_lane_utilization": 0.7,
                                                 "fp32_insts_frac_of_valu": 0.5},
                          "pt_bin_trace_g_jit": {"hbm_bytes_per_launch": 1.0, "fp32_flops_per_launch": 6.0e9}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "zz_pmc.json").write_text(json.dumps(pmc))
    import flop_calib

    ev = {"march_steps": 3.0, "xform_union": 20.0, "shape_evals": 30.0, "culled": 5.0, "samples": 40.0}
    cal = {"configs": 24, "classes": {"trace": {"executed_flops_per_event": ev, "rms_rel_residual": 0.01,
                                                "survey_weights": {k: 1.0 for k in ev}},
                                      "shade": {"executed_flops_per_event": {}, "survey_weights": {}}}}
    (tmp_path / "profiles" / "zz_flop_calibration.json").write_text(json.dumps(cal))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = _report(frame)["roofline"]
    m = r["measured"]
    pmc_flops = 4.0e9 * 0.5 * 8 + 6.0e9 * 0.5 * 1
    assert m["fp32_tflops_pmc"] == pytest.approx(pmc_flops / 1.5e-3 / 1e12, abs=5e-4)
    assert m["no_fma_ceiling"] == pytest.approx(bench.PEAK_F32_TFLOPS / 2)
    assert m["fp32_frac_of_no_fma_ceiling"] == pytest.approx(2 * m["fp32_frac_pmc"], abs=2e-4)
    assert m["valu_lane_slots_busy"] == pytest.approx(0.56)
    _, prog, st, taps = frame
    x = flop_calib.features(st, taps, prog.n_aabb)["trace"]
    fl = sum(ev[k] * x[k] for k in ev)
    assert m["tflops_executed_calibrated"] == pytest.approx(fl / 1.5e-3 / 1e12, abs=5e-4)
    assert m["frac_executed_calibrated"] == pytest.approx(fl / 1.5e-3 / 1e12 / bench.PEAK_F32_TFLOPS, abs=1e-4)
    assert m["frac_survey_weights"] == r["frac"]
    assert set(m["by_event"]) == set(ev) and sum(v["executed_share"] for v in m["by_event"].values()) == \
        pytest.approx(1.0, abs=1e-3)
    assert m["calibration_source"].startswith(os.path.join("profiles", "zz_flop_calibration.json"))
