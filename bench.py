#!/usr/bin/env python3
"""Headline benchmark: Msamples/s of the SDF path-trace hot path.

Workload (BASELINE.json configs[2], the metric's "1920x1080x8-bounce"): the
32-node sdf_editor graph (scenes.c3_graph32), 1920x1080, 8 bounces, progressive
accumulation, 256 spp per render.  One *step* = one pt_dispatch of ``--spp``
(default 256: the whole C3 render) frames per pixel over this rank's tiles.
Inputs (scene tables, image) are resident in HBM before timing.

Multi-GPU (``torchrun --nproc-per-node N``): cyclic 8x8-tile ownership, each
rank renders its 1/N of the tiles for N*spp frames per step (weak scaling:
fixed samples per GPU), and the step ends with the RCCL sum-reduce of the
accumulation image onto rank 0 (bit-identical to a 1-GPU render).  At N > 1
the line also carries ``c4_strong``: BASELINE config 4 (3840x2160, 256 spp,
8 bounces, the same scene) split over the N GPUs (strong scaling: each rank
renders all 256 frames of its 1/N of the tiles), with the reduce timed on
its own.  ``--config c4`` makes that the headline (``scaling: strong``);
``--config c2|c5|c1`` bench the other single-GPU configs.

Prints ONE JSON line (rank 0).  See DESIGN.md 5 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec at 1920×1080×8-bounce; achieved HBM GB/s vs gfx950 peak"
PEAK_F32_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (vector); wave64 v_fma_f32 issues in 2 cycles on SIMD-32
PEAK_HBM_GBS = 8000.0  # spec

# Algorithmic flop weights per counted event; FMA = 2,
# sqrt/sin/cos excluded (counted as transcendentals).
W_XFORM = 54
W_SDF = {"sdf_sphere": 7, "sdf_cube": 19, "sdf_torus": 11, "sdf_octahedron": 22}
W_FINALISE = 1
W_COMB = {"comb_union": 1, "comb_sub": 3, "comb_assign": 0}
W_MARCH = 10
W_NORMAL = 29  # per calc_normal (6 maps counted separately)
W_AABB = 40
W_SHADE = 100
W_CAMERA = 25
W_ACCUM = 10
# Executed (not algorithmic) work of a shape evaluation the distance bound
# dropped: the test that dropped it -- the translate
# and scale of the transform's first steps (6), |t|^2 (5), the target's
# margin (3) and the compare (2) -- instead of its transform, SDF and combine.
W_CULL_TEST = 16


def shade_flops(st: dict, taps: dict, n_aabb: int) -> float:
    """The part of algorithmic_flops() done by the binned pipeline's shade
    passes: calc_normal's six taps when they run there (`taps`: the tap share
    of the stats run, PathTracer.tap_stats; zeros otherwise), the bounds() of
    every continuing ray (all slab tests but the primary rays' n_aabb per
    sample, which the gen pass or the first trace pass run) and shading +
    Russian roulette of every hit."""
    return (map_flops(taps) + W_NORMAL * (taps["normal_maps"] // 6)
            + W_AABB * (st["aabb_tests"] - st["samples"] * n_aabb) + W_SHADE * st["shaded"])


def trace_flops(st: dict, taps: dict, n_aabb: int, gen_trace: bool) -> float:
    """The part of algorithmic_flops() done by the binned pipeline's trace
    passes: the march (and calc_normal when its taps run there) -- all but
    the shade passes' share, the fold's accumulation and, unless the first
    trace pass makes its own camera rays (gen_trace), the gen pass's camera
    rays and primary bounds()."""
    gen = 0.0 if gen_trace else (W_CAMERA + W_AABB * n_aabb) * st["samples"]
    return algorithmic_flops(st) - shade_flops(st, taps, n_aabb) - W_ACCUM * st["samples"] - gen


def culled_flops(st: dict) -> float:
    """Algorithmic flops of st's culled shape evaluations that did not run:
    transform + finalise + SDF (the share's mean SDF weight: the counters do
    not split culls by kind) + combine (1), less the W_CULL_TEST flops of the
    test that dropped each one."""
    n, c = st.get("xform_shape", 0), st.get("culled", 0)
    if not n or not c:
        return 0.0
    sdf_mean = sum(w * st[k] for k, w in W_SDF.items()) / n
    return float(c) * (W_XFORM + W_FINALISE + sdf_mean + 1 - W_CULL_TEST)


def executed_split(st: dict, taps: dict, n_aabb: int, gen_trace: bool) -> tuple:
    """(trace, shade) flops that the kernels executed: each pass's
    algorithmic flops less its culled evaluations (culled_flops) -- the
    trace passes' culls are st's minus the taps' (PathTracer.tap_stats)."""
    trace_share = {k: v - taps.get(k, 0) for k, v in st.items()}
    return (trace_flops(st, taps, n_aabb, gen_trace) - culled_flops(trace_share),
            shade_flops(st, taps, n_aabb) - culled_flops(taps))


def map_flops(st: dict) -> float:
    """map() work: transforms, finalise, SDFs and combines."""
    xf = st["xform_union"] + st["xform_shape"]
    f = W_XFORM * xf + W_FINALISE * xf
    f += sum(w * st[k] for k, w in W_SDF.items())
    f += sum(w * st[k] for k, w in W_COMB.items())
    return float(f)


def algorithmic_flops(st: dict) -> float:
    f = map_flops(st)
    f += W_MARCH * st["march_steps"] + W_NORMAL * (st["normal_maps"] // 6) + W_AABB * st["aabb_tests"]
    f += W_SHADE * st["shaded"] + (W_CAMERA + W_ACCUM) * st["samples"]
    return float(f)


def pipeline_bytes(st: dict, pixels: float, gen_trace: bool = False, gen_norec: bool = False) -> dict:
    """Algorithmic HBM bytes of one dispatch of the binned pipeline
    (pt_binned.h), from the instrumented run's counters: S samples, G
    segments (rays entering a trace pass), H shaded hits.  Misses G - H end
    in the trace pass; G - S rays continue from a shade pass; H - (G - S)
    paths end there.  Rays are 64 B records (PtRay), hit quads 16 B.
    - gen writes each sample's ray and zeroes its colour slot (64 + 16 B)
      and lists it (4 B) -- or, gen_trace (the bench default), there is no
      gen pass: the first trace pass makes its rays and stores them at their
      slots (64 B), and each sample's colour slot is written once in pass 0
      (16 B: by the trace pass at a miss, by the shade pass at a hit);
    - scatter reads every later slot's 4 B key and writes a 4 B binned slot
      (the first pass takes generation order);
    - trace reads a slot (4 B) and its ray (64 B) (not in the first pass
      with gen_trace) and writes one 16 B hit quad per ray, hit or miss;
    - shade reads each traced ray's quad (16 B) and each hit's ray (64 B,
      gathered by slot) and writes the next ray + key (64 + 4 B) or a NONE
      key (4 B);
    - fold reads each frame's colour (16 B) and reads + writes the texel
      (32 B per pixel);
    - gen_norec (gen_trace with <= 32 check[] entries, the bench scene): the
      first pass stores no rays, and shade pass 0 makes its hits' camera rays
      again instead of gathering them (64 B less per sample in the trace
      pass and per first-segment hit, `shaded_first`, in the shade pass).
    Not counted: the colour slot's read-modify-write at emitting hits after
    the first (32 B each; no counter separates them) and the high mask words
    of scenes with > 64 check[] entries (the bench scene has 24)."""
    S, G, H = float(st["samples"]), float(st["segments"]), float(st["shaded"])
    cont, miss = G - S, G - H
    ended = H - cont
    traced_in = G - S if gen_trace else G
    parts = {"gen": 0.0 if gen_trace else 84.0 * S,
             "scatter": 8.0 * cont,
             "trace": 68.0 * traced_in + 16.0 * G + (64.0 * S if gen_trace and not gen_norec else 0.0),
             "shade": 16.0 * G + 64.0 * (H - (float(st["shaded_first"]) if gen_norec else 0.0)) + 68.0 * cont
             + 4.0 * (ended + miss),
             "fold": 16.0 * S + 32.0 * pixels}
    if gen_trace:
        parts["colour0"] = 16.0 * S
    parts["total"] = sum(parts.values())
    # per trace kernel: the march-only passes (bounces 1..) and the first pass
    parts["trace_m"] = (68.0 + 16.0) * (G - S)
    parts["trace_first"] = parts["trace"] - parts["trace_m"]
    return parts


def schedule_metrics(st_all: dict, taps: dict) -> dict:
    """SIMD efficiency of the wavefront schedule from the instrumented run:
    the trace passes (st_all minus the shade pass's normal taps), and the
    taps' own wave-level shape evaluations."""
    st = {k: v - taps.get(k, 0) for k, v in st_all.items()}
    maps = st["march_steps"] + st["normal_maps"]
    out = {}
    if taps.get("normal_maps"):
        out["shade_taps"] = {"lane_shapes_per_map": round(taps["xform_shape"] / taps["normal_maps"], 3),
                             "lane_evals_per_map": round((taps["xform_shape"] - taps["culled"]) / taps["normal_maps"], 3),
                             "wave_shapes_per_map": round(taps["wave_shapes"] / max(1, taps["wave_maps"]), 3),
                             "wave_evals_per_map": round(taps["wave_evals"] / max(1, taps["wave_maps"]), 3)}
    if st.get("wave_maps"):  # wave-level map() evaluations of the trace passes (per-map instruction budgets)
        out["trace_wave_maps"] = st["wave_maps"]
    if st.get("wave_shapes"):
        out["map_lane_util"] = round(st["xform_shape"] / (64.0 * st["wave_shapes"]), 4)
        out["wave_shapes_per_map"] = round(st["wave_shapes"] / max(1, st["wave_maps"]), 3)
        out["lane_shapes_per_map"] = round(st["xform_shape"] / max(1, maps), 3)
    if st.get("wave_iters"):
        out["lane_busy"] = round(1.0 - st["lane_idle"] / (64.0 * st["wave_iters"]), 4)
        out["idle_shade"] = round(st["idle_shade"] / (64.0 * st["wave_iters"]), 4)
        out["idle_free"] = round(st["idle_free"] / (64.0 * st["wave_iters"]), 4)
        out["maps_per_sample"] = round(maps / max(1, st["samples"]), 2)
    if st_all.get("bounds_waves"):  # bounds()' waves that redid every box exactly (an undecided lane)
        out["bounds_exact_waves"] = round(st_all.get("bounds_exact", 0) / st_all["bounds_waves"], 5)
    if st.get("cyc_total"):  # share of wave time per phase (instrumented kernel)
        out["wave_time"] = {k: round(st["cyc_" + k] / st["cyc_total"], 4)
                            for k in ("refill", "bounds", "map", "shade")}
        out["wave_cycles_per_iter"] = round(st["cyc_total"] / max(1, st["wave_iters"]), 1)
    return out


def profiled(config: dict):
    """The newest committed rocprofv3 PMC summary (profiles/*_pmc.json,
    scripts/summarize_profile.py) of this same workload with per-kernel
    figures, taken with ONE pipeline (bench.py --pipelines 1: each kernel's
    counters are its own, as roofline.frac's times are), as (summary, path);
    None if there is none."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        cfg = d.get("bench_config") or {}
        keys = ("width", "height", "bounces", "spp_per_step", "workload")
        if all(cfg.get(k) == config.get(k) for k in keys) and cfg.get("pipelines") == 1 and d.get("per_kernel"):
            best = (d, os.path.relpath(f, ROOT))
    return best


PEAK_F32_NO_FMA_TFLOPS = PEAK_F32_TFLOPS / 2.0  # one flop per lane-op: the ceiling without FMA contraction


def flop_calibration():
    """The newest committed executed-flop calibration
    (profiles/*_flop_calibration.json, scripts/flop_calib.py: FP32 flops
    per counted event fitted to PMC instruction counts over scenes x
    bounces) as (calibration, path); None if there is none."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_flop_calibration.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("classes"):
            best = (d, os.path.relpath(f, ROOT))
    return best


def calibrated_flops(cal: dict, cls: str, st: dict, taps: dict, n_aabb: int) -> tuple:
    """(executed flops, {event: (count, executed flops, SURVEY-weight
    flops)}) of one kernel class over a dispatch's counters, at the
    calibration's fitted weights."""
    sdir = os.path.join(ROOT, "scripts")
    if sdir not in sys.path:
        sys.path.insert(0, sdir)
    from flop_calib import features

    c = cal["classes"][cls]
    x = features(st, taps, n_aabb)[cls]
    by = {k: (x[k], x[k] * w, x[k] * c["survey_weights"][k]) for k, w in c["executed_flops_per_event"].items()}
    return float(sum(v[1] for v in by.values())), by


def measured_view(pmc_flops, pk: dict, src: str, time_ms: float, cal, cls: str, st: dict, taps: dict, n_aabb: int,
                  survey_frac: float) -> dict:
    """roofline.measured: what the hardware did in the dominant kernel class
    (VERDICT r05 item 3), over the same solo launches as roofline.frac
    (time_ms: their summed HIP-event time).  pmc_flops: the FP32 flops of
    those launches by the kernels' own instruction counts in the
    one-pipeline PMC profile (add / mul 1, fma 2 per lane, at each kernel's
    lane utilisation; scaled to this run's launch size); pk: the dominant
    kernel's derived counters there (VALU issue, lane utilisation, lane-slots
    busy).  The contract leaves almost no FMAs (no contraction),
    so a lane-op carries <= 1 flop: half the FP32 peak, 78.65 TFLOP/s, is
    the no-FMA ceiling.  From the calibration (cal): the counted events at
    their fitted executed weights over the same time --
    frac_executed_calibrated, the SURVEY-weight frac (survey_frac)
    reconciled with the PMC instruction classes -- and the per-event split."""
    out = {"peak": PEAK_F32_TFLOPS, "no_fma_ceiling": PEAK_F32_NO_FMA_TFLOPS, "unit": "TFLOP/s",
           "kernel_class": cls, "frac_survey_weights": survey_frac}
    if pmc_flops and time_ms:
        tf = pmc_flops / (time_ms * 1e-3) / 1e12
        out.update({"fp32_tflops_pmc": round(tf, 3), "fp32_frac_pmc": round(tf / PEAK_F32_TFLOPS, 4),
                    "fp32_frac_of_no_fma_ceiling": round(tf / PEAK_F32_NO_FMA_TFLOPS, 4)})
    if pk:
        hv = hw_view(pk)
        for k in ("valu_issue_frac_of_peak", "valu_lane_utilization", "valu_lane_slots_busy", "wave_time_waitcnt"):
            if k in hv:
                out[k] = hv[k]
        if pk.get("fp32_insts_frac_of_valu") is not None:
            out["fp32_insts_frac_of_valu"] = round(pk["fp32_insts_frac_of_valu"], 4)
        out["pmc_source"] = f"{src} (one pipeline, per launch, scaled to this run's launch size; time: this run's solo launches)"
    if cal is not None and time_ms:
        c, csrc = cal
        fl, by = calibrated_flops(c, cls, st, taps, n_aabb)
        tf = fl / (time_ms * 1e-3) / 1e12
        cc = c["classes"][cls]
        out.update({"tflops_executed_calibrated": round(tf, 3), "frac_executed_calibrated": round(tf / PEAK_F32_TFLOPS, 4),
                    "calibration_source": f"{csrc} (scripts/flop_calib.py: NNLS of PMC FP32 flops on the counted "
                                          f"events over {c.get('configs')} scene x bounce configurations; rms relative "
                                          f"residual {cc.get('rms_rel_residual')})",
                    "by_event": {k: {"count": int(v[0]), "executed_flops_per_event": cc["executed_flops_per_event"][k],
                                     "survey_flops_per_event": cc["survey_weights"][k],
                                     "executed_share": round(v[1] / fl, 4) if fl else None}
                                 for k, v in by.items()}})
        if out.get("fp32_tflops_pmc"):
            out["calibrated_over_pmc"] = round(tf / out["fp32_tflops_pmc"], 4)
    return out


def hw_view(derived: dict) -> dict:
    """The hardware counters' view of a kernel beside its algorithmic frac:
    VALU issue (fraction of the wave64 issue rate) x lane utilisation = the
    fraction of FP32 lane-slots that did work."""
    keys = ("valu_issue_frac_of_peak", "valu_lane_utilization", "salu_per_valu", "wave_time_waitcnt",
            "wave_time_wait_issue")
    out = {k: round(derived[k], 4) for k in keys if k in derived}
    if "valu_issue_frac_of_peak" in out and "valu_lane_utilization" in out:
        out["valu_lane_slots_busy"] = round(derived["valu_issue_frac_of_peak"] * derived["valu_lane_utilization"], 4)
    if derived.get("fp32_tflops_measured"):
        # the FP32 flops the kernel executed by its own instruction counts
        # (add/mul 1, fma 2, at its lane utilisation) over its time
        out["fp32_tflops_measured"] = round(derived["fp32_tflops_measured"], 3)
        out["fp32_frac_measured"] = round(derived["fp32_tflops_measured"] / PEAK_F32_TFLOPS, 4)
    return out


def cpu_quota():
    """CPUs' worth of time the cgroup lets this process use (cpu.max), or
    None when unlimited / not readable."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_info() -> dict:
    """Host CPU of this box: model, logical CPUs, the CPUs this process may
    run on (affinity) and the cgroup's CPU quota."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"model": model, "os_cpu_count": os.cpu_count(), "affinity": affinity, "quota": cpu_quota()}


def cpu_baseline(scene, w, h, bounces, threads: int, row_stride: int, spp, target_s: float = 12.0) -> dict:
    """The C oracle (test infrastructure: the CPU restatement of the
    reference's per-pixel loop, pthreads) on `threads` host threads, over
    every row_stride-th row of the same frame.  spp None: chosen from a
    1-spp calibration run so the timed run takes about target_s seconds."""
    import tempfile

    from oracle import oracle as O  # test infrastructure: the CPU restatement

    info = cpu_info()
    build = "oracle/pt_oracle.c, gcc -O3 -march=native -ffp-contract=off"
    try:  # compiled for this host (the shipped .so targets x86-64-v3)
        O.use_library(O.build_native(tempfile.mkdtemp(prefix="pt_oracle_")))
    except (OSError, RuntimeError, Exception) as e:  # noqa: BLE001 - report, keep the shipped build
        build = f"oracle/libpt_oracle.so (x86-64-v3; native build failed: {type(e).__name__})"
    osc = O.OracleScene(scene.rows())
    c = O.Constants(0.0, 1, float(np.float32(w) / np.float32(h)), 1)
    s = O.Settings(0, bounces, 1.0, 1.0, 0)
    rows = len(range(0, h, row_stride))
    t0 = time.perf_counter()
    osc.render(w, h, c, s, 1, row_stride=row_stride, threads=threads)  # warm caches + calibration
    cal = time.perf_counter() - t0
    if spp is None:
        spp = int(max(1, min(64, round(target_s / max(cal, 1e-3)))))
    t0 = time.perf_counter()
    osc.render(w, h, c, s, spp, row_stride=row_stride, threads=threads)
    dt = time.perf_counter() - t0
    samples = rows * w * spp
    quota = info["quota"]
    return {"value": samples / dt / 1e6, "unit": "Msamples/sec", "cores": threads, "kind": "port",
            "cpu_model": info["model"], "os_cpu_count": info["os_cpu_count"], "cpus_available": usable_cpus(info),
            "cpu_affinity": info["affinity"], "cgroup_cpu_quota": quota,
            "sample": f"C oracle ({build}, pthreads: {threads} threads; this process may use {usable_cpus(info)} "
                      f"CPUs at once: affinity mask {info['affinity']}"
                      f"{'' if quota is None else f', cgroup quota {quota} CPUs of time'}) on every "
                      f"{row_stride}th row of the same {w}x{h} {bounces}-bounce frame, {spp} spp ({samples} "
                      f"samples, {dt:.1f} s; spp set by a {cal:.1f} s 1-spp calibration run)"}


def usable_cpus(info: dict) -> int:
    """The CPUs this process can actually run on at once: its affinity mask,
    capped by the cgroup's CPU quota (cpu.max) where one is set -- more
    threads than the quota only time-share it (measured on the GPU box: 256
    threads under a 16-CPU quota ran 0.47 Msamples/s, 16 threads ~0.78)."""
    n = info["affinity"]
    if info.get("quota"):
        n = min(n, max(1, int(info["quota"])))
    return max(1, n)


def default_cpu_threads() -> int:
    """One pthread per usable CPU (usable_cpus): the oracle runs pthreads,
    so OMP_NUM_THREADS does not apply."""
    return usable_cpus(cpu_info())


def solo_pipeline(pt, aspect: float, frames_step: int) -> dict:
    """Per-kernel times for the roofline (outside the timed region): one
    dispatch of ONE pipeline's share of a chunk (ceil(frames per chunk /
    pipelines) frames, so the chunk buffers fit as they are) with bin_lanes 1.  Its trace
    and shade passes then run alone, so each launch's HIP-event time is the
    kernel's own -- in the timed steps the two pipelines' kernels share the
    GPU and their event times overlap.  The instrumented twin of the same
    frames gives their exact counters."""
    from compute_path_tracer_amd import _native as N

    lanes = int(pt.get_option("bin_lanes"))
    w, h = pt.size
    n_pix = -(-w // 8) * -(-h // 8) * 64  # (one rank: every 8x8 tile)
    chunk = max(1, min(frames_step, int(pt.get_option("bin_samples")) // n_pix))  # frames per chunk
    frames = -(-chunk // lanes)  # one pipeline's share of a chunk: the buffers fit as they are
    c = N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1)
    kernel = int(pt.get_option("kernel"))
    pt.set_option("bin_lanes", 1)
    # the binned passes even when one pipeline's share is small enough for
    # the automatic choice to take the tile-resident kernel
    pt.set_option("kernel", "binned")
    try:
        st = pt.stats(c, frames)
        taps = pt.tap_stats()
        pt.dispatch(c, frames)
        pt.sync()
        return {"frames": frames, "st": st, "taps": taps, "dispatch_ms": pt.last_dispatch_ms(),
                "trace_ms": pt.get_option("trace_ms"), "trace_n": int(pt.get_option("trace_launches")),
                "shade_ms": pt.get_option("shade_ms"), "shade_n": int(pt.get_option("shade_launches"))}
    finally:
        pt.set_option("bin_lanes", lanes)
        pt.set_option("kernel", kernel)


def table_kernel_leg(pt, prog, aspect: float, frames: int, steps: int = 2) -> dict:
    """Throughput of the table scene kernel (outside the timed region).  The
    headline runs the values-baked build (jit_bake 2's tier-up, installed in
    setup by jit_wait).  A value edit (DataArray::update, primitives.rs:
    131-151: a buffer refresh, no recompile) drops that build, and an editing
    session renders on the table kernel -- node values read from the table --
    until the rebuild for the new values lands.  This times that kernel on
    the same workload: jit_bake 0 + the same values, one warm-up and `steps`
    dispatches of `frames` frames, wall time around each; then the baked
    build is restored."""
    from compute_path_tracer_amd import _native as N

    w, h = pt.size
    c = N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1)
    pt.set_option("jit_bake", 0)
    pt.set_data(prog.data)
    try:
        if pt.get_option("jit_tier_active") or not pt.get_option("jit_active"):
            return None  # (not the table kernel: nothing to report)
        pt.dispatch(c, frames)
        pt.sync()
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            pt.dispatch(c, frames)
            pt.sync()
            ts.append(time.perf_counter() - t0)
        dt = float(np.mean(ts))
        return {"value": round(w * h * frames / dt / 1e6, 3), "unit": "Msamples/sec",
                "ms_per_step": round(dt * 1e3, 3), "steps": steps,
                "kernel": "table scene kernel (jit_bake 0: node values read from the table; what renders between "
                          "a value edit and its values-baked rebuild)"}
    finally:
        pt.set_option("jit_bake", 2)
        pt.set_data(prog.data)
        pt.set_option("jit_wait", 1)


def edit_slot(prog) -> int:
    """The data[] slot value_edit_leg nudges: the first shape's size -- a
    value the generated map() uses (so the values-baked source changes) and
    no identity flag depends on (those are scale 1, zero position and zero
    rotation axis: pt_jit.cpp), so the table kernel's source stays the same
    and only the values-baked build is rebuilt."""
    for o in prog.op_dicts():
        if o["opcode"] == 1 and np.isfinite(float(prog.data[o["size"][0]])):  # PT_OP_SHAPE
            return int(o["size"][0])
    raise ValueError("no shape")


def edited_data(prog, ulps: int) -> tuple:
    """(slot, data[]) with the edit_slot value moved `ulps` steps up the
    float grid (away from zero)."""
    k = edit_slot(prog)
    edited = np.ascontiguousarray(prog.data, dtype=np.float32).copy()
    edited[k:k + 1] = (edited[k:k + 1].view(np.int32) + np.int32(ulps)).view(np.float32)
    return k, edited


def value_edit_leg(pt, prog) -> dict:
    """What one value edit costs an editing session (outside the timed
    region).  The reference's edit is a buffer refresh
    (DataArray::update, primitives.rs:131-151; sdf_editor.rs:248-252): here
    pt_set_data uploads the table at once, the table scene kernel renders
    from the next dispatch on (table_kernel's throughput), and the
    values-baked build for the new values compiles on a worker thread
    (hipRTC; the edited values' source is in no cache) and replaces it when
    it lands.  One Float (edit_slot) is nudged by a few ulps; tier_up_s is the
    wall time from pt_set_data until that build is installed (jit_wait),
    tier_compile_s the compile's own seconds.  Then the original values are
    restored (their baked build comes from the shipped cache)."""
    data = np.ascontiguousarray(prog.data, dtype=np.float32)
    # a different small edit every run (1..4095 ulps): hipRTC / comgr keep a
    # compile cache of their own, and an earlier run on the same box (the GPU
    # tests run this leg too) must not have compiled the edited source
    ulps = int(np.random.default_rng(time.time_ns() ^ os.getpid()).integers(1, 4096))
    k, edited = edited_data(prog, ulps)
    pt.set_option("jit_bake", 2)
    t0 = time.perf_counter()
    pt.set_data(edited)
    t1 = time.perf_counter()
    on_table = bool(pt.get_option("jit_active")) and not pt.get_option("jit_tier_active")
    pt.set_option("jit_wait", 1)
    t2 = time.perf_counter()
    out = {"tier_up_s": round(t2 - t0, 3), "tier_compile_s": round(pt.get_option("jit_tier_seconds"), 3),
           "set_data_s": round(t1 - t0, 4), "table_kernel_meanwhile": on_table,
           "tier_active_after": bool(pt.get_option("jit_tier_active")), "edited_slot": k, "edit_ulps": ulps,
           "edit": "a shape size (data[edited_slot]) nudged by edit_ulps ulps, a different edit every run (no "
                   "compile cache has seen it); no identity flag flips, so the table kernel is not rebuilt; the "
                   "values-baked build is"}
    pt.set_data(data)
    pt.set_option("jit_wait", 1)
    return out


def max_over_ranks(dist, v: float, device: str, op: str = "MAX") -> float:
    if dist is None:
        return v
    import torch

    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
    return float(t.item())


def check_tiles_spec(n_tiles: int, world: int, k: int = 8, seed: int = 0) -> tuple:
    """(r, M): the 8x8 tiles t with t % M == r that rank 0 re-renders to
    check the assembled image -- about k of them, spread over the image.  M
    is the largest modulus <= n_tiles // k with M % world == 1, so the k
    tiles r, r + M, ... belong to k consecutive ranks (tile t is rank
    t % world's, distributed.py): a cyclic split over up to k GPUs has every
    rank's share checked."""
    m0 = max(1, n_tiles // max(1, k))
    m = m0 - (m0 - 1) % max(1, world)
    if m < 1:
        m = 1
    r = int(np.random.default_rng(seed).integers(0, m))
    return r, m


def tile_ids(width: int, height: int) -> np.ndarray:
    """Global 8x8 tile id of every texel, [height][width] (pt_binned.h
    pixel_of: tile g covers x in [(g % tiles_x) * 8, +8), y in [(g // tiles_x)
    * 8, +8), tiles_x = ceil(width / 8))."""
    tiles_x = -(-width // 8)
    y, x = np.mgrid[0:height, 0:width]
    return (y // 8) * tiles_x + (x // 8)


def compare_tiles(img: np.ndarray, ref: np.ndarray, r: int, m: int) -> dict:
    """Bit-for-bit comparison of the assembled image with a render of the
    tiles t % m == r alone (ref: zero outside them, pt_set_tiles): every
    texel of those tiles, all four channels, as bit patterns (NaN texels
    included)."""
    h, w = img.shape[:2]
    ids = tile_ids(w, h)
    sel = ids % m == r
    a = img.view(np.uint32)[sel]
    b = ref.view(np.uint32)[sel]
    bad = int(np.count_nonzero((a != b).any(axis=-1)))
    outside_zero = bool(not np.any(ref.view(np.uint32)[~sel]))
    tiles = sorted(int(t) for t in np.unique(ids[sel]))
    return {"tiles": tiles, "texels": int(np.count_nonzero(sel)), "mismatched_texels": bad,
            "ref_zero_outside": outside_zero, "bit_exact": bad == 0 and outside_zero and bool(np.any(sel))}


def special_tiles(img: np.ndarray, limit: int = 16) -> list:
    """The 8x8 tiles of an image holding a texel that a sum-reduce could
    alter: a non-finite channel (a NaN payload, an infinity: C3 and C5 hold
    NaN texels from the reference's normalize of a zero vector)
    or a negative zero (-0 + +0 is +0), at most `limit` of them, in tile
    order (as test_gpu_parity.py's full-size check picks them)."""
    h, w = img.shape[:2]
    bits = img.view(np.uint32)
    odd = (~np.isfinite(img)).any(axis=-1) | (bits == 0x80000000).any(axis=-1)
    return sorted({int(t) for t in np.unique(tile_ids(w, h)[odd])})[:limit]


def compare_one_tile(img: np.ndarray, ref: np.ndarray, t: int) -> dict:
    """Bit-for-bit comparison of tile t of the assembled image with a render
    of tile t alone (ref: zero outside it)."""
    h, w = img.shape[:2]
    ids = tile_ids(w, h)
    sel = ids == t
    bad = int(np.count_nonzero((img.view(np.uint32)[sel] != ref.view(np.uint32)[sel]).any(axis=-1)))
    return {"tile": t, "texels": int(np.count_nonzero(sel)), "mismatched_texels": bad,
            "ref_zero_outside": bool(not np.any(ref.view(np.uint32)[~sel]))}


def validate_tiles(img: np.ndarray, prog, settings, width: int, height: int, device: int, frames: int,
                   world: int, seed: int, special_limit: int = 16) -> dict:
    """Rank 0's check of the assembled (reduced) image after the timed steps:
    a fresh context renders ~8 tiles of the image -- pt_set_tiles(r, M), see
    check_tiles_spec -- over every frame the run accumulated (frame 1 ..
    frames, as TileSplitRender counts them, path_tracer.rs:110-111), and the
    texels must equal the image's bit for bit (the texel of
    test_compute.glsl:242-245 that the reduce's sum must preserve).  Then
    every tile the image holds a non-finite or negative-zero texel in
    (special_tiles, at most 16) is rendered alone and checked the same way:
    the texels most likely to change in a reduce.  Cost: ~(8 + 16) x 64
    pixels x frames samples."""
    from compute_path_tracer_amd import _native as N
    from compute_path_tracer_amd.path_tracer import PathTracer

    n_tiles = -(-width // 8) * -(-height // 8)
    r, m = check_tiles_spec(n_tiles, world, seed=seed)
    special = special_tiles(img, special_limit)
    t0 = time.perf_counter()
    c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(width) / np.float32(height)), last_clear=1)
    ref = PathTracer(width, height, prog, device=device, settings=settings)
    extra = []
    try:
        # the binned passes whatever the sample count (the automatic choice
        # would give a one-rank run's ~4 M samples to the tile-resident
        # kernel, whose ~9 waves would take seconds)
        ref.set_option("kernel", "binned")
        ref.set_tiles(r, m)
        ref.dispatch(c, frames)
        want = ref.read_image()
        for t in special:  # each alone (tile t is the only one with t % n_tiles == t; set_tiles clears)
            ref.set_tiles(t, n_tiles)
            ref.dispatch(c, frames)
            extra.append(compare_one_tile(img, ref.read_image(), t))
    finally:
        ref.close()
    out = compare_tiles(img, want, r, m)
    ok = out["bit_exact"] and all(e["mismatched_texels"] == 0 and e["ref_zero_outside"] for e in extra)
    out.update({"frames": frames, "modulus": m, "residue": r,
                "owner_ranks": sorted({t % world for t in out["tiles"]}),
                "special_tiles": [e["tile"] for e in extra],
                "special_owner_ranks": sorted({e["tile"] % world for e in extra}),
                "special_texels": sum(e["texels"] for e in extra),
                "mismatched_texels": out["mismatched_texels"] + sum(e["mismatched_texels"] for e in extra),
                "bit_exact": bool(ok),
                "check_s": round(time.perf_counter() - t0, 3)})
    return out


def validation_failures(out: dict) -> list:
    """Why an N-GPU line must not be trusted (bench.py exits non-zero):
    RCCL's communicator does not hold n_gpus ranks, or rank 0's tile check
    (validate_tiles) or the full re-render (--validate) found a texel that
    differs -- for the headline and for the c4_strong leg alike."""
    bad = []
    for name, o in (("headline", out), ("c4_strong", out.get("c4_strong"))):
        if not o:
            continue
        n = o.get("n_gpus", 1)
        if n > 1 and o.get("reduce_backend") == "rccl" and o.get("rccl_ranks") != n:
            bad.append(f"{name}: RCCL communicator has {o.get('rccl_ranks')} ranks, n_gpus is {n}")
        for key in ("tile_check", "validation"):
            v = o.get(key)
            if v is not None and not v.get("bit_exact"):
                bad.append(f"{name}: {key} not bit-exact ({v.get('mismatched_texels', '?')} texels differ)")
    return bad


def rank_render_ms(dist, ms: float, device: str) -> dict:
    """One dispatch's device time (HIP events on the rank's stream) over the
    ranks: min / max and their ratio -- the cyclic tile split's load balance
    (distributed.py)."""
    lo = max_over_ranks(dist, ms, device, "MIN")
    hi = max_over_ranks(dist, ms, device, "MAX")
    return {"min": round(lo, 3), "max": round(hi, 3), "max_over_min": round(hi / lo, 4) if lo > 0 else None}


def reduce_probe(tr, pt, barrier, dist, device: str, reps: int = 3) -> float:
    """ms of one image reduce alone (after the render), max over ranks,
    median of `reps`."""
    if tr.world == 1:
        return 0.0
    ts = []
    for _ in range(reps):
        pt.sync()
        barrier()
        t0 = time.perf_counter()
        tr.reduce(0)
        pt.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    return max_over_ranks(dist, float(np.median(ts)), device)


def strong_leg(local_rank, rank, world, mode, barrier, dist, device, steps: int, warmup: int) -> dict:
    """BASELINE config 4 (3840x2160, 256 spp, 8 bounces, the 32-node scene)
    split over the ranks' tiles: each step renders the whole image's 256
    frames once (every rank all 256 frames of its 1/N of the tiles) and
    reduces it onto rank 0."""
    from compute_path_tracer_amd import _native as N
    from compute_path_tracer_amd import scenes
    from compute_path_tracer_amd.distributed import TileSplitRender
    from compute_path_tracer_amd.path_tracer import PathTracer
    from compute_path_tracer_amd.sdf_editor import CompData

    scene, w, h, spp, bounces = scenes.CONFIGS["c4"]
    prog = scenes.SCENES[scene]().compile(CompData())
    settings = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(w, h, prog, device=local_rank, settings=settings)
    pt.set_option("jit_wait", 1)
    tr = TileSplitRender(pt, rank, world, float(np.float32(w) / np.float32(h)), reduce=mode, scaling="strong")
    rccl_ranks = pt.comm_size() if world > 1 and mode == "rccl" else None
    for _ in range(warmup):
        tr.step(spp)
        tr.reduce(0)
    pt.sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(spp)
        tr.reduce(0)
    pt.sync()
    barrier()
    dt = max_over_ranks(dist, time.perf_counter() - t0, device)
    render = rank_render_ms(dist, pt.last_dispatch_ms(), device)  # the last step's render on each rank's stream
    red = reduce_probe(tr, pt, barrier, dist, device)
    img = tr.image(0)  # (every rank takes part in the reduce)
    check = validate_tiles(img, prog, settings, w, h, local_rank, tr.frame - 1, world, seed=4) if rank == 0 else None
    pt.close()
    return {"metric": "Msamples/sec, BASELINE config 4 split over the GPUs",
            "value": round(w * h * spp * steps / dt / 1e6, 3), "unit": "Msamples/sec", "scaling": "strong",
            "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": round(dt * 1e3 / steps, 3),
            "render_ms_max_rank": render["max"], "render_ms_per_rank": render, "reduce_ms": round(red, 3),
            "rccl_ranks": rccl_ranks, "reduce_backend": mode, "tile_check": check,
            "config": {"workload": f"c3 {w}x{h}, {bounces} bounces, {spp} spp per step over all GPUs",
                       "width": w, "height": h, "bounces": bounces, "spp_per_step": spp,
                       "parallelism": f"tiles{world}", "reduce": "RCCL ncclReduce(sum) onto rank 0"
                       if mode == "rccl" else "host sum over torch.distributed (gloo)"}}


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_cmd(argv: list, n: int, port: int) -> list:
    """The torch.distributed.run command that runs this script as n ranks
    (one process per GPU) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def resolve_world(gpus, env=os.environ):
    """(world, launch): the rank count this run is for, and whether this
    process must first start that many ranks itself.
    - a launcher set WORLD_SIZE: it must equal --gpus when given (SystemExit
      otherwise: the line would claim the wrong n_gpus);
    - no launcher and --gpus N > 1: launch N ranks (bench.py starts them);
    - otherwise one rank."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {n}")
    return n, n > 1


def main() -> None:
    from compute_path_tracer_amd import scenes as _scenes

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks, one process each).  Without a launcher, N > 1 starts N ranks through "
                         "torch.distributed.run; under one it must equal WORLD_SIZE.  Default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(_scenes.CONFIGS),
                    help="BASELINE config: c3 (the metric's, default), c4 (2160p split over the GPUs: strong "
                         "scaling), c2, c5, c1")
    ap.add_argument("--spp", type=int, default=None,
                    help="frames per pixel per step (per GPU-share when weak); default the config's "
                         "(c3: 256 = one step is the whole render)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--bounces", type=int, default=None)
    ap.add_argument("--scene", default=None)
    ap.add_argument("--pipelines", type=int, default=None,
                    help="binned pipelines per chunk (pt_set_option bin_lanes; default the library's 2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this process may use")
    ap.add_argument("--cpu-row-stride", type=int, default=1)
    ap.add_argument("--cpu-spp", type=int, default=None,
                    help="CPU baseline spp (default: sized to ~12 s by a 1-spp calibration run)")
    ap.add_argument("--c4-steps", type=int, default=2,
                    help="N > 1: steps of the config-4 strong-scaling leg (0 skips it)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + host image reduce: rehearsal with ranks sharing one GPU")
    ap.add_argument("--validate", action="store_true",
                    help="rank 0 re-renders every frame on one GPU and checks the assembled image bit for bit")
    ap.add_argument("--no-tile-check", action="store_true",
                    help="skip rank 0's default check of ~8 tiles of the assembled image against a fresh render")
    ap.add_argument("--no-table-kernel", action="store_true",
                    help="skip the one-GPU timing of the table scene kernel (jit_bake 0: what a value-editing "
                         "session runs)")
    args = ap.parse_args()
    world, launch = resolve_world(args.gpus)
    if launch:
        # N ranks from one command line: torch.distributed.run as a child
        # process, started before anything here touches the GPU (no exec);
        # rank 0 prints the line on the shared stdout
        import subprocess

        rc = subprocess.run(launcher_cmd(sys.argv[1:], world, free_port()), cwd=ROOT).returncode
        sys.exit(rc)
    cscene, cw, ch, cspp, cb = _scenes.CONFIGS[args.config]
    scene_name = args.scene or cscene
    width, height = args.width or cw, args.height or ch
    bounces = cb if args.bounces is None else args.bounces
    spp = args.spp or cspp
    scaling = "strong" if args.config == "c4" else "weak"

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PT_BENCH_SHARE_GPU"):  # test aid: all ranks on GPU 0 (single-GPU boxes)
        local_rank = 0
    dist = None
    dev = "cpu"
    if world > 1:
        import torch
        import torch.distributed as dist_

        dist = dist_
        torch.cuda.set_device(local_rank)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            dev = "cuda"
        else:
            dist.init_process_group("gloo")

    from compute_path_tracer_amd import _native as N
    from compute_path_tracer_amd import scenes
    from compute_path_tracer_amd.path_tracer import PathTracer
    from compute_path_tracer_amd.sdf_editor import CompData

    from compute_path_tracer_amd.distributed import TileSplitRender

    ed = scenes.SCENES[scene_name]()
    prog = ed.compile(CompData())
    settings = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(width, height, prog, device=local_rank, settings=settings)
    if args.pipelines is not None:
        pt.set_option("bin_lanes", args.pipelines)
    # setup, untimed: install the values-baked scene kernel (jit_bake 2 tier-up;
    # an interactive caller keeps rendering on the table kernel meanwhile)
    pt.set_option("jit_wait", 1)
    aspect = float(np.float32(width) / np.float32(height))
    mode = "rccl" if args.dist_backend == "nccl" else "host"
    tr = TileSplitRender(pt, rank, world, aspect, reduce=mode, scaling=scaling)
    # the ranks RCCL itself counts in the reduce's communicator (null: no RCCL reduce)
    rccl_ranks = pt.comm_size() if world > 1 and mode == "rccl" else None
    spp_step = spp * world if scaling == "weak" else spp  # frames per rank per step

    def barrier():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[local_rank])
            else:
                dist.barrier()

    def step():
        tr.step(spp)
        tr.reduce(0)  # RCCL sum of the tile images onto rank 0 (no-op at world 1)

    # algorithmic work per step from the instrumented kernel (outside timing)
    st = pt.stats(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp_step)
    taps = pt.tap_stats()  # the shade pass's normal-tap share of st

    for _ in range(args.warmup):
        step()
    pt.sync()
    barrier()
    kernel_ms, trace_ms, trace_n, shade_ms, shade_n = [], [], [], [], []

    chunks = []
    # what the timed dispatches ran (the later legs -- solo pipeline, table
    # kernel -- overwrite the library's read-back): whether the first pass made
    # its own camera rays (gen_trace) and stored no ray records (gen_norec),
    # which select the algorithmic byte model (pipeline_bytes)
    first_pass = {}

    def record_times():
        kernel_ms.append(pt.last_dispatch_ms())  # whole dispatch (all pipeline kernels)
        chunks.append(int(pt.get_option("bin_chunks")))
        first_pass["gen_trace"] = bool(pt.get_option("gen_trace"))
        first_pass["gen_norec"] = bool(pt.get_option("gen_norec"))
        n = int(pt.get_option("trace_launches"))
        if n:  # binned pipeline: the trace / shade passes, timed by events on each pipeline's stream
            trace_ms.append(pt.get_option("trace_ms"))
            trace_n.append(n)
            shade_ms.append(pt.get_option("shade_ms"))
            shade_n.append(int(pt.get_option("shade_launches")))

    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if world == 1:
            record_times()
    pt.sync()
    barrier()
    dt = max_over_ranks(dist, time.perf_counter() - t0, dev)
    # the table of check[] sets after the last timed dispatch:
    # the distinct sets its last chunk saw (of PT_BINS slots) and the sets
    # that found no slot and shared a hash bin (-1: no table in use)
    bin_table = {"slots": 4096, "sets_last_chunk": int(pt.get_option("bin_sets")),
                 "overflow": int(pt.get_option("bin_overflow"))}
    if world > 1:
        # per-launch kernel time on this rank (events on the library stream)
        tr.step(spp)
        record_times()
    render = rank_render_ms(dist, kernel_ms[-1], dev)  # one step's dispatch on each rank
    reduce_ms = reduce_probe(tr, pt, barrier, dist, dev)
    # every frame rendered so far, assembled on rank 0 (all ranks take part
    # in the reduce); checked there against a fresh render of ~8 tiles, and
    # with --validate against a re-render of the whole image
    img = tr.image(0)
    # the boundary's one host transfer per render: the RGBA32F image read
    # back (pt_read_accum, the reference's save_image copy, state.rs:243-263),
    # timed alone after the steps; value_pcie_inclusive counts it once per step
    readback = None
    if world == 1:
        rb = []
        for _ in range(3):
            pt.sync()
            t1 = time.perf_counter()
            pt.read_image()
            rb.append(time.perf_counter() - t1)
        readback = float(np.median(rb))
    validation = None
    if rank == 0:
        if not args.no_tile_check:
            tile_check = validate_tiles(img, prog, settings, width, height, local_rank, tr.frame - 1, world, seed=3)
        if args.validate:
            ref = PathTracer(width, height, prog, device=local_rank, settings=settings)
            ref.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), tr.frame - 1)
            want = ref.read_image()
            validation = {"frames": tr.frame - 1,
                          "bit_exact": bool(np.array_equal(img.view(np.uint32), want.view(np.uint32)))}
            ref.close()
    # (after the checks: the solo and table-kernel runs overwrite the image)
    solo = solo_pipeline(pt, aspect, spp_step) if world == 1 and trace_n else None
    table = table_kernel_leg(pt, prog, aspect, spp_step) if world == 1 and trace_n and not args.no_table_kernel \
        else None
    if table is not None:
        table.update(value_edit_leg(pt, prog))

    pixels = width * height
    samples_step = pixels * spp * (world if scaling == "weak" else 1)  # all ranks
    value = samples_step * args.steps / dt / 1e6
    ms_step = dt * 1e3 / args.steps

    out = None
    if rank == 0:
        out = report(args, pt, st, taps, prog, scene_name, width, height, bounces, spp, spp_step, world, scaling,
                     value, ms_step, kernel_ms, trace_ms, trace_n, shade_ms, shade_n, reduce_ms, ed, validation,
                     solo, chunks, first_pass)
        out["rccl_ranks"] = rccl_ranks
        out["reduce_backend"] = mode if world > 1 else None
        out["render_ms_per_rank"] = render
        out["tile_check"] = tile_check
        out["schedule"]["bin_table"] = bin_table
        if readback is not None:
            out["host_readback"] = {
                "bytes": int(width * height * 16), "ms": round(readback * 1e3, 3),
                "gbs": round(width * height * 16 / readback / 1e9, 2),
                "value_pcie_inclusive": round(samples_step * args.steps / (dt + args.steps * readback) / 1e6, 3),
                "scope": "value with one image readback (pt_read_accum, RGBA32F) per step added; the headline "
                         "value is device-resident (inputs in HBM, the image stays there, as the display pass "
                         "reads it)"}
        if table is not None:
            out["table_kernel"] = table
    pt.close()
    if world > 1 and scaling == "weak" and args.c4_steps > 0 and not args.validate:
        leg = strong_leg(local_rank, rank, world, mode, barrier, dist, dev, args.c4_steps, 1)
        if out is not None:
            out["c4_strong"] = leg
    if out is not None:
        # the line says itself whether it may be trusted (a consumer reading
        # only the JSON sees it, not just the exit status)
        fails = validation_failures(out)
        out["valid"] = not fails
        out["invalid_reasons"] = fails
        print(json.dumps(out), flush=True)
    if dist is not None:
        barrier()
        dist.destroy_process_group()
    rc = exit_status(out)
    if rc:
        sys.exit(rc)


def exit_status(out) -> int:
    """bench.py's exit status once the line is printed: 1 (with the reasons
    on stderr) when validation_failures finds any, else 0.  Ranks other than
    0 hold no line (None) and exit 0."""
    fails = validation_failures(out) if out is not None else []
    if fails:
        print("bench.py: the line is NOT valid: " + "; ".join(fails), file=sys.stderr, flush=True)
        return 1
    return 0


def report(args, pt, st, taps, prog, scene_name, width, height, bounces, spp, spp_step, world, scaling, value,
           ms_step, kernel_ms, trace_ms, trace_n, shade_ms, shade_n, reduce_ms, ed, validation, solo=None,
           chunks=None, first_pass=None) -> dict:
    """Rank 0's JSON line.  first_pass: gen_trace / gen_norec
    as the timed dispatches ran them (record_times); read back here if
    absent."""
    d_ms = float(np.mean(kernel_ms))  # one dispatch = one step's frames of this rank
    n_chunks = float(np.mean(chunks)) if chunks else 1.0  # binned chunks per dispatch
    flops_step = algorithmic_flops(st)
    rank_pixels = st["samples"] / max(1, spp_step)
    image_bytes = 32.0 * rank_pixels  # 16 B RGBA32F load + 16 B store per pixel per dispatch
    jit = bool(pt.get_option("jit_active"))
    fp = first_pass or {}
    gen_trace = fp["gen_trace"] if "gen_trace" in fp else bool(pt.get_option("gen_trace"))
    gen_norec = fp["gen_norec"] if "gen_norec" in fp else bool(pt.get_option("gen_norec"))
    pipe = pipeline_bytes(st, rank_pixels, gen_trace=gen_trace, gen_norec=gen_norec)
    shade_taps = bool(pt.get_option("shade_taps")) and jit
    n_aabb = prog.n_aabb
    shade = None
    eq = None  # the reference-equivalent view (algorithmic flops over the overlapped timed launches)
    if trace_n:  # dominant kernel: the binned trace pass
        hot = ("pt_bin_trace_m_jit" if shade_taps else "pt_bin_trace_jit") if jit else "pt_bin_trace_kernel"
        shade_kernel = "pt_bin_shade_t_jit" if shade_taps else "pt_bin_shade_kernel"
        launches = float(np.mean(trace_n))
        t_ms = float(np.mean(trace_ms))
        s_ms, s_n = float(np.mean(shade_ms)), float(np.mean(shade_n))
        alg_t = trace_flops(st, taps, n_aabb, gen_trace)
        alg_s = shade_flops(st, taps, n_aabb)
        eq = {"trace_frac": round(alg_t / (t_ms * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4),
              "shade_frac": round(alg_s / (s_ms * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4),
              "trace_ms_per_launch": round(t_ms / launches, 3), "shade_ms_per_launch": round(s_ms / max(1.0, s_n), 3),
              "timing": f"the timed steps: {int(pt.get_option('bin_lanes'))} pipelines, whose kernels share the GPU "
                        "(their launches' event times overlap)",
              "flops": "algorithmic: every counted event at its SURVEY 8(d) weight, culled evaluations included "
                       "(what the reference's loop would execute)"}
        # executed flops over the timed steps' overlapped launch times: the
        # kernels share the GPU there, so their fractions of one peak must
        # sum to <= 1 (the algorithmic view above does not: culled work)
        ov_t, ov_s = executed_split(st, taps, n_aabb, gen_trace)
        ov = {"trace_frac": round(ov_t / (t_ms * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4),
              "shade_frac": round(ov_s / (s_ms * 1e-3) / 1e12 / PEAK_F32_TFLOPS, 4), "timing": eq["timing"],
              "flops": "executed (as roofline.flops)"}
        ov["sum"] = round(ov["trace_frac"] + ov["shade_frac"], 4)
        # executed flops over each kernel's own time: the one-pipeline run
        # (solo_pipeline) when there is one, else the timed steps
        if solo is not None:
            ex_t, ex_s = executed_split(solo["st"], solo["taps"], n_aabb, gen_trace)
            tk_ms, tk_n, sk_ms, sk_n = solo["trace_ms"], solo["trace_n"], solo["shade_ms"], solo["shade_n"]
            timing = (f"one pipeline alone (bin_lanes 1, {solo['frames']} frames = one pipeline's share of a "
                      "step, outside the timed region): HIP events around each launch on its stream")
        else:
            ex_t, ex_s = executed_split(st, taps, n_aabb, gen_trace)
            tk_ms, tk_n, sk_ms, sk_n = t_ms, launches, s_ms, s_n
            timing = eq["timing"]
        achieved_tf = ex_t / (tk_ms * 1e-3) / 1e12
        s_tf = ex_s / (sk_ms * 1e-3) / 1e12
        k_flops, k_ms, kl = ex_t, tk_ms / max(1.0, tk_n), tk_n
        shade = {"kernel": shade_kernel,
                 "achieved": round(s_tf, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(s_tf / PEAK_F32_TFLOPS, 4), "executed_flops_per_launch": round(ex_s / max(1.0, sk_n)),
                 "ms_per_launch": round(sk_ms / max(1.0, sk_n), 3), "launches": sk_n,
                 "ms_per_step_summed": round(s_ms, 3), "launches_per_step": s_n,
                 "scope": "calc_normal's six taps (map() work + 29), bounds() of continuing rays (40 per slab test) "
                          "and shading + RR (100 per hit), less culled tap evaluations"}
    else:  # the tile-resident kernels do the whole path in one launch
        hot = "pt_wave_jit" if jit else "pt_wave_kernel"
        launches = kl = 1.0
        k_ms = d_ms
        k_flops = flops_step - culled_flops(st)
        achieved_tf = k_flops / (d_ms * 1e-3) / 1e12
        timing = "the timed dispatches (one kernel)"
    path_tf = flops_step / (d_ms * 1e-3) / 1e12
    achieved_gbs = pipe["total"] / (d_ms * 1e-3) / 1e9  # whole dispatch: every pass's algorithmic bytes
    data = f"synthetic (scenes.{scenes_fn(scene_name)}"
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": data + ("" if scene_name != "c3" else ": 32-node sdf_editor graph, seed 42") + ")",
        "config": {"workload": f"{scene_name} {width}x{height}, {bounces} bounces, "
                               + (f"{spp * world} spp per step ({spp} per GPU-share)" if scaling == "weak"
                                  else f"{spp} spp per step over all GPUs") + ", progressive accumulate",
                   "width": width, "height": height, "bounces": bounces,
                   "spp_per_step": spp * world if scaling == "weak" else spp, "parallelism": f"tiles{world}",
                   "pipelines": int(pt.get_option("bin_lanes")), "baseline_config": args.config,
                   "scene_kernel": "values-baked tier (jit_bake 2 tier-up, installed before timing; the table "
                                   "kernel an editing session runs between value edits: table_kernel)"
                                   if jit and pt.get_option("jit_tier_active") else
                                   ("table scene kernel" if jit else "op-list interpreter"),
                   # chunking (pt_runtime.hip bin_samples: fixed per context from the device's total memory)
                   "bin_samples": int(pt.get_option("bin_samples")), "chunks_per_dispatch": n_chunks,
                   "bin_fallback": bool(pt.get_option("bin_fallback"))},
        "roofline": {"bound": "valu",
                     "bound_note": "FP32 vector ALU: no dense contraction on this path, so no MFMA, and arithmetic "
                                   "intensity ~65 flop/B of measured traffic is above the HBM ridge; the metric's "
                                   "HBM GB/s is reported under hbm",
                     "kernel": hot, "achieved": round(achieved_tf, 3), "peak": PEAK_F32_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_F32_TFLOPS, 4), "traffic": None,
                     "traffic_source": None,
                     "flops": "executed: the counted events at their SURVEY 8(d) weights, less each culled shape "
                              f"evaluation's transform + SDF + combine (a culled one costs its {W_CULL_TEST}-flop test)",
                     "timing": timing,
                     "algorithmic_flops_per_sample": round(flops_step / max(1, st["samples"]), 1),
                     "kernel_flops_per_launch": round(k_flops / max(1.0, kl)),
                     "kernel_scope": "trace passes (the first with its camera rays and primary bounds()): march "
                                     "map() work + 10 per step" if gen_trace else "trace passes: march",
                     "kernel_ms_per_launch": round(k_ms, 3), "kernel_launches_per_step": launches,
                     "solo_launches": solo["trace_n"] if solo is not None else None,
                     "dispatch_ms_per_step": round(d_ms, 3),
                     "path_achieved": round(path_tf, 3), "path_frac": round(path_tf / PEAK_F32_TFLOPS, 4)},
        "hbm": {"achieved": round(achieved_gbs, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved_gbs / PEAK_HBM_GBS, 6),
                "scope": "the binned pipeline's own algorithmic bytes per dispatch (all passes: 64 B ray records "
                         "between passes, the price of binning) / dispatch time; SURVEY 8(d)'s algorithmic bytes "
                         "of the metric are the image's 32 B per pixel per dispatch (image_gbs)",
                "algorithmic_bytes_per_dispatch": pipe["total"],
                "bytes_per_sample": round(pipe["total"] / max(1, st["samples"]), 1),
                "by_pass": {k: v for k, v in pipe.items() if k not in ("total", "trace_m", "trace_first")},
                "image_bytes_per_dispatch": image_bytes,
                "image_gbs": round(image_bytes / (d_ms * 1e-3) / 1e9, 3)},
        "work": st,
        "schedule": schedule_metrics(st, taps),
        "jit": {"active": jit, "compile_s": round(pt.get_option("jit_seconds"), 3),
                "tier_active": bool(pt.get_option("jit_tier_active")),
                "tier_compile_s": round(pt.get_option("jit_tier_seconds"), 3),
                "trace_waves_per_simd": pt.get_option("jit_trace_waves"),
                # 1: the scene kernels came from the shipped cache (lib/jitcache), 0: this process compiled them
                "from_shipped_cache": int(pt.get_option("jit_cache")),
                "shade_waves_per_simd": pt.get_option("jit_shade_waves")},
    }
    if shade is not None:
        out["roofline"]["shade"] = shade
        # the two kernels' executed fractions while they share the GPU (the
        # timed steps): <= 1 by construction of a consistent accounting; each
        # one's solo frac (roofline.frac, shade.frac) is over its own time
        out["roofline"]["overlapped"] = ov
        out["roofline"]["fracs_sum"] = ov["sum"]
    if eq is not None:
        out["roofline"]["reference_equivalent"] = eq
        out["roofline"]["reference_equivalent_frac"] = eq["trace_frac"]
    if world > 1:
        out["reduce_ms"] = round(reduce_ms, 3)
    if validation is not None:
        out["validation"] = validation
    # display pass, outside the timed region: HBM-bound
    # elementwise kernel, 16 B read + 4 B written per pixel (sRGB8 surface)
    pt.display(srgb8=True)
    dms = [pt.get_option("display_ms") for _ in range(3) if pt.display(srgb8=True) is not None]
    disp_ms = float(min(dms))
    d_bytes = 20.0 * width * height
    out["display"] = {"kernel": "pt_display_kernel (srgb8)", "ms": round(disp_ms, 4),
                      "achieved_gbs": round(d_bytes / (disp_ms * 1e-3) / 1e9, 1), "peak_gbs": PEAK_HBM_GBS,
                      "algorithmic_bytes": d_bytes}
    prof = profiled(out["config"])
    if prof is not None and trace_n:
        pd, src = prof
        pk = pd["per_kernel"]
        # measured HBM bytes per launch (FETCH_SIZE + WRITE_SIZE, calibrated
        # on the pipeline's own access shapes: scripts/summarize_profile.py)
        # next to the same kernel's algorithmic bytes per launch
        lanes = int(pt.get_option("bin_lanes"))
        # one first pass (pt_bin_trace_g_jit) per pipeline per chunk
        n_first = float(lanes) * n_chunks
        n_march = max(1.0, float(np.mean(trace_n)) - n_first)
        # the profile ran one pipeline: a launch there carries `lanes` times
        # the frames of a launch here
        scale = float(pd["bench_config"].get("pipelines", 1)) / float(lanes)
        tk = pk.get(hot) or {}
        if "hbm_bytes_per_launch" in tk:
            # per access shape (profiles/r04q_calib_traffic.json): FETCH_SIZE
            # counts the 64 B record gathers at 1.00 of their bytes; WRITE_SIZE
            # counts the march pass's only stores, 16 B hit quads at scattered
            # binned positions, at 2.00 (a 32 B granule moves), so the
            # corrected figure halves the writes.  The 4 B slot reads (6 % of
            # the bytes) are left as counted.
            fetch, write = tk.get("fetch_bytes_per_launch"), tk.get("write_bytes_per_launch")
            if fetch is not None and write is not None and hot == "pt_bin_trace_m_jit":
                out["roofline"]["traffic"] = round((fetch + 0.5 * write) * scale)
                out["roofline"]["traffic_uncorrected"] = round(tk["hbm_bytes_per_launch"] * scale)
                corr = "FETCH_SIZE + WRITE_SIZE / 2 (the 16 B scattered hit-quad stores count twice)"
            else:
                out["roofline"]["traffic"] = round(tk["hbm_bytes_per_launch"] * scale)
                corr = "FETCH_SIZE + WRITE_SIZE, uncorrected"
            out["roofline"]["traffic_source"] = (f"{src} (one pipeline, scaled to this run's launch size): {corr}, "
                                                 f"KiB -> B, per {hot} launch; calibration of the counters on the "
                                                 "pipeline's access shapes: profiles/r04q_calib_traffic.json")
            out["roofline"]["traffic_algorithmic"] = round(pipe["trace_m"] / n_march)
        first = pk.get("pt_bin_trace_g_jit") or {}
        if gen_trace and "hbm_bytes_per_launch" in first:
            out["roofline"]["traffic_first_pass"] = {"kernel": "pt_bin_trace_g_jit",
                                                     "measured": round(first["hbm_bytes_per_launch"] * scale),
                                                     "algorithmic": round(pipe["trace_first"] / n_first)}
        sk = pk.get(shade["kernel"]) if shade else None
        if sk and "hbm_bytes_per_launch" in sk:
            # uncorrected: its 16 B coalesced quad reads count half, its
            # scattered 16 B colour updates twice (r04q_calib_traffic.json)
            out["roofline"]["shade"]["traffic"] = round(sk["hbm_bytes_per_launch"] * scale)
            out["roofline"]["shade"]["traffic_note"] = "FETCH_SIZE + WRITE_SIZE, uncorrected"
            out["roofline"]["shade"]["traffic_algorithmic"] = round(pipe["shade"] / max(1.0, float(np.mean(shade_n))))
        out["hbm"]["trace_kernel_measured_bytes_per_launch"] = out["roofline"].get("traffic")
        if tk:
            out["roofline"]["hw"] = dict(hw_view(tk), source=src)
        if solo is not None and tk.get("fp32_flops_per_launch"):
            # the solo dispatch's trace launches: one first pass per chunk, the
            # rest march-only (one pipeline)
            n_g = float(solo.get("chunks", n_chunks)) if gen_trace else 0.0
            n_m = max(0.0, float(solo["trace_n"]) - n_g)
            pmc = tk["fp32_flops_per_launch"] * scale * n_m + \
                (first.get("fp32_flops_per_launch", 0.0) * scale * n_g if gen_trace else 0.0)
            out["roofline"]["measured"] = measured_view(
                pmc, tk, src, solo["trace_ms"], flop_calibration(), "trace", solo["st"], solo["taps"], n_aabb,
                out["roofline"]["frac"])
        if sk:
            out["roofline"]["shade"]["hw"] = dict(hw_view(sk), source=src)
    if not args.no_cpu_baseline and world == 1:
        threads = args.cpu_threads or default_cpu_threads()
        out["cpu_baseline"] = cpu_baseline(ed, width, height, bounces, threads, args.cpu_row_stride, args.cpu_spp)
    return out


def scenes_fn(name: str) -> str:
    from compute_path_tracer_amd import scenes

    return scenes.SCENES[name].__name__


if __name__ == "__main__":
    main()
