#!/usr/bin/env python3
"""Executed FP32 flops per counted event, from the hardware (VERDICT r05
item 3): reconcile SURVEY 8(d)'s algorithmic weights with what the scene
kernels' instructions actually do.

Two steps:

1. ``run`` (on the GPU, under one rocprofv3 PMC pass; ``run <out> sweep``:
   C3 over bounce counts x fields of view, the rows the weights are fitted
   on; ``run <out>``: eight scenes x three bounce counts, for the
   measured-over-SURVEY ratio per scene):

       rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \\
           SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \\
           --kernel-trace -d gpurun_out/flopcal -o pmc --output-format csv -- \\
           python3 scripts/flop_calib.py run gpurun_out/flopcal_configs.jsonl

   renders a set of scenes x bounce counts (one pipeline, binned passes),
   each as an instrumented dispatch (pt_dispatch_stats: the exact event
   counters, kernels named *_stats) followed by the same dispatch on the
   shipped kernels, whose counters the PMC pass records.

2. ``fit`` (anywhere):

       python scripts/flop_calib.py fit gpurun_out/flopcal_sweep gpurun_out/flopcal_sweep.jsonl \\
           gpurun_out/flopcal gpurun_out/flopcal_configs.jsonl > profiles/r06_flop_calibration.json

   groups the PMC rows by configuration (each instrumented block opens
   one), turns each dispatch's instruction counts into FP32 flops (add and
   mul 1, fma 2 per lane, at the dispatch's own VALU lane utilisation: the
   accounting of scripts/summarize_profile.py), sums them per kernel class
   (trace: pt_bin_trace_m_jit + pt_bin_trace_g_jit; shade:
   pt_bin_shade_t_jit) and fits, by non-negative least squares, the flops
   per event of each class's counters.  The weights it prints are what the
   kernels execute per event; bench.py applies them to its own counters
   (roofline.measured.frac_executed_calibrated).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCENES = ("c1", "c2", "c3", "cull", "tiny", "nested", "farbox", "wide")
BOUNCES = (1, 4, 8)
W, H, SPP = 480, 272, 16
# the C3 sweep the weights are fitted on (the kernels are specialised per
# scene -- constants baked, identity steps folded -- so a shape evaluation
# costs a different number of flops in every scene): bounce counts and
# fields of view change the mix of march steps, union transforms, executed
# and culled shape evaluations, camera rays, taps, box tests and shading
SWEEP_BOUNCES = (1, 2, 3, 4, 6, 8, 12, 16)
SWEEP_FOV = (0.5, 1.0, 2.0)

TRACE = ("pt_bin_trace_m_jit", "pt_bin_trace_g_jit")
SHADE = ("pt_bin_shade_t_jit",)

# regressors per kernel class, from the instrumented dispatch's counters
# (st: all passes; taps: the shade pass's normal taps) -- see features()
TRACE_EVENTS = ("march_steps", "xform_union", "shape_evals", "culled", "samples")
SHADE_EVENTS = ("tap_maps", "tap_xform_union", "tap_shape_evals", "tap_culled", "box_tests", "shaded")


def features(st: dict, taps: dict, n_aabb: int) -> dict:
    """Event counts per kernel class.  Trace passes: st less the taps' share
    (the first pass's camera rays and primary bounds() included); shade
    passes: the taps' map() work, the continuing rays' bounds() and the
    shading.  Shape evaluations count the executed ones (less culled)."""
    tr = {k: v - taps.get(k, 0) for k, v in st.items()}
    return {
        # (samples: a camera ray + the primary rays' bounds(), n_aabb slab tests
        # -- one event in a scene, the two are proportional)
        "trace": {"march_steps": tr["march_steps"], "xform_union": tr["xform_union"],
                  "shape_evals": tr["xform_shape"] - tr["culled"], "culled": tr["culled"],
                  "samples": st["samples"]},
        "shade": {"tap_maps": taps["normal_maps"], "tap_xform_union": taps["xform_union"],
                  "tap_shape_evals": taps["xform_shape"] - taps["culled"], "tap_culled": taps["culled"],
                  "box_tests": st["aabb_tests"] - st["samples"] * n_aabb, "shaded": st["shaded"]},
    }


# SURVEY 8(d)'s weights for the same events (bench.py): what the algorithmic
# accounting charges, to set beside the fitted executed weights
def survey_weights(mean_sdf: float, mean_tap_sdf: float, n_aabb: int) -> dict:
    import bench

    ev = bench.W_XFORM + bench.W_FINALISE + 1  # transform + finalise + combine
    return {"trace": {"march_steps": bench.W_MARCH, "xform_union": bench.W_XFORM + bench.W_FINALISE + 1,
                      "shape_evals": ev + mean_sdf, "culled": bench.W_CULL_TEST,
                      "samples": bench.W_CAMERA + bench.W_AABB * n_aabb},
            "shade": {"tap_maps": bench.W_NORMAL / 6.0, "tap_xform_union": bench.W_XFORM + bench.W_FINALISE + 1,
                      "tap_shape_evals": ev + mean_tap_sdf, "tap_culled": bench.W_CULL_TEST,
                      "box_tests": bench.W_AABB, "shaded": bench.W_SHADE}}


def run(out_path: str, mode: str = "scenes") -> None:
    from compute_path_tracer_amd import _native as N
    from compute_path_tracer_amd import scenes
    from compute_path_tracer_amd.path_tracer import PathTracer
    from compute_path_tracer_amd.sdf_editor import CompData

    if mode == "sweep":
        cfgs = [("c3", b, fov) for fov in SWEEP_FOV for b in SWEEP_BOUNCES]
    else:
        cfgs = [(name, b, 1.0) for name in SCENES for b in BOUNCES]
    progs = {}
    with open(out_path, "w") as f:
        for name, b, fov in cfgs:
            if name not in progs:
                progs[name] = scenes.SCENES[name]().compile(CompData())
            prog = progs[name]
            if True:
                st_ = N.Settings(debug=0, bounces=b, scale=1.0, fov=fov, aabb=0)
                pt = PathTracer(W, H, prog, settings=st_)
                pt.set_option("kernel", "binned")
                pt.set_option("bin_lanes", 1)
                pt.set_option("jit_wait", 1)
                c = N.Constants(time=0.0, frame=1, aspect=float(np.float32(W) / np.float32(H)), last_clear=1)
                st = pt.stats(c, SPP)
                taps = pt.tap_stats()
                pt.dispatch(c, SPP)
                pt.sync()
                rec = {"scene": name, "bounces": b, "fov": fov, "width": W, "height": H, "spp": SPP, "n_aabb": prog.n_aabb,
                       "jit_tier_active": bool(pt.get_option("jit_tier_active")),
                       "gen_trace": bool(pt.get_option("gen_trace")), "st": st, "taps": taps}
                f.write(json.dumps(rec) + "\n")
                f.flush()
                print(name, b, fov, flush=True)
                pt.close()


def pmc_rows(src: str) -> list:
    """[(dispatch id, kernel, {counter: value})] in dispatch order."""
    rows = {}
    for fn in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            d = int(r["Dispatch_Id"])
            rows.setdefault(d, [r["Kernel_Name"], {}])
            rows[d][1][r["Counter_Name"]] = rows[d][1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(d, rows[d][0], rows[d][1]) for d in sorted(rows)]


def fp32_flops(c: dict) -> float:
    util = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]) if c.get("SQ_ACTIVE_INST_VALU") else 0.0
    ops = c.get("SQ_INSTS_VALU_ADD_F32", 0.0) + c.get("SQ_INSTS_VALU_MUL_F32", 0.0) + 2.0 * c.get(
        "SQ_INSTS_VALU_FMA_F32", 0.0)
    return ops * 64.0 * util


def group(rows: list, n_cfg: int) -> list:
    """Per configuration: {class: flops} of its shipped-kernel dispatches
    (those after the configuration's instrumented block, before the next)."""
    groups, cur = [], None
    for _, k, c in rows:
        # (the instrumented dispatch's scene kernels end in _stats; its scan,
        # scatter and fold kernels are the shipped ones and belong to no class)
        if "stats" in k or "<true>" in k:
            if cur is None or cur["trace_launches"] or cur["shade_launches"]:
                cur = {"trace": 0.0, "shade": 0.0, "trace_launches": 0, "shade_launches": 0}
                groups.append(cur)
            continue
        if cur is None:
            continue
        for cls, names in (("trace", TRACE), ("shade", SHADE)):
            if any(k.startswith(n) for n in names):
                cur[cls] += fp32_flops(c)
                cur[cls + "_launches"] += 1
    if len(groups) != n_cfg:
        raise SystemExit(f"{len(groups)} instrumented blocks in the PMC rows, {n_cfg} configurations")
    return groups


def load(pairs: list) -> list:
    """[(configuration, {class: measured flops, class_launches: n})] over
    one or more (PMC directory, configurations file) runs."""
    out = []
    for src, cfg_path in pairs:
        cfgs = [json.loads(l) for l in open(cfg_path) if l.strip()]
        out += list(zip(cfgs, group(pmc_rows(src), len(cfgs))))
    return out


def fit(pairs: list, scene: str = "c3") -> dict:
    """NNLS fit of each class's executed flops per event on `scene`'s rows
    (its kernels are specialised: the weights hold for that scene), and
    every row's measured flops next to the SURVEY weights' (the ratio per
    scene shows what the specialisation removes)."""
    from scipy.optimize import nnls

    import bench

    data = load(pairs)
    fit_rows = [(c, g) for c, g in data if c["scene"] == scene]
    ref = max(fit_rows, key=lambda r: (r[0]["bounces"] == 8 and r[0].get("fov", 1.0) == 1.0, r[0]["bounces"]))[0]
    sdf_mean = sum(w * ref["st"][k] for k, w in bench.W_SDF.items()) / max(1, ref["st"]["xform_shape"])
    tap_sdf = sum(w * ref["taps"][k] for k, w in bench.W_SDF.items()) / max(1, ref["taps"]["xform_shape"])
    out = {"source": [{"pmc": os.path.relpath(a, ROOT), "configs": os.path.relpath(b, ROOT)} for a, b in pairs],
           "accounting": "FP32 flops per dispatch = (ADD_F32 + MUL_F32 + 2 FMA_F32) x 64 x VALU lane utilisation "
                         "(SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU); transcendentals excluded",
           "fit_scene": scene, "configs": len(fit_rows), "size": [W, H, SPP], "classes": {}}
    for cls, names in (("trace", TRACE_EVENTS), ("shade", SHADE_EVENTS)):
        sw = survey_weights(sdf_mean, tap_sdf, ref["n_aabb"])[cls]
        X = np.array([[features(c["st"], c["taps"], c["n_aabb"])[cls][n] for n in names] for c, _ in fit_rows], float)
        y = np.array([g[cls] for _, g in fit_rows], float)
        scale = X.max(axis=0)
        scale[scale == 0] = 1.0
        wfit, _ = nnls(X / scale, y)
        wfit = wfit / scale
        pred = X @ wfit
        resid = (y - pred) / np.maximum(y, 1.0)
        alg = X @ np.array([sw[n] for n in names])
        rows = [{"bounces": c["bounces"], "fov": c.get("fov", 1.0), "events": dict(zip(names, X[i].tolist())),
                 "measured_flops": float(y[i]),
                 "fitted_flops": float(pred[i]), "survey_weight_flops": float(alg[i]),
                 "rel_residual": round(float(resid[i]), 4), "launches": g[cls + "_launches"]}
                for i, (c, g) in enumerate(fit_rows)]
        # every scene of the runs: measured over SURVEY-weight flops (each
        # scene at its own mean SDF weight)
        by_scene = {}
        for c, g in data:
            sm = sum(w * c["st"][k] for k, w in bench.W_SDF.items()) / max(1, c["st"]["xform_shape"])
            ts = sum(w * c["taps"][k] for k, w in bench.W_SDF.items()) / max(1, c["taps"]["xform_shape"])
            swc = survey_weights(sm, ts, c["n_aabb"])[cls]
            a = sum(features(c["st"], c["taps"], c["n_aabb"])[cls][n] * swc[n] for n in names)
            by_scene.setdefault(c["scene"], []).append(round(g[cls] / a, 4) if a else None)
        out["classes"][cls] = {
            "kernels": list(TRACE if cls == "trace" else SHADE),
            "events": list(names),
            "executed_flops_per_event": {n: round(float(w), 3) for n, w in zip(names, wfit)},
            "survey_weights": {n: round(float(sw[n]), 3) for n in names},
            "max_abs_rel_residual": round(float(np.max(np.abs(resid))), 4),
            "rms_rel_residual": round(float(np.sqrt(np.mean(resid ** 2))), 4),
            "measured_over_survey": {"fit_scene_rows": [round(float(v), 4) for v in y / alg],
                                     "by_scene_bounces_1_4_8": by_scene},
            "rows": rows}
    return out


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "scenes")
    else:  # fit pmc_dir configs.jsonl [pmc_dir configs.jsonl ...]
        a = sys.argv[2:]
        print(json.dumps(fit(list(zip(a[0::2], a[1::2]))), indent=1))
