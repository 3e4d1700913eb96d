#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (gpurun_out/prof_<tag>) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<tag>_pmc.json (per-launch counters of the hot kernel and derived
metrics, plus the derived metrics of the other pipeline kernels) and
profiles/<tag>_summary.md.

HBM bytes per launch: FETCH_SIZE*1024 + WRITE_SIZE*1024, each counter from
its own pass.  MI355X_MICROARCH.md ("HBM") has FETCH_SIZE at exactly half of
a wide coalesced 16 B/lane read and leaves other shapes uncalibrated; the
pipeline's own shapes were calibrated with known-byte probes (pt_probe.hip,
profiles/r04q_calib_traffic.json): a 64 B record gathered by slot reads
FETCH_SIZE = its bytes (ratio 1.0), a 64 B record store WRITE_SIZE = its
bytes, a 16 B store at a scattered position WRITE_SIZE = 2x (a 32 B write
granule moved), a 16 B/lane coalesced read FETCH_SIZE = half.  The sums
here are the raw counters.  They are not exact for every kernel: the march
pass's (pt_bin_trace_m_jit) only stores are 16 B hit quads at scattered
positions, which WRITE_SIZE counts twice, so bench.py reports its traffic as
FETCH_SIZE + WRITE_SIZE / 2 (fetch_bytes_per_launch and
write_bytes_per_launch are kept apart for that); the shade pass mixes
shapes (coalesced 16 B quad reads counted half, scattered 16 B colour
updates twice, exact 64 B gathers and stores) and is left uncorrected.
The hot kernel is the binned trace pass when present (averages over its
launches), else the tile-resident kernel; every kernel's figures are in
per_kernel.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOT = ("pt_bin_trace_m_jit", "pt_bin_trace_jit", "pt_bin_trace_kernel", "pt_wave_jit", "pt_wave_kernel", "pt_render_kernel")


def hot_name(name: str) -> bool:
    return any(name.startswith(h) and "stats" not in name and "<true>" not in name for h in HOT)


def collect(src: str) -> dict:
    """{kernel name: (per-launch counters, launch meta)} over every PMC pass."""
    counters, launches, meta = {}, {}, {}
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            n, k = r["Kernel_Name"], r["Counter_Name"]
            counters.setdefault(n, {})
            counters[n][k] = counters[n].get(k, 0.0) + float(r["Counter_Value"])
            launches.setdefault(n, {}).setdefault(k, set()).add(r["Dispatch_Id"])
            meta[n] = {"kernel": n, "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                       "lds_bytes": int(r["LDS_Block_Size"]), "grid": int(r["Grid_Size"]),
                       "workgroup": int(r["Workgroup_Size"])}
    return {n: ({k: v / max(1, len(launches[n][k])) for k, v in c.items()}, meta[n]) for n, c in counters.items()}


def derive(c: dict) -> dict:
    d = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
        d["write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch"] = d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"]
    if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
        d["valu_lane_utilization"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_INSTS_VALU"):
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        d["gpu_cycles"] = cyc
        d["valu_issue_per_simd_cycle"] = c["SQ_INSTS_VALU"] / (1024.0 * cyc)
        d["valu_issue_frac_of_peak"] = d["valu_issue_per_simd_cycle"] / 0.5  # wave64 VALU = 2 cycles on SIMD32
        d["salu_per_valu"] = c.get("SQ_INSTS_SALU", 0.0) / c["SQ_INSTS_VALU"]
    if "SQ_INSTS_VALU_FMA_F32" in c and "valu_lane_utilization" in d:
        # FP32 flops the kernel executed, from its instruction counts: add and
        # mul 1, fma 2 per lane (transcendentals excluded, as in the
        # algorithmic weights), at the kernel's mean VALU lane utilisation
        ops = c.get("SQ_INSTS_VALU_ADD_F32", 0.0) + c.get("SQ_INSTS_VALU_MUL_F32", 0.0) + \
            2.0 * c["SQ_INSTS_VALU_FMA_F32"]
        d["fp32_flops_per_launch"] = ops * 64.0 * d["valu_lane_utilization"]
        d["fp32_trans_insts_per_launch"] = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        if c.get("SQ_INSTS_VALU"):
            d["fp32_insts_frac_of_valu"] = (ops - c["SQ_INSTS_VALU_FMA_F32"]) / c["SQ_INSTS_VALU"]
    if c.get("SQ_WAVE_CYCLES"):
        tot = c["SQ_WAVE_CYCLES"]
        d["wave_time_active"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / tot
        d["wave_time_wait_issue"] = c.get("SQ_WAIT_INST_ANY", 0.0) / tot
        d["wave_time_waitcnt"] = c.get("SQ_WAIT_ANY", 0.0) / tot
    return d


def launch_split(src: str, n_solo: int) -> dict:
    """Average kernel-trace durations (ms) of the trace passes (march-only +
    first pass) and the shade passes, split into bench.py's last n_solo
    launches of each (its one-pipeline solo dispatch, the roofline's timing)
    and all earlier ones (warm-up and timed steps)."""
    f = os.path.join(src, "kt", "kt_kernel_trace.csv")
    if not os.path.exists(f) or n_solo <= 0:
        return {}
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    for key, names in (("trace", ("pt_bin_trace_m_jit", "pt_bin_trace_g_jit")), ("shade", ("pt_bin_shade_t_jit",))):
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows if r["Kernel_Name"] in names]
        if len(ms) > n_solo:
            out[key + "_solo_ms"] = sum(ms[-n_solo:]) / n_solo
            out[key + "_timed_ms"] = sum(ms[:-n_solo]) / (len(ms) - n_solo)
    return out


def main(tag: str, src: str = None) -> None:
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(ks, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(ks)))
    bench_line = None
    for line in open(os.path.join(src, "kt_bench.log")):
        if line.startswith("{"):
            bench_line = json.loads(line)
    present = [r["Name"] for r in stats if hot_name(r["Name"])]
    hot = min(present, key=lambda n: [i for i, h in enumerate(HOT) if n.startswith(h)][0]) if present else None
    per_kernel = collect(src)
    per_launch, meta = per_kernel.get(hot, ({}, {}))
    d = derive(per_launch)

    def avg_s(name):
        t = [float(r["AverageNs"]) * 1e-9 for r in stats if r["Name"] == name]
        return t[0] if t else None

    ktime = avg_s(hot)
    # bench.py's HIP events time every trace launch, the first pass's
    # pt_bin_trace_g_jit (own camera rays) included: the launch-weighted
    # average over both is the figure to compare
    trace_rows = [r for r in stats if r["Name"] == hot or r["Name"] == "pt_bin_trace_g_jit"]
    calls = sum(int(r["Calls"]) for r in trace_rows)
    trace_avg = sum(float(r["TotalDurationNs"]) for r in trace_rows) * 1e-9 / calls if calls else None
    if ktime and "hbm_bytes_per_launch" in d:
        d["hbm_gbs_measured"] = d["hbm_bytes_per_launch"] / ktime / 1e9
    others, every = {}, {}
    for n, (c, m) in sorted(per_kernel.items()):
        if "<true>" in n or "stats" in n:
            continue
        ed = derive(c)
        kt = avg_s(n)
        ed["avg_s_kernel_trace"] = kt
        if kt and "hbm_bytes_per_launch" in ed:
            ed["hbm_gbs_measured"] = ed["hbm_bytes_per_launch"] / kt / 1e9
        if kt and "fp32_flops_per_launch" in ed:
            ed["fp32_tflops_measured"] = ed["fp32_flops_per_launch"] / kt / 1e12
        every[n] = dict(ed, vgpr=m.get("vgpr"), grid=m.get("grid"))
    for n, (c, _) in sorted(per_kernel.items()):
        if n == hot or "<true>" in n or "stats" in n:
            continue
        od = derive(c)
        kt = avg_s(n)
        if kt and "hbm_bytes_per_launch" in od:
            od["hbm_gbs_measured"] = od["hbm_bytes_per_launch"] / kt / 1e9
        others[n] = od
    out = {"tag": tag, "kernel": meta, "per_launch_counters": per_launch, "derived": d,
           "kernel_avg_s_kernel_trace": ktime,
           "trace_launch_avg_s_kernel_trace": trace_avg,
           "bench_config": bench_line["config"] if bench_line else None,
           "bench_value": bench_line["value"] if bench_line else None,
           "bench_kernel_ms_hip_events": bench_line["roofline"]["kernel_ms_per_launch"] if bench_line else None,
           "bench_shade_ms_hip_events": (bench_line["roofline"].get("shade") or {}).get("ms_per_launch")
           if bench_line else None,
           "shade_avg_s_kernel_trace": avg_s("pt_bin_shade_t_jit"),
           "other_kernels": others, "per_kernel": every}
    # bench.py's own HIP-event times next to the kernel trace of the same run:
    # its solo dispatch (the roofline's timing) and the steps before it
    rl = bench_line["roofline"] if bench_line else {}
    n_solo = rl.get("solo_launches") or ((rl.get("shade") or {}).get("launches")
                                         if str(rl.get("timing", "")).startswith("one pipeline alone") else None)
    if n_solo:
        ls = launch_split(src, int(n_solo))
        eq = bench_line["roofline"].get("reference_equivalent") or {}
        out["event_vs_trace_ms"] = {
            "trace_solo": (bench_line["roofline"]["kernel_ms_per_launch"], ls.get("trace_solo_ms")),
            "shade_solo": ((bench_line["roofline"].get("shade") or {}).get("ms_per_launch"), ls.get("shade_solo_ms")),
            "trace_steps": (eq.get("trace_ms_per_launch"), ls.get("trace_timed_ms")),
            "shade_steps": (eq.get("shade_ms_per_launch"), ls.get("shade_timed_ms"))}
    with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    lines = [f"# rocprofv3 summary `{tag}`", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py {bench_line['steps'] if bench_line else ''}`"
             " (see scripts/profile.sh); PMC passes one counter group each.", "",
             "## Kernel stats", "", "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
    for r in stats:
        lines.append(f"| {r['Name']} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
    if out.get("event_vs_trace_ms"):
        lines += ["", "bench.py HIP events vs rocprofv3 kernel trace, ms per launch (trace = march-only + first pass):"]
        for k, (ev, kt) in out["event_vs_trace_ms"].items():
            lines.append(f"- {k}: events {ev}, kernel trace {kt}")
    lines += ["", f"HIP-event time per trace launch inside bench.py: "
                  f"{out['bench_kernel_ms_hip_events']} ms; rocprofv3 over the same launches "
                  f"({hot} + pt_bin_trace_g_jit, launch-weighted): "
                  f"{trace_avg * 1e3 if trace_avg else None} ms", "",
              f"HIP-event time per shade launch inside bench.py: {out['bench_shade_ms_hip_events']} ms; "
              f"rocprofv3 (pt_bin_shade_t_jit): "
              f"{out['shade_avg_s_kernel_trace'] * 1e3 if out['shade_avg_s_kernel_trace'] else None} ms", "",
              "## Hot kernel counters (per launch)", "", f"kernel: {meta}", ""]
    for k, v in sorted(per_launch.items()):
        lines.append(f"- {k}: {v:.6g}")
    lines += ["", "## Derived", ""]
    for k, v in d.items():
        lines.append(f"- {k}: {v:.6g}")
    if others:
        lines += ["", "## Other pipeline kernels (derived, per launch)", ""]
        for n, od in others.items():
            lines.append(f"- `{n}`: " + ", ".join(f"{k} {v:.4g}" for k, v in od.items()))
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(json.dumps(out["derived"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
