#!/usr/bin/env python3
"""Print the key fields of the last JSON line of a bench.py log."""
import json
import sys

line = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
w = d.get("work", {})
cull = {}
if w.get("xform_shape"):
    cull = {"lane_culled": round(w["culled"] / w["xform_shape"], 4),
            "wave_evals_per_shape": round(w["wave_evals"] / max(1, w["wave_shapes"]), 4),
            "wave_evals_per_map": round(w["wave_evals"] / max(1, w["wave_maps"]), 3)}
r = d["roofline"]
sh, eq = r.get("shade", {}), r.get("reference_equivalent", {})
print(d["value"], "trace_ms_launch", eq.get("trace_ms_per_launch"), "shade_ms_launch", eq.get("shade_ms_per_launch"),
      "solo trace/shade ms", r["kernel_ms_per_launch"], sh.get("ms_per_launch"), "frac", r["frac"], sh.get("frac"),
      json.dumps(d.get("schedule", {})), json.dumps(cull))
