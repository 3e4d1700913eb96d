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
sh = d["roofline"].get("shade", {})
print(d["value"], d["roofline"]["kernel_ms_per_launch"], "shade_ms_step", sh.get("ms_per_step_summed"),
      "trace_ms_step", round(d["roofline"]["kernel_ms_per_launch"] * d["roofline"]["kernel_launches_per_step"], 3),
      json.dumps(d.get("schedule", {})), json.dumps(cull))
