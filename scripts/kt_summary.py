"""One line per run: per-step device time of each binned pipeline kernel
(non-instrumented launches, 3 dispatches per bench run: warm-up + 2 steps)
and the bench value.  Usage: python scripts/kt_summary.py <rocprofv3 -d dir>"""
import csv
import json
import os
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows = list(csv.DictReader(open(os.path.join(d, "kt_kernel_stats.csv"))))
out = {}
for r in rows:
    n = r["Name"].split("(")[0]
    if "stats" in n or not n.startswith("pt_bin"):
        continue
    out[n.replace("pt_bin_", "")] = round(float(r["TotalDurationNs"]) / 1e6 / steps, 2)
val = None
log = d + ".log"
if os.path.exists(log):
    for line in open(log):
        if line.startswith("{"):
            val = json.loads(line).get("value")
print(json.dumps({"dir": os.path.basename(d), "value": val, "ms_per_step": out}))
