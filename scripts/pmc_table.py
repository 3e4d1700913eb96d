#!/usr/bin/env python3
"""Per-launch PMC counter means per kernel from scripts/pmc_passes.sh output.
usage: python scripts/pmc_table.py gpurun_out/pmc_<tag> [kernel-substring ...]"""
import collections
import csv
import glob
import json
import sys

src = sys.argv[1]
want = sys.argv[2:] or ["pt_bin_trace_m_jit", "pt_bin_shade_t_jit"]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
ids = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob(f"{src}/p*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "stats" in k or "<true>" in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ids[k][r["Counter_Name"]].add(r["Dispatch_Id"])
out = {}
for k, c in tot.items():
    if not any(w in k for w in want):
        continue
    out[k] = {n: v / max(1, len(ids[k][n])) for n, v in sorted(c.items())}
print(json.dumps(out, indent=1))
