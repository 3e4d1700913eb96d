#!/usr/bin/env python3
"""Ratios of rocprofv3's FETCH_SIZE / WRITE_SIZE (KiB) to the known bytes of
each traffic probe (scripts/pmc_calib.sh output dir) -> <dir>/calib.json."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
plain = json.loads([l for l in open(os.path.join(d, "calib_plain.log")) if l.startswith("{")][-1])
out = {}
for counter in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(d, f"calib_{counter}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            for name, p in plain.items():
                if name in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    b = float(r["Counter_Value"]) * 1024.0
                    out.setdefault(name, dict(p))[counter.lower() + "_bytes"] = b
                    out[name][counter.lower() + "_ratio"] = round(b / p["bytes"], 4)
json.dump(out, open(os.path.join(d, "calib.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
