#!/usr/bin/env python3
"""Print the key fields of the last JSON line of a bench.py log."""
import json
import sys

line = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1]
d = json.loads(line)
print(d["value"], d["roofline"]["kernel_ms_per_launch"], json.dumps(d.get("schedule", {})))
