#!/usr/bin/env python3
"""Run the library's traffic probes (pt_probe.hip) once and print one JSON
line: per probe kernel its known bytes, device time and GB/s.  Run under
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE by scripts/pmc_calib.sh."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from compute_path_tracer_amd import _native as N  # noqa: E402

NAMES = ("pt_probe_gather64", "pt_probe_stream16", "pt_probe_scatter16", "pt_probe_store64")
log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ms = (ctypes.c_float * 4)()
nb = (ctypes.c_uint64 * 4)()
N.check("pt_traffic_probe", N.lib().pt_traffic_probe(0, log2n, ms, nb))
print(json.dumps({n: {"bytes": int(nb[k]), "ms": round(ms[k], 4), "gbs": round(nb[k] / (ms[k] * 1e-3) / 1e9, 1)}
                  for k, n in enumerate(NAMES)}))
