#!/usr/bin/env python3
"""Device time of one dispatch per kernel family over workload sizes, to place
the automatic kernel choice (pt_runtime make_launch: the tile-resident wave
kernel below a sample count, the binned passes above).  Usage:
python scripts/kernel_crossover.py > gpurun_out/crossover.jsonl"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from compute_path_tracer_amd import _native as N  # noqa: E402
from compute_path_tracer_amd import scenes  # noqa: E402
from compute_path_tracer_amd.path_tracer import PathTracer  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402

KERNELS = {"wave": 2, "binned": 3}  # pt_device.h PT_KERNEL_WAVEFRONT, PT_KERNEL_BINNED
for scene, bounces in (("c1", 1), ("c2", 4), ("c3", 8)):
    prog = scenes.SCENES[scene]().compile(CompData())
    for w, h, spp in ((256, 256, 1), (512, 512, 1), (512, 512, 4), (1024, 1024, 4), (1920, 1080, 4), (1920, 1080, 16)):
        st = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
        pt = PathTracer(w, h, prog, settings=st)
        pt.set_option("jit_wait", 1)
        aspect = float(np.float32(w) / np.float32(h))
        out = {"scene": scene, "width": w, "height": h, "spp": spp, "samples": w * h * spp}
        for name, k in KERNELS.items():
            pt.set_option("kernel", k)
            pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)  # warm-up
            pt.sync()
            best = 1e9
            for _ in range(3):
                pt.clear()
                pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)
                pt.sync()
                best = min(best, pt.last_dispatch_ms())
            out[name + "_ms"] = round(best, 3)
        pt.close()
        print(json.dumps(out), flush=True)
