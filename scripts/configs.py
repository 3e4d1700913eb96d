#!/usr/bin/env python3
"""Every BASELINE.json config on one GPU (scenes.CONFIGS): full resolution,
spp and bounces, one pt_dispatch each, device time from HIP events.  C4 is
the 8-GPU config; here it runs whole on one GPU (its per-GPU share is 1/8).
Usage: python scripts/configs.py [c1 c2 ...] > profiles/<tag>_configs.jsonl"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from compute_path_tracer_amd import _native as N  # noqa: E402
from compute_path_tracer_amd import scenes  # noqa: E402
from compute_path_tracer_amd.path_tracer import PathTracer  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402

names = sys.argv[1:] or list(scenes.CONFIGS)
for name in names:
    scene, w, h, spp, bounces = scenes.CONFIGS[name]
    prog = scenes.SCENES[scene]().compile(CompData())
    st = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
    pt = PathTracer(w, h, prog, settings=st)
    pt.set_option("jit_wait", 1)  # setup: the values-baked scene kernel, as bench.py
    aspect = float(np.float32(w) / np.float32(h))
    # warm-up with the timed dispatch's own spp: the same kernel choice, and
    # the binned pipeline's chunk buffers (sized by the dispatch's samples,
    # up to 81.6 GB) allocated before timing -- a smaller warm-up left their
    # allocation, or the first launch of the binned kernels, inside the timed
    # dispatch (r02s: C2 at 68-5000 Msamples/s from box to box)
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)
    pt.sync()
    pt.clear()
    t0 = time.perf_counter()
    pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)
    pt.sync()
    wall = time.perf_counter() - t0
    ms = pt.last_dispatch_ms()
    img = pt.read_image()
    print(json.dumps({"config": name, "scene": scene, "width": w, "height": h, "spp": spp, "bounces": bounces,
                      "device_ms": round(ms, 2), "wall_ms": round(wall * 1e3, 2),
                      "msamples_s": round(w * h * spp / (ms * 1e-3) / 1e6, 1),
                      "mean_radiance": float(img[..., :3].mean())}), flush=True)
    pt.close()
