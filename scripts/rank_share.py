#!/usr/bin/env python3
"""Weak-scaling rehearsal on one GPU: time one rank's share of a multi-GPU
step (its 1/N of the 8x8 tiles, 64*N frames) for N = 1, 2, 4, 8.  Per-rank
time should stay flat as N grows; the RCCL image reduce is not included.
Usage: python scripts/rank_share.py [--spp 64] [--reps 2]"""
import argparse
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

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
args = ap.parse_args()
prog = scenes.c3_graph32().compile(CompData())
st = N.Settings(debug=0, bounces=8, scale=1.0, fov=1.0, aabb=0)
aspect = float(np.float32(args.width) / np.float32(args.height))
for world in (1, 2, 4, 8):
    pt = PathTracer(args.width, args.height, prog, settings=st)
    pt.set_tiles(0, world)
    frames = args.spp * world
    c = N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1)
    pt.dispatch(c, frames)  # warm-up (allocation, JIT)
    pt.sync()
    best = None
    for _ in range(args.reps):
        t0 = time.perf_counter()
        pt.dispatch(c, frames)
        pt.sync()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    samples = args.width * args.height * args.spp  # this rank's share
    print(json.dumps({"world": world, "frames": frames, "rank_ms": round(best * 1e3, 2),
                      "rank_msamples_s": round(samples / best / 1e6, 1),
                      "dispatch_ms": round(pt.last_dispatch_ms(), 2)}), flush=True)
    pt.close()
