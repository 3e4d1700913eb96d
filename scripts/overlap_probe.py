"""Timing probe: two independent contexts dispatching alternately (no host
sync between steps) vs one context, same 256-spp C3 steps.  Estimates what
overlapping consecutive dispatches (one's drain with the next one's first
passes) could gain.  Not a parity check (the two images are separate)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from compute_path_tracer_amd import _native as N, scenes  # noqa: E402
from compute_path_tracer_amd.path_tracer import PathTracer  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402

W, H, SPP, STEPS = 1920, 1080, 256, 6
prog = scenes.c3_graph32().compile(CompData())
st = N.Settings(debug=0, bounces=8, scale=1.0, fov=1.0, aabb=0)
aspect = float(np.float32(W) / np.float32(H))
ctxs = [PathTracer(W, H, prog, settings=st) for _ in range(2)]
for p in ctxs:
    p.set_option("jit_wait", 1)
    p.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), SPP)
    p.sync()
for mode in ("one", "two", "one", "two"):
    use = ctxs[:1] if mode == "one" else ctxs
    t0 = time.perf_counter()
    for s in range(STEPS):
        use[s % len(use)].dispatch(N.Constants(time=0.0, frame=1 + s * SPP, aspect=aspect, last_clear=1), SPP)
    for p in use:
        p.sync()
    dt = time.perf_counter() - t0
    print(f"{mode}: {W * H * SPP * STEPS / dt / 1e6:.1f} Msamples/s", flush=True)
