#!/usr/bin/env python3
"""Find non-finite texels of a full-size render and re-render their 8x8
tiles with the oracle (rank = tile, nranks = #tiles selects one tile) to
check the GPU result there bit for bit."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from compute_path_tracer_amd import _native as N  # noqa: E402
from compute_path_tracer_amd import scenes  # noqa: E402
from compute_path_tracer_amd.path_tracer import PathTracer  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402
from oracle import oracle as O  # noqa: E402  (test infrastructure: the checker)

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
scene, w, h, spp, bounces = scenes.CONFIGS[name]
ed = scenes.SCENES[scene]()
st = N.Settings(debug=0, bounces=bounces, scale=1.0, fov=1.0, aabb=0)
pt = PathTracer(w, h, ed.compile(CompData()), settings=st)
aspect = float(np.float32(w) / np.float32(h))
pt.dispatch(N.Constants(time=0.0, frame=1, aspect=aspect, last_clear=1), spp)
img = pt.read_image()
bad = np.argwhere(~np.isfinite(img[..., :3]).all(-1))
tx = (w + 7) // 8
tiles = sorted({(int(y) // 8) * tx + int(x) // 8 for y, x in bad})
print(json.dumps({"config": name, "nonfinite_texels": int(len(bad)), "tiles": len(tiles), "first": bad[:4].tolist()}))
osc = O.OracleScene(ed.rows())
ntiles = tx * ((h + 7) // 8)
for t in tiles[:4]:
    ref = osc.render(w, h, O.Constants(0.0, 1, aspect, 1), O.Settings(0, bounces, 1.0, 1.0, 0), spp, rank=t,
                     nranks=ntiles, threads=16)
    y0, x0 = (t // tx) * 8, (t % tx) * 8
    a, b = img[y0:y0 + 8, x0:x0 + 8], ref[y0:y0 + 8, x0:x0 + 8]
    print(json.dumps({"tile": t, "bit_exact": bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))),
                      "oracle_nonfinite": int((~np.isfinite(b[..., :3])).any(-1).sum())}), flush=True)
