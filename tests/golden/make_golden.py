#!/usr/bin/env python3
"""Regenerates the committed fixtures in tests/golden/.

1. shader_out_topology.json -- parsed from the ONLY captured output of the
   reference scene compiler, /root/reference/assets/shaders/path_tracer/
   shader_out/test_compute.glsl:185-392 (2 header unions, 7 shapes).  Records,
   in emission order, every data[] slot the generated bounds()/map() reads,
   the check[] guard of each shape and the combine statement.  Only numbers
   are extracted (no source text is kept).
2. rng_kat.json -- wang_hash / gen_rng / RandomFloat01 known answers from the
   pure-integer restatement in tests/pyref.py (rng.glsl:1-36).
3. oracle_*.npy -- small oracle images (regression pins of the C oracle,
   cross-checked against tests/pyref.py when generated).

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

REF_GLSL = "/root/reference/assets/shaders/path_tracer/shader_out/test_compute.glsl"


def _ints(s):
    return [int(v) for v in re.findall(r"data\[(\d+)\]", s)]


def parse_topology(path: str) -> dict:
    txt = open(path).read()
    b0 = txt.index("CHECK_ARRAY bool[")
    n_check = int(re.search(r"CHECK_ARRAY bool\[(\d+)\]", txt).group(1))
    bounds_txt = txt[b0:txt.index("#define MAXHIT")]
    bounds = []
    for m in re.finditer(r"if \((.*?)\) \{\s*back\[(\d+)\] = true;", bounds_txt, re.S):
        cond, idx = m.group(1), int(m.group(2))
        if cond.strip() == "false":
            bounds.append({"back": idx, "enabled": False})
            continue
        # from_pos_size(vec3(up) + vec3(sp), (SO * ( us * ss)) * ex)
        pos_part, size_part = cond.split("from_pos_size(", 1)[1].split(",", 3)[0:3], None
        mm = re.search(r"from_pos_size\((vec3\([^)]*\)) \+ (vec3\([^)]*\)), \((.*?) \* \( (data\[\d+\]) \* (data\[\d+\])\)\) \* (data\[\d+\])",
                       cond)
        up, sp, so, us, ss, ex = mm.groups()
        bounds.append({"back": idx, "enabled": True, "union_position": _ints(up), "shape_position": _ints(sp),
                       "size": _ints(so), "union_scale": _ints(us)[0], "shape_scale": _ints(ss)[0],
                       "aabb_exaggeration": _ints(ex)[0]})
    map_txt = txt[txt.index("Hit map(vec3 pu0"):]
    map_txt = map_txt[:map_txt.index("return start;")]
    unions = []
    for ub in re.finditer(r"Hit u1 = MAXHIT;(.*?)start = (op\w+)\(start, u1\);\} //(\w+)", map_txt, re.S):
        body, comb, name = ub.group(1), ub.group(2), ub.group(3)
        ut = re.search(r"pu1 \*= 1\.0 / data\[(\d+)\];\s*pu1 = move\(pu1, (vec3\([^)]*\)) \* \(1\.0 / data\[(\d+)\]\)\);"
                       r"\s*pu1 = rot3D\(pu1, (vec3\([^)]*\))\);", body)
        shapes = []
        for sm in re.finditer(r"if \((check\[(\d+)\]|true)\)\s*\{(.*?)\n\s*\}", body, re.S):
            guard, chk, sb = sm.group(1), sm.group(2), sm.group(3)
            tr = re.search(r"(u1s\d+)p \*= 1\.0 / data\[(\d+)\];\s*\1p = move\(\1p, (vec3\([^)]*\)) \* \(1\.0 / "
                           r"data\[(\d+)\]\)\);\s*\1p = rot3D\(\1p, (vec3\([^)]*\))\);", sb)
            sdf = re.search(r"(sdCube|sdSphere)\(u1s\d+p, (.*?)\),\s*Mat\((.*?)\)\s*\);", sb, re.S)
            fin = re.search(r"u1s\d+\.d /= 1\.0 / data\[(\d+)\];", sb)
            comb_s = re.search(r"u1 = (opUnion|opSubtraction)\(u1, u1s\d+\);|u1 = u1s\d+;", sb)
            shapes.append({
                "check": int(chk) if chk is not None else None,
                "kind": "Cube" if sdf.group(1) == "sdCube" else "Sphere",
                "scale": int(tr.group(2)), "position": _ints(tr.group(3)), "scale_again": int(tr.group(4)),
                "rotation": _ints(tr.group(5)), "size": _ints(sdf.group(2)), "material": _ints(sdf.group(3)),
                "finalise_scale": int(fin.group(1)),
                "combine": comb_s.group(1) if comb_s.group(1) else "assign",
            })
        unions.append({"name": name, "scale": int(ut.group(1)), "position": _ints(ut.group(2)),
                       "scale_again": int(ut.group(3)), "rotation": _ints(ut.group(4)), "combine": comb,
                       "shapes": shapes})
    return {"source": "assets/shaders/path_tracer/shader_out/test_compute.glsl:185-392", "n_check": n_check,
            "bounds": bounds, "unions": unions}


def rng_kat() -> dict:
    import pyref

    seeds = [0, 1, 61, 0xFFFFFFFF, 0x12345678, 0x80000000, 26699, 9277]
    seq = {}
    for s in seeds:
        out, st = [], s
        for _ in range(8):
            st = pyref.wang_hash(st)
            out.append(st)
        seq[str(s)] = out
    gen = []
    for (x, y, f, w, h) in [(0, 0, 0, 256, 256), (255, 255, 1, 256, 256), (1919, 1079, 7, 1920, 1080),
                            (3839, 2159, 123456, 3840, 2160), (17, 3, -5, 64, 48), (0, 1079, 2**31 - 1, 1920, 1080)]:
        gen.append({"x": x, "y": y, "frame": f, "w": w, "h": h, "seed": pyref.gen_rng(x, y, f, w, h)})
    f01 = []
    for s in [1, 12345, 0xDEADBEEF]:
        r = pyref.Rng(s)
        f01.append({"seed": s, "bits": [int(np.float32(r.f01()).view(np.uint32)) for _ in range(6)]})
    return {"wang_hash": seq, "gen_rng": gen, "random01": f01}


def oracle_images():
    from compute_path_tracer_amd import scenes
    from oracle import oracle as O
    import pyref

    cases = {
        "oracle_c1_32x32_s2_b1": ("c1", 32, 32, 2, 1, 0),
        "oracle_c2_16x12_s2_b4": ("c2", 16, 12, 2, 4, 0),
        "oracle_c3_8x6_s1_b8": ("c3", 8, 6, 1, 8, 0),
        "oracle_nested_8x8_s1_b4": ("nested", 8, 8, 1, 4, 0),
        "oracle_c3_dbg1_8x6": ("c3", 8, 6, 1, 8, 1),
        "oracle_c3_dbg2_8x6": ("c3", 8, 6, 1, 8, 2),
        "oracle_c3_dbg3_8x6": ("c3", 8, 6, 1, 8, 3),
    }
    meta = {}
    for name, (sc, w, h, spp, b, dbg) in cases.items():
        rows = scenes.SCENES[sc]().rows()
        a = float(np.float32(w) / np.float32(h))
        img = O.OracleScene(rows).render(w, h, O.Constants(0.0, 1, a, 1), O.Settings(dbg, b, 1.0, 1.0, 0), spp)
        py = pyref.render(rows, w, h, 1, 1, a, b, spp, debug=dbg)
        same = np.array_equal(img.view(np.uint32), py.view(np.uint32))
        print(f"{name}: oracle == pyref: {same}")
        assert same, name
        np.save(os.path.join(HERE, name + ".npy"), img, allow_pickle=False)
        meta[name] = {"scene": sc, "w": w, "h": h, "spp": spp, "bounces": b, "debug": dbg, "frame": 1,
                      "last_clear": 1, "sha256": hashlib.sha256(img.tobytes()).hexdigest()}
    with open(os.path.join(HERE, "oracle_images.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    if os.path.exists(REF_GLSL):
        with open(os.path.join(HERE, "shader_out_topology.json"), "w") as f:
            json.dump(parse_topology(REF_GLSL), f, indent=1)
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(rng_kat(), f, indent=1)
    if "--no-images" not in sys.argv:
        oracle_images()
