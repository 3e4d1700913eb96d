#!/usr/bin/env python3
"""Would a wave-level union-box skip pay in the shade pass's bounds()?
(decide with a CPU measurement before any kernel work.)

The shade pass computes bounds() -- one slab test per box, 24 boxes in C3 --
for each continuing ray, one thread per binned position, 64 positions per
wave.  A top-level union's boxes could be skipped by the whole wave when no
lane's ray hits the union's enclosing box (a ray that misses a box enclosing
a union's boxes misses each of them: the IEEE slab values are monotone in
the plane coordinates).  This measures how often that happens:

* the oracle (test infrastructure, the CPU restatement) renders C3 with its
  segment log on (every path segment: ray, check[] mask);
* the positions of shade pass k are the rays of segment k in binned order:
  sorted by their check[] set, then by the earlier segments' sets (the
  scatter keeps a bin's slots in their previous order), then by path;
* 64 consecutive positions form a wave; its lanes are the positions whose
  path goes on, each testing the NEXT segment's ray (the one bounds() is
  computed for);
* for every (wave, top-level union with >= 2 boxes) pair: does any lane's
  ray hit the union's enclosing box (the f32 min / max of its boxes)?

Reported: the fraction of (wave, union) pairs no lane hits, and the box
tests that would be skipped net of the enclosing tests themselves, as a
fraction of all box tests.  Threshold: build the skip if the
pair fraction is >= 25 %.

    python scripts/union_box_skip.py [width height spp] > profiles/r06_union_box_skip.json
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from compute_path_tracer_amd import scenes  # noqa: E402
from compute_path_tracer_amd.sdf_editor import CompData  # noqa: E402
from oracle import oracle as O  # noqa: E402  (test infrastructure: the CPU restatement)


class Segment(ctypes.Structure):  # pt_oracle.h pto_segment
    _fields_ = [("ro", ctypes.c_float * 3), ("rd", ctypes.c_float * 3), ("mask", ctypes.c_uint64 * 2),
                ("seg", ctypes.c_int32), ("steps", ctypes.c_int32), ("hit", ctypes.c_int32), ("pad", ctypes.c_int32)]


def boxes_by_union(prog) -> tuple:
    """(lo[n,3], hi[n,3], union index per box): the scene's boxes as the
    oracle's bounds() forms them (pt_oracle.c bounds_ct: centre = union
    position + shape position, half size = so * (union scale * shape scale)
    * exaggeration) and the top-level union each belongs to."""
    d = prog.data.astype(np.float32)
    ops = prog.op_dicts()
    top_of_check, depth, top = {}, 0, -1
    for o in ops:
        if o["opcode"] == 0:  # union begin
            if depth == 0:
                top += 1
            depth += 1
        elif o["opcode"] == 2:
            depth -= 1
        elif o["check"] >= 0:
            top_of_check[o["check"]] = top
    lo, hi, uni = [], [], []
    for a in prog.aabb_dicts():
        c = np.array([d[a["union_position"][i]] + d[a["shape_position"][i]] for i in range(3)], np.float32)
        if a["so_kind"] == 0:
            so = np.full(3, d[a["size"][0]], np.float32)
        elif a["so_kind"] == 1:
            so = np.array([d[a["size"][i]] for i in range(3)], np.float32)
        elif a["so_kind"] == 3:
            R, r = d[a["size"][0]], d[a["size"][1]]
            so = np.array([R + r, r, R + r], np.float32)
        else:
            so = np.ones(3, np.float32)
        sc = np.float32(d[a["union_scale"]] * d[a["shape_scale"]])
        hs = (so * sc) * np.float32(d[a["aabb_exaggeration"]])
        lo.append(c - hs)
        hi.append(c + hs)
        uni.append(top_of_check[a["back"]])
    return np.array(lo, np.float32), np.array(hi, np.float32), np.array(uni)


def hits(lo, hi, ro, rd) -> np.ndarray:
    """aabb.glsl's slab test of every ray against one box, f32 (bool[n])."""
    with np.errstate(divide="ignore", invalid="ignore"):
        t0 = (lo[None, :] - ro) / rd
        t1 = (hi[None, :] - ro) / rd
    tn = np.fmax.reduce(np.fmin(t0, t1), axis=1)
    tf = np.fmin.reduce(np.fmax(t0, t1), axis=1)
    return (tn < tf) & (tf > 0)


def main() -> None:
    w, h, spp = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (192, 108, 16)
    ed = scenes.SCENES["c3"]()
    prog = ed.compile(CompData())
    lo, hi, uni = boxes_by_union(prog)
    unions = sorted(set(uni.tolist()))
    osc = O.OracleScene(ed.rows())
    cap = w * h * spp * 10
    log = (Segment * cap)()
    L = O.lib()
    L.pto_set_segment_log(log, cap)
    bounces = 8
    osc.render(w, h, O.Constants(0.0, 1, float(np.float32(w) / np.float32(h)), 1), O.Settings(0, bounces, 1.0, 1.0, 0),
               spp, threads=1, counters=True)
    n = L.pto_segment_log_count()
    L.pto_set_segment_log(None, 0)
    arr = np.ctypeslib.as_array(log)[:n]
    seg = arr["seg"].astype(np.int64)
    ro = np.stack([arr["ro"][:, i] for i in range(3)], 1).astype(np.float32)
    rd = np.stack([arr["rd"][:, i] for i in range(3)], 1).astype(np.float32)
    mask = arr["mask"][:, 0].astype(np.uint64)
    # paths: the log is path after path, segments in order (seg 0 starts one)
    path = np.cumsum(seg == 0) - 1
    nxt = np.full(n, -1, np.int64)  # the next segment of the same path
    cont = (np.arange(n - 1) + 1 < n) & (seg[1:] == seg[:-1] + 1)
    nxt[:-1][cont] = np.arange(1, n)[cont]
    # the sets of the path's earlier segments (sort keys after its own)
    prev = [np.zeros(n, np.uint64) for _ in range(bounces + 1)]
    for j in range(1, bounces + 1):  # prev[j][i] = mask of segment seg[i] - j of the same path (0 if none)
        src = np.arange(n) - j
        ok = (src >= 0) & (seg - j >= 0)
        prev[j][ok] = mask[src[ok]]
    per_union = {u: int(np.count_nonzero(uni == u)) for u in unions}
    multi = [u for u in unions if per_union[u] >= 2]
    pairs = skipped_pairs = 0
    box_tests = skipped_boxes = enclosing_tests = 0
    waves = lanes_total = 0
    by_union = {u: [0, 0] for u in multi}
    for k in range(bounces):  # shade pass k computes bounds() of segment k + 1
        pos = np.nonzero(seg == k)[0]
        keys = [path[pos]] + [prev[j][pos] for j in range(k, 0, -1)] + [mask[pos]]
        order = pos[np.lexsort(keys)]  # last key primary: this segment's set, then earlier sets, then path
        for w0 in range(0, len(order), 64):
            win = order[w0:w0 + 64]
            nx = nxt[win]
            nx = nx[nx >= 0]
            if len(nx) == 0:
                continue
            waves += 1
            lanes_total += len(nx)
            box_tests += len(lo)
            for u in multi:
                sel = uni == u
                elo, ehi = lo[sel].min(0), hi[sel].max(0)
                hit = hits(elo, ehi, ro[nx], rd[nx]).any()
                pairs += 1
                enclosing_tests += 1
                by_union[u][0] += 1
                if not hit:
                    skipped_pairs += 1
                    skipped_boxes += per_union[u]
                    by_union[u][1] += 1
    out = {"scene": "c3", "width": w, "height": h, "spp": spp, "bounces": bounces, "segments_logged": int(n),
           "paths": int(path[-1] + 1), "shade_waves": waves, "lanes_per_wave": round(lanes_total / max(1, waves), 2),
           "boxes": int(len(lo)), "top_level_unions": len(unions), "unions_with_2plus_boxes": len(multi),
           "boxes_per_union": {str(u): per_union[u] for u in unions},
           "wave_union_pairs": pairs, "pairs_no_lane_hits": skipped_pairs,
           "pair_fraction_skippable": round(skipped_pairs / max(1, pairs), 4),
           "per_union_fraction_skippable": {str(u): round(v[1] / max(1, v[0]), 4) for u, v in by_union.items()},
           "box_tests": box_tests, "box_tests_skipped": skipped_boxes, "enclosing_tests_added": enclosing_tests,
           "net_box_test_fraction_saved": round((skipped_boxes - enclosing_tests) / max(1, box_tests), 4),
           "threshold": "build the skip if pair_fraction_skippable >= 0.25 (VERDICT r05 item 2)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
