#!/usr/bin/env python3
"""Instruction budget of a scene kernel: the static
instruction mix of one kernel of a scripts/jit_isa.py dump, by class, and --
given a one-pipeline PMC summary (profiles/*_pmc.json with SQ_INSTS_VALU,
the SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F32, INT32, INT64, CVT counters and
the stats counters' wave_maps) -- the dynamic VALU mix per wave-level map()
evaluation: FP32 arithmetic, transcendental, integer, conversion and the
rest (compares, selects, min/max, moves: the counters do not split them;
the static mix of the kernel's code apportions that rest).

    python scripts/isa_budget.py /tmp/jit_isa/c3.s pt_bin_trace_m_jit [pmc.json wave_maps_per_launch]
"""
from __future__ import annotations

import json
import re
import sys
from collections import Counter

CLASSES = [
    ("fp32", r"^v_(add|sub|subrev|mul|fma|fmac|mac|madak|madmk|fmaak|fmamk)_f32"),
    ("minmax", r"^v_(max|min|max3|min3|med3)_f32"),
    ("cmp", r"^v_cmpx?_"),
    ("select", r"^v_cndmask_b32"),
    ("trans", r"^v_(sqrt|rsq|rcp|exp|log|sin|cos)_f32"),
    ("div", r"^v_(div_scale|div_fmas|div_fixup|frexp|ldexp)"),
    ("cvt", r"^v_cvt_"),
    ("move", r"^v_(mov|readfirstlane|readlane|writelane)_b(32|64)|_dpp$"),
    ("int", r"^v_(add|sub|subrev|and|or|xor|not|lshl|lshr|ashr|bfe|bfi|mul_lo|mul_hi|min|max|lshl_add|lshl_or|"
            r"add3|or3|and_or|xad|sad|mbcnt|bcnt|alignbit|perm|bfm|ffbh|ffbl|cndmask)_"),
    ("valu_other", r"^v_"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc)"),
    ("nop", r"^s_nop"),
    ("wait", r"^s_waitcnt"),
    ("smem", r"^s_(load|buffer_load|store|dcache)"),
    ("salu", r"^s_"),
    ("lds", r"^ds_"),
    ("vmem", r"^(global|buffer|flat|scratch)_"),
]


def kernel_lines(path: str, name: str) -> list:
    out, on = [], False
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            on = m.group(1) == name
            continue
        if on and line.startswith("\t"):
            out.append(line.split()[0])
    return out


def classify(ops: list) -> Counter:
    c = Counter()
    for op in ops:
        op = re.sub(r"_e(32|64)$", "", op)
        for cls, pat in CLASSES:
            if re.search(pat, op):
                c[cls] += 1
                break
        else:
            c["other"] += 1
    return c


VALU_CLASSES = ("fp32", "minmax", "cmp", "select", "trans", "div", "cvt", "move", "int", "valu_other")


def main() -> None:
    path, name = sys.argv[1], sys.argv[2]
    ops = kernel_lines(path, name)
    st = classify(ops)
    valu = sum(st[k] for k in VALU_CLASSES)
    print(f"{name}: {len(ops)} instructions, {valu} VALU (static)")
    for k, v in st.most_common():
        print(f"  {k:11s} {v:6d}  {v / max(1, valu):6.3f} of VALU" if k in VALU_CLASSES else f"  {k:11s} {v:6d}")
    if len(sys.argv) > 4:
        pmc = json.load(open(sys.argv[3]))
        maps = float(sys.argv[4])
        hot = pmc.get("kernel") or {}
        if hot.get("kernel") != name:
            raise SystemExit(f"{sys.argv[3]} holds raw counters for {hot.get('kernel')}, not {name}")
        c = pmc["per_launch_counters"]
        per = {k: c[k] / maps for k in c if k.startswith("SQ_INSTS")}
        v = per.get("SQ_INSTS_VALU", 0.0)
        known = {k.replace("SQ_INSTS_VALU_", "").lower(): per.get(k, 0.0) for k in
                 ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
                  "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT")}
        rest = v - sum(known.values())
        print(f"dynamic, per wave-level map(): VALU {v:.1f}, SALU {per.get('SQ_INSTS_SALU', 0):.1f}")
        for k, x in known.items():
            print(f"  {k:10s} {x:7.1f}  {x / v:6.3f}")
        srest = sum(st[k] for k in ("minmax", "cmp", "select", "move", "div", "valu_other"))
        print(f"  rest       {rest:7.1f}  {rest / v:6.3f}   (static split of the rest:)")
        for k in ("cmp", "select", "minmax", "move", "div", "valu_other"):
            print(f"    {k:10s} {rest * st[k] / max(1, srest):7.1f}")


if __name__ == "__main__":
    main()
