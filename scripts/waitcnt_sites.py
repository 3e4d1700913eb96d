#!/usr/bin/env python3
"""Where a scene kernel waits on vector memory: every
`s_waitcnt vmcnt(N)` of one kernel, with the source line it sits at and the
vector-memory operations it drains.

gfx950 (gfx9) retires vector loads AND stores through the one in-order
`vmcnt` counter, so `vmcnt(N)` waits until at most the N most recently
issued vector-memory operations are still outstanding: every older load,
store and atomic must have completed.  This walks the kernel's code
backwards in address order from each wait (a static, straight-line view:
across a branch target it lists what precedes in address order) and names
the operations older than the N youngest, up to the previous full drain.

Input: a disassembly with source lines (llvm-objdump -d -l) of the scene
kernels compiled from their dumped source with line tables:

    PT_JIT_BAKE=1 python scripts/jit_isa.py c3 /tmp/jit_isa_b
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \\
        -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize \\
        -gline-tables-only --cuda-device-only --no-gpu-bundle-output -c \\
        -Icompute_path_tracer_amd/csrc -Iinclude -x hip /tmp/jit_isa_b/c3.hip -o c3g.co
    llvm-objdump -d -l --mcpu=gfx950 c3g.co > c3g.s
    python scripts/waitcnt_sites.py c3g.s pt_bin_shade_t_jit [--json out.json]
"""
from __future__ import annotations

import json
import os
import re
import sys

VMEM = re.compile(r"^(global|buffer|flat|scratch)_(load|store|atomic)\w*")
WAIT = re.compile(r"^s_waitcnt\b.*\bvmcnt\((\d+)\)")


def parse(path: str, kernel: str) -> list:
    """[(addr, op, text, src)] of `kernel`, src = the last '; file:line'."""
    out, on, src = [], False, "?"
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            on = m.group(1) == kernel
            continue
        if not on:
            continue
        if line.startswith("; ") and ":" in line:
            f, _, ln = line[2:].strip().rpartition(":")
            if ln.isdigit():
                src = f"{os.path.basename(f)}:{ln}"
            continue
        if line.startswith("\t"):
            text = line.strip().split("//")[0].strip()
            am = re.search(r"//\s*([0-9A-F]+):", line)
            out.append((int(am.group(1), 16) if am else 0, text.split()[0], text, src))
    return out


def kind(op: str) -> str:
    m = VMEM.match(op)
    if not m:
        return ""
    return {"load": "load", "store": "store", "atomic": "atomic"}[m.group(2)]


def sites(ins: list, window: int = 48) -> list:
    res = []
    for i, (addr, op, text, src) in enumerate(ins):
        m = WAIT.match(text)
        if not m:
            continue
        n = int(m.group(1))
        older = []  # vmem ops before the wait, youngest first
        for j in range(i - 1, max(-1, i - 4000), -1):
            a2, op2, t2, s2 = ins[j]
            m2 = WAIT.match(t2)
            if m2 and int(m2.group(1)) == 0:
                break  # everything before a full drain has completed
            k = kind(op2)
            if k:
                older.append((a2, k, op2, s2))
                if len(older) >= window:
                    break
        drained = older[n:]
        res.append({"addr": hex(addr), "wait": text, "src": src, "vmcnt": n,
                    "outstanding_kept": [f"{k} {o} @{s}" for _, k, o, s in older[:n]],
                    "drained": [f"{k} {o} @{s}" for _, k, o, s in drained],
                    "drained_stores": sum(1 for _, k, _, _ in drained if k in ("store", "atomic"))})
    return res


def main() -> None:
    path, kernel = sys.argv[1], sys.argv[2]
    ins = parse(path, kernel)
    res = sites(ins)
    vm = [(hex(a), kind(o), o, s) for a, o, _, s in ins if kind(o)]
    print(f"{kernel}: {len(ins)} instructions, {len(vm)} vector-memory ops, {len(res)} vmcnt waits")
    print("vector-memory ops (address order):")
    for a, k, o, s in vm:
        print(f"  {a} {k:6s} {o:28s} {s}")
    print("vmcnt waits:")
    for r in res:
        print(f"  {r['addr']} {r['wait']:40s} at {r['src']}: drains {len(r['drained'])} "
              f"({r['drained_stores']} stores/atomics)")
        for d in r["drained"][:8]:
            print(f"      {d}")
    if "--json" in sys.argv:
        json.dump({"kernel": kernel, "vmem_ops": [list(v) for v in vm], "waits": res},
                  open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
