#!/usr/bin/env python3
"""Per-kernel, per-launch averages of every counter in rocprofv3 --pmc CSV
runs (the *_counter_collection.csv under each directory given), for the
binned pipeline's kernels; derived ratios for the shade / march kernels
where the counters are present.
    python scripts/pmc_kernels.py gpurun_out/prof_r05x/pmc1 gpurun_out/prof_r05x/pmc2 ...
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("pt_bin_shade_t_jit", "pt_bin_trace_m_jit", "pt_bin_trace_g_jit", "pt_bin_scatter_kernel")


def main(dirs) -> None:
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                name = next((n for n in KERNELS if k.startswith(n) and not k.startswith(n + "_stats")), None)
                if name is None:
                    continue
                tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name][r["Counter_Name"]].add(r["Dispatch_Id"])
    out = {}
    for k, cs in tot.items():
        per = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
        der = {}
        g = per.get
        if g("SQ_INSTS_VALU"):
            for c in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS"):
                if g(c) is not None:
                    der[c.lower() + "_per_valu"] = g(c) / g("SQ_INSTS_VALU")
        if g("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT"):
                if g(c) is not None:
                    der[c.lower() + "_frac_of_wave_cycles"] = g(c) / g("SQ_WAVE_CYCLES")
        if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
            der["l2_hit_rate"] = g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
        if g("TCP_TOTAL_CACHE_ACCESSES_sum") and g("TCP_TCC_READ_REQ_sum") is not None:
            der["l1_read_miss_to_l2_per_access"] = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum")
        out[k] = {"per_launch": per, "derived": der, "launches": max(len(s) for s in disp[k].values())}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1:])
