#!/bin/bash
# torch-first bench with the spilling 8-wave build forced (PT_JIT_*_WAVES=8: no fallback)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "PT_JIT=1" "PT_JIT_TRACE_WAVES=8 PT_JIT_SHADE_WAVES=8" "PT_JIT=1" "PT_JIT_TRACE_WAVES=8 PT_JIT_SHADE_WAVES=8"; do
  env $v timeout -k 10 300 python -c "import torch, runpy, sys; sys.argv=['bench.py','--steps','4','--warmup','1','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab.tmp 2>&1
  rc=$?
  j=$(python -c "import json;d=json.loads([l for l in open('gpurun_out/ab.tmp') if l.startswith('{')][-1]);print(d['jit'])" 2>/dev/null)
  echo "torch-first $v rc=$rc $(python scripts/parse_bench.py gpurun_out/ab.tmp 2>/dev/null | cut -c1-90) $j" | tee -a gpurun_out/ab_torchwaves.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/ab.tmp; exit $rc; }
done
