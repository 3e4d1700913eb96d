#!/bin/bash
# Bench with and without torch imported before the library: a torch-first
# process (every GPU test, bench.py at N > 1) compiles the scene kernels with
# torch's bundled hipRTC / comgr; jit.*_vgprs shows the build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for first in none torch none torch; do
  if [ $first = torch ]; then
    timeout -k 10 300 python -c "import torch, runpy, sys; sys.argv=['bench.py','--steps','4','--warmup','1','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab.tmp 2>&1
  else
    timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab.tmp 2>&1
  fi
  rc=$?
  v=$(python -c "import json;d=json.loads([l for l in open('gpurun_out/ab.tmp') if l.startswith('{')][-1]);print(d['jit'])" 2>/dev/null)
  echo "first=$first rc=$rc $(python scripts/parse_bench.py gpurun_out/ab.tmp 2>/dev/null | cut -c1-90) $v" | tee -a gpurun_out/ab_torchfirst.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/ab.tmp; exit $rc; }
done
