#!/bin/bash
# Bench with torch imported before the library (as every GPU test and bench.py
# at N > 1 do): PT_JIT_ISOLATE=0 compiles the scene kernels with whatever
# hipRTC the process holds (torch's bundled copy), 1 (default) with the image's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for iso in 0 1 0 1; do
  PT_JIT_ISOLATE=$iso timeout -k 10 300 python -c "import torch, runpy, sys; sys.argv=['bench.py','--steps','4','--warmup','1','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab.tmp 2>&1
  rc=$?
  echo "torch-first PT_JIT_ISOLATE=$iso rc=$rc $(python scripts/parse_bench.py gpurun_out/ab.tmp 2>/dev/null | cut -c1-90)" | tee -a gpurun_out/ab_torchfirst.log
  [ $rc -eq 0 ] || { tail -20 gpurun_out/ab.tmp; exit $rc; }
done
