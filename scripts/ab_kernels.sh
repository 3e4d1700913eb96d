#!/bin/bash
# A/B of kernel variants on the bench workload, one process per variant.
# Variants: env-var sets separated by ";" in AB_VARIANTS (the hook for
# experiments on the scene kernels is PT_JIT_DEFS; a whole built tree: ab_trees.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=";" read -ra VARS <<< "${AB_VARIANTS:-PT_JIT_DEFS=;PT_JIT_DEFS=}"
for v in "${VARS[@]}"; do
  env $v timeout -k 10 300 python bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/ab.tmp 2>&1
  rc=$?
  echo "$v rc=$rc $(python scripts/parse_bench.py gpurun_out/ab.tmp 2>/dev/null)" | tee -a gpurun_out/ab.log
  if [ $rc -ne 0 ]; then cat gpurun_out/ab.tmp; exit $rc; fi
done
