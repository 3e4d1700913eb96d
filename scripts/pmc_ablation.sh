#!/bin/bash
# VALU instruction counts per kernel launch under timing ablations (PT_JIT_DEFS
# variants, wrong images): the first shade pass sees the same hits either way,
# so its count difference is the ablated part's cost.  Usage:
#   ABL="BASE PT_EXP_NOBOUNDS" bash scripts/pmc_ablation.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in ${ABL:-BASE PT_EXP_NOBOUNDS}; do
  if [ "$v" = BASE ]; then D=""; else D=$v; fi
  PT_BIN_LANES=1 PT_JIT_DEFS=$D timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --kernel-trace \
    -d "$R/gpurun_out/pmcabl_$v" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > "$R/gpurun_out/pmcabl_$v.log" 2>&1 || exit 1
  echo "$v ok"
done
