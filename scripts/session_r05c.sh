#!/bin/bash
# Round 5: 2^11-bin histogram + shade quad prefetch (PT_SHADE_PF=2) A/B
# against the round-4 tree, three alternating pairs; parity subset first.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
(cd ab/b11 && timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py -k "binned or full_size or bounce_range or progressive or wide or cull" > "$R/gpurun_out/r05c_pytest_b11.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05c_pytest_b11.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 \
  bash scripts/ab_trees.sh ab/r04 ab/b11 "ab/b11@PT_JIT_DEFS=PT_SHADE_PF=0"
