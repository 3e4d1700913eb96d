#!/bin/bash
# Round 5: shade-pass quad prefetch A/B.  Parity of the
# frozen tree's binned kernels first, then alternating benches of the round-4
# tree, the prefetch tree (PT_SHADE_PF=2, default) and its PF=0 variant.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
(cd ab/pf && timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py tests/test_gpu_multirank.py::test_one_gpu_validate_and_tile_check -k "binned or full_size or bounce_range or progressive or one_gpu" > "$R/gpurun_out/r05b_pytest_pf.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r05b_pytest_pf.log; [ $rc -eq 0 ] || exit $rc
AB_PAIRS=2 AB_STEPS=10 AB_WARMUP=2 \
  bash scripts/ab_trees.sh ab/r04 ab/pf "ab/pf@PT_JIT_DEFS=PT_SHADE_PF=0"
