#!/bin/bash
# Round 5: the first pass frame-fastest (a window = one pixel over 64 frames)
# -- the GPU parity suite on ab/pix, then alternating benches against ab/base
# (HEAD before it).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
(cd ab/${T:-pix} && timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py > "$R/gpurun_out/r05z_pytest_${T:-pix}.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05z_pytest_${T:-pix}.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ${BASE:-ab/base} ab/${T:-pix}
