#!/bin/bash
# Round 5: the first pass's wave-level box skip -- the whole
# GPU suite on the frozen tree ab/skip, then alternating benches against the
# tree without it (ab/base = the commit before).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
(cd ab/skip && timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests > "$R/gpurun_out/${TAG:-r05h}_pytest_skip.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG:-r05h}_pytest_skip.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/base ab/skip
