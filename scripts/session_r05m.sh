#!/bin/bash
# Round 5: bins from a table of check[] sets -- GPU parity
# cases on the frozen tree ab/btab, then alternating benches against ab/base
# (the tree before it).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
(cd ab/btab && timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py -k "binned or c3 or wide or cull or full_size" > "$R/gpurun_out/r05m_pytest_btab.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05m_pytest_btab.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/base ab/btab
