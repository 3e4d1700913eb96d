#!/bin/bash
# Round 5: the set table's first probe issued before the ray's stores and a
# fast return for a set found in its hash slot (ab/bp), and
# on top the shade pass's hit quad in one load (ab/hq) -- GPU parity cases
# on ab/hq, then alternating benches of ab/r05n, ab/bp and ab/hq.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
T=hq; [ -d ab/hq ] || T=bp
(cd ab/$T && timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py -k "bin_table or binned_lanes or sub_chunks or (parity_path_trace and binned)" \
   > "$R/gpurun_out/r05o_pytest_$T.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05o_pytest_$T.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
if [ -d ab/hq ]; then
  AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/r05n ab/bp ab/hq
else
  AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/r05n ab/bp
fi
