#!/bin/bash
# Round 5: the first pass writes no ray records; shade pass 0 makes each
# traced camera ray again (gen_norec) -- the GPU parity suite on ab/norec,
# then alternating benches against ab/hq.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
(cd ab/norec && timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
   tests/test_gpu_parity.py > "$R/gpurun_out/r05q_pytest_norec.log" 2>&1)
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05q_pytest_norec.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/hq ab/norec
