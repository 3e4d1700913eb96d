#!/bin/bash
# Round 5 final-tree check on the frozen tree ab/<TREE>: the whole GPU suite,
# smoke, and the driver-form bench (steps 20, warmup 5).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
T=${TAG:-r05d}; D="$R/ab/${TREE:-r05d}"
mkdir -p "$R/gpurun_out"
cd "$D"
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
  > "$R/gpurun_out/${T}_pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$R/gpurun_out/${T}_pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > "$R/gpurun_out/${T}_smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$R/gpurun_out/${T}_smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$R/gpurun_out/${T}_bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 "$R/gpurun_out/${T}_bench.log"
exit $rc
