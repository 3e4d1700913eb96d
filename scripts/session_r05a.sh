#!/bin/bash
# Round 5, first GPU call: the new GPU tests (C harness render, self-checking
# multi-rank lines, one-GPU --validate), smoke, then the driver-form bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r05a}
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -m gpu \
  tests/test_abi_harness.py tests/test_gpu_multirank.py > gpurun_out/${T}_pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${T}_pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${T}_bench.log
exit $rc
