#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench; outputs gpurun_out/<tag>_*.
# Stops at the first step that crashes or times out (pytest's failure code 1
# is a test result, not a crash: the session goes on).
#   scripts/gpu_session.sh <tag> [pytest args...]   (BENCH_ARGS env: bench flags)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}; shift || true
O=${GPU_OUT:-gpurun_out}  # (a frozen copy's session writes to the repo's gpurun_out)
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 \
    --timeout-method thread "$@" > $O/${tag}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/${tag}_pytest_gpu.log | tail -25
  ok $rc || exit $rc
fi
if [ "${SKIP_SMOKE:-0}" != 1 ]; then
  timeout -k 10 180 python __graft_entry__.py > $O/${tag}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 $O/${tag}_smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > $O/${tag}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 600 $O/${tag}_bench.log
  exit $rc
fi
