#!/bin/bash
# PT_JIT_SUBCUT A/B: parity subset with the cut on (the default), then bench pairs against it off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "binned_jit or jit or full_size or work_counters" > gpurun_out/subcut_pytest.log 2>&1
rc=$?; echo "subcut parity rc=$rc"; tail -3 gpurun_out/subcut_pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=4 AB_VARIANTS="PT_JIT=1;PT_JIT_SUBCUT=0;PT_JIT=1;PT_JIT_SUBCUT=0;PT_BIN_LANES=1;PT_BIN_LANES=1 PT_JIT_SUBCUT=0" bash scripts/ab_kernels.sh
