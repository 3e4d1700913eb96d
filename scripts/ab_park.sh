#!/bin/bash
# PT_PARK_EARLY A/B: parity subset with the variant, then bench pairs (+ grid sweeps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V="PT_JIT_DEFS=PT_PARK_EARLY=${PARK:-1}"
env $V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "binned_jit and (path_trace or bounce_range or debug_views or lanes) or full_size or binned_tier" \
  > gpurun_out/park_pytest.log 2>&1
rc=$?; echo "park parity rc=$rc"; tail -3 gpurun_out/park_pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=4 AB_VARIANTS="PT_JIT=1;$V;PT_JIT=1;$V;PT_BIN_LANES=1;PT_BIN_LANES=1 $V" bash scripts/ab_kernels.sh
