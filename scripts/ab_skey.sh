#!/bin/bash
# PT_SPATIAL_KEY A/B: parity subset with the spatial order on, then bench pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PT_SPATIAL_KEY=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "binned and (path_trace or bounce_range or lanes or sub_chunks) or full_size" \
  > gpurun_out/skey_pytest.log 2>&1
rc=$?; echo "skey parity rc=$rc"; tail -3 gpurun_out/skey_pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=4 AB_VARIANTS="PT_JIT=1;PT_SPATIAL_KEY=1;PT_SPATIAL_KEY=2;PT_JIT=1;PT_SPATIAL_KEY=1;PT_SPATIAL_KEY=2;PT_BIN_LANES=1;PT_BIN_LANES=1 PT_SPATIAL_KEY=2" bash scripts/ab_kernels.sh
