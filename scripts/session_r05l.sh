#!/bin/bash
# Round 5: the first pass's box-skip edge cases (fov, windows across the image centre).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R/ab/r05l"; mkdir -p "$R/gpurun_out"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "box_skip_edges or full_size or parity_path_trace" > "$R/gpurun_out/r05l_pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$R/gpurun_out/r05l_pytest.log"; exit $rc
