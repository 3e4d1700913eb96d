#!/bin/bash
# One A/B session: optionally the GPU parity suite on the candidate (a
# frozen tree ab/<X>, or the repo with PT_JIT_DEFS for a scene-kernel knob),
# then alternating benches of the candidates on one box (scripts/ab_trees.sh:
# a tree, optionally with environment settings, "ab/x" or ".@PT_JIT_DEFS=A").
# The log lands in gpurun_out/<TAG>_ab.log (and the parity log in
# gpurun_out/<TAG>_pytest.log).
#   TAG=r06x [PARITY=ab/x | PARITY=.@PT_JIT_DEFS=A] [PAIRS=3] [STEPS=10] \
#     [ARGS="--no-tile-check --no-table-kernel"] bash scripts/gpu_ab.sh base cand...
# (replaces round 5's one-off session_r05*.sh A/B scripts)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
T=${TAG:?TAG}
export PT_JIT_CACHE=${PT_JIT_CACHE:-2}  # (a knob's scene kernels compile once per box)
if [ -n "${PARITY:-}" ]; then
  t=${PARITY%%@*}; envs=""; [ "$t" != "$PARITY" ] && envs=${PARITY#*@}
  (cd "$R/$t" && env $envs timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 \
     --timeout-method thread -m gpu tests/test_gpu_parity.py > "$R/gpurun_out/${T}_pytest.log" 2>&1)
  rc=$?; echo "pytest rc=$rc"; tail -3 "gpurun_out/${T}_pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
rm -f gpurun_out/ab_trees.log
AB_PAIRS=${PAIRS:-3} AB_STEPS=${STEPS:-10} AB_WARMUP=2 AB_ARGS="${ARGS:---no-tile-check --no-table-kernel}" \
  timeout -k 10 1000 bash scripts/ab_trees.sh "$@"
rc=$?; cp gpurun_out/ab_trees.log "gpurun_out/${T}_ab.log"; exit $rc
