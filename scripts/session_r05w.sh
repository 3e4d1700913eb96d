#!/bin/bash
# Round 5: knob re-check on the final kernels -- the tapping shade pass at 16
# blocks per CU (ab/s16) against 14 (ab/final), and three pipelines.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
rm -f gpurun_out/ab_trees.log
AB_PAIRS=3 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel" bash scripts/ab_trees.sh ab/final ab/s16 || exit $?
cp gpurun_out/ab_trees.log gpurun_out/r05w_ab_shade16.log
rm -f gpurun_out/ab_trees.log
AB_PAIRS=2 AB_STEPS=10 AB_WARMUP=2 AB_ARGS="--no-tile-check --no-table-kernel --pipelines 3" bash scripts/ab_trees.sh ab/final
cp gpurun_out/ab_trees.log gpurun_out/r05w_pipelines3.log
