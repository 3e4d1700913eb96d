#!/bin/bash
# Round 5: one-pipeline rocprofv3 kernel traces of the first pass with and
# without the primary box skip (ab/base, ab/skip, ab/skip with the fused DPP
# reductions), to see pt_bin_trace_g_jit's own time.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export GPU_OUT="$R/gpurun_out"; mkdir -p "$GPU_OUT"
GRAFT_REPO_ROOT="$R/ab/base" PROF_TAG=r05i_base PROF_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --pipelines 1" \
  bash "$R/scripts/profile.sh" || exit $?
GRAFT_REPO_ROOT="$R/ab/skip" PROF_TAG=r05i_skip PROF_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --pipelines 1" \
  bash "$R/scripts/profile.sh" || exit $?
PT_JIT_DEFS=PT_WRED_DPP_ASM GRAFT_REPO_ROOT="$R/ab/skip" PROF_TAG=r05i_skipasm \
  PROF_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --pipelines 1" bash "$R/scripts/profile.sh" || exit $?
for t in base skip skipasm; do echo "== $t"; grep -E "trace_g_jit|trace_m_jit\"|shade_t_jit\"" "$GPU_OUT/prof_r05i_$t/kt/kt_kernel_stats.csv" | cut -c1-160; done
