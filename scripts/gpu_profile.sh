#!/bin/bash
# One profiling session on a tree (the repo, or a frozen copy ab/<TREE>):
# a one-pipeline rocprofv3 kernel trace + the PMC passes (each kernel's
# counters its own: VALU issue and lane use, waits, FETCH/WRITE_SIZE, the
# FP32 / INT / CVT instruction mix), the default two-pipeline kernel trace,
# optionally every BASELINE config (scripts/configs.py) and a bench.
# Outputs gpurun_out/prof_<TAG>_l1, prof_<TAG>_l2 (scripts/summarize_profile.py
# turns them into profiles/<TAG>_l{1,2}_*), <TAG>_configs.jsonl, <TAG>_bench.log.
#   TAG=r06d [TREE=final] [CONFIGS=1] [BENCH=1] bash scripts/gpu_profile.sh
# (replaces round 4-5's one-off session_r0*.sh profiling scripts)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R"; [ -n "${TREE:-}" ] && D="$R/ab/$TREE"
T=${TAG:?TAG}
export GPU_OUT="$R/gpurun_out"
mkdir -p "$GPU_OUT"
MIX="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l1 PROF_ARGS="--steps 4 --warmup 1 --no-cpu-baseline --pipelines 1" \
  PMC_ARGS="--pipelines 1" \
  PMC_PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY;FETCH_SIZE;WRITE_SIZE;$MIX" \
  bash "$R/scripts/profile.sh" pmc || exit $?
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l2 bash "$R/scripts/profile.sh" || exit $?
if [ "${CONFIGS:-0}" = 1 ]; then
  (cd "$D" && timeout -k 10 600 python scripts/configs.py > "$GPU_OUT/${T}_configs.jsonl" 2> "$GPU_OUT/${T}_configs.err")
  rc=$?; echo "configs rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  (cd "$D" && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$GPU_OUT/${T}_bench.log" 2>&1)
  rc=$?; echo "bench rc=$rc"; python "$R/scripts/parse_bench.py" "$GPU_OUT/${T}_bench.log" | cut -c1-200; exit $rc
fi
