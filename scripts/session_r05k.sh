#!/bin/bash
# Round 5 final-tree profiles + driver-form bench of the frozen tree ab/<TREE>: a one-pipeline rocprofv3
# kernel trace + PMC passes (the round-4 set plus the VALU instruction mix
# for the trace kernel's budget), then the default
# two-pipeline kernel trace.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-r05k}"; T=${TAG:-r05k}
export GPU_OUT="$R/gpurun_out"
mkdir -p "$GPU_OUT"
MIX="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l1 PROF_ARGS="--steps 4 --warmup 1 --no-cpu-baseline --pipelines 1" \
  PMC_ARGS="--pipelines 1" \
  PMC_PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY;FETCH_SIZE;WRITE_SIZE;$MIX" \
  bash "$R/scripts/profile.sh" pmc || exit $?
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l2 bash "$R/scripts/profile.sh" || exit $?
(cd "$D" && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$GPU_OUT/${T}_bench.log" 2>&1)
rc=$?; echo "bench rc=$rc"; python "$R/scripts/parse_bench.py" "$GPU_OUT/${T}_bench.log" | cut -c1-200; exit $rc
