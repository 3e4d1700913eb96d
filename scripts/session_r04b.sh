#!/bin/bash
# Round 4 measurement call on the frozen tree ab/r04b: the driver-form bench,
# a one-pipeline rocprofv3 kernel trace + PMC passes (per-kernel counters for
# the roofline), the default two-pipeline kernel trace, every BASELINE config.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-r04b}"; T=${TAG:-r04b}
export GPU_OUT="$R/gpurun_out"
mkdir -p "$GPU_OUT"
(cd "$D" && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$GPU_OUT/${T}_bench.log" 2>&1)
rc=$?; echo "bench rc=$rc"; tail -c 400 "$GPU_OUT/${T}_bench.log"; [ $rc -eq 0 ] || exit $rc
# FP32 op counters for a measured flop rate, when this rocprofv3 lists them
(cd /tmp && timeout -k 10 120 rocprofv3 -L > "$GPU_OUT/${T}_counters.txt" 2>&1)
F32="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"
EXTRA=""
if grep -q SQ_INSTS_VALU_FMA_F32 "$GPU_OUT/${T}_counters.txt" && grep -q SQ_INSTS_VALU_ADD_F32 "$GPU_OUT/${T}_counters.txt" \
   && grep -q SQ_INSTS_VALU_MUL_F32 "$GPU_OUT/${T}_counters.txt" && grep -q SQ_INSTS_VALU_TRANS_F32 "$GPU_OUT/${T}_counters.txt"; then
  EXTRA=";$F32"
fi
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l1 PROF_ARGS="--steps 4 --warmup 1 --no-cpu-baseline --pipelines 1" \
  PMC_ARGS="--pipelines 1" \
  PMC_PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY;FETCH_SIZE;WRITE_SIZE$EXTRA" \
  bash "$R/scripts/profile.sh" pmc || exit $?
GRAFT_REPO_ROOT="$D" PROF_TAG=${T}_l2 bash "$R/scripts/profile.sh" || exit $?
(cd "$D" && timeout -k 10 600 python scripts/configs.py > "$GPU_OUT/${T}_configs.jsonl" 2> "$GPU_OUT/${T}_configs.err")
rc=$?; echo "configs rc=$rc"; cat "$GPU_OUT/${T}_configs.jsonl" | cut -c1-200
exit $rc
