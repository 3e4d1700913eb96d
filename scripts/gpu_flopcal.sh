#!/bin/bash
# The PMC pass of scripts/flop_calib.py: FP32 instruction counts of every
# scene-kernel dispatch of its configurations (MODE sweep: C3 over bounce
# counts x fields of view; scenes: eight scenes x three bounce counts).
# Outputs gpurun_out/flopcal_<MODE>/ (PMC CSV) and gpurun_out/flopcal_<MODE>.jsonl.
#   bash scripts/gpu_flopcal.sh sweep|scenes
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
M=${1:-sweep}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
  SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \
  --kernel-trace -d "$R/gpurun_out/flopcal_$M" -o pmc --output-format csv -- \
  python3 "$R/scripts/flop_calib.py" run "$R/gpurun_out/flopcal_$M.jsonl" $M > "$R/gpurun_out/flopcal_$M.log" 2>&1
rc=$?; echo "flopcal $M rc=$rc"; tail -2 "$R/gpurun_out/flopcal_$M.log"; exit $rc
