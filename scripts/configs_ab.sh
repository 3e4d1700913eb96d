#!/bin/bash
# scripts/configs.py under several env sets (';'-separated CFG_VARIANTS),
# each in its own process: gpurun_out/cfg_<tag>.jsonl, one line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "${CFG_VARIANTS:-PT_BIN_LANES=2}"
for v in "${VARS[@]}"; do
  for r in $(seq ${CFG_REPS:-1}); do
    env $v timeout -k 10 300 python scripts/configs.py ${CFG_NAMES:-c2} > gpurun_out/cfg.tmp 2>&1
    rc=$?
    sed "s/^{/{\"env\": \"$v\", /" gpurun_out/cfg.tmp | grep '^{' | tee -a gpurun_out/cfg_${1:-x}.jsonl
    [ $rc -eq 0 ] || { cat gpurun_out/cfg.tmp; exit $rc; }
  done
done
