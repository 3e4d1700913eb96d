#!/bin/bash
# rocprofv3 runs for the bench workload (kernel trace + stats, then PMC passes).
# Usage: PROF_TAG=r01 bash scripts/profile.sh [pmc]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${PROF_TAG:-r01}"
OUT="${GPU_OUT:-$R/gpurun_out}/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# (no tile check, no table-kernel leg: their launches carry the same kernel
# names and would mix into the per-kernel statistics)
ARGS="${PROF_ARGS:---steps 4 --warmup 1 --no-cpu-baseline} --no-tile-check --no-table-kernel"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" $ARGS > "$OUT/kt_bench.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; tail -1 "$OUT/kt_bench.log"
[ $rc -eq 0 ] || exit $rc
if [ "${1:-}" = "pmc" ]; then
  i=0
  IFS=';' read -ra PASSES <<< "${PMC_PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY;FETCH_SIZE;WRITE_SIZE}"
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace -d "$OUT/pmc$i" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-tile-check --no-table-kernel ${PMC_ARGS:-} > "$OUT/pmc${i}.log" 2>&1
    rc=$?; echo "pmc pass $i ($p) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
