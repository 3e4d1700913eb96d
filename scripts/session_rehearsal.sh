#!/bin/bash
# One-GPU rehearsal of the N-GPU bench line: bench.py --gpus 2 / 4 launching
# its own ranks, all on GPU 0 (PT_BENCH_SHARE_GPU), reducing over gloo on the
# host (RCCL refuses two ranks on one device).  Default: the driver's form --
# the full 1080p workload, no --validate, the line's own tile check
# (including the non-finite tiles) and the c4_strong leg; RANK_ARGS replaces
# the workload flags.  Then BASELINE config 4 on one GPU (--config c4).
#   TAG=r06j [TREE=x] [RANK_ARGS="..."] bash scripts/session_rehearsal.sh
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R"; [ -n "${TREE:-}" ] && D="$R/ab/$TREE"
T=${TAG:?TAG}
O="$R/gpurun_out"; mkdir -p "$O"
for n in 2 4; do
  (cd "$D" && PT_BENCH_SHARE_GPU=1 OMP_NUM_THREADS=4 timeout -k 10 600 python bench.py --gpus $n --dist-backend gloo \
     ${RANK_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --c4-steps 1} \
     > "$O/${T}_mgpu_rehearsal_${n}rank.log" 2>&1)
  rc=$?; echo "ranks $n rc=$rc"; tail -c 300 "$O/${T}_mgpu_rehearsal_${n}rank.log"; [ $rc -eq 0 ] || exit $rc
done
(cd "$D" && timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/${T}_bench_c4.log" 2>&1)
rc=$?; echo "c4 rc=$rc"; tail -c 300 "$O/${T}_bench_c4.log"; exit $rc
