#!/bin/bash
# One-GPU rehearsal of the N-GPU bench paths on the frozen tree ab/<TREE>:
# bench.py --gpus 2 / 4 launching its own ranks (all on GPU 0, gloo host
# reduce, --validate: the assembled image against a one-context render),
# then BASELINE config 4 on one GPU (--config c4).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-r04c}"; T=${TAG:-r04c}
O="$R/gpurun_out"; mkdir -p "$O"
for n in 2 4; do
  (cd "$D" && PT_BENCH_SHARE_GPU=1 OMP_NUM_THREADS=4 timeout -k 10 400 python bench.py --gpus $n --dist-backend gloo \
     --width 960 --height 544 --spp 8 --steps 2 --warmup 1 --validate --no-cpu-baseline \
     > "$O/${T}_mgpu_rehearsal_${n}rank.log" 2>&1)
  rc=$?; echo "ranks $n rc=$rc"; tail -c 300 "$O/${T}_mgpu_rehearsal_${n}rank.log"; [ $rc -eq 0 ] || exit $rc
done
(cd "$D" && timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > "$O/${T}_bench_c4.log" 2>&1)
rc=$?; echo "c4 rc=$rc"; tail -c 300 "$O/${T}_bench_c4.log"; exit $rc
