#!/bin/bash
# Round 5 one-GPU rehearsal of the driver's N-GPU line on the frozen tree
# ab/<TREE>: bench.py --gpus 2 / 4 at the full workload (1080p, 256 spp per
# GPU-share, c4_strong leg), ranks sharing GPU 0 over gloo, WITHOUT
# --validate: the line must prove itself (tile_check, render_ms_per_rank).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-r05f}"; T=${TAG:-r05f}
O="$R/gpurun_out"; mkdir -p "$O"
for n in 2 4; do
  (cd "$D" && PT_BENCH_SHARE_GPU=1 OMP_NUM_THREADS=4 timeout -k 10 500 python bench.py --gpus $n --dist-backend gloo \
     --steps 2 --warmup 1 --c4-steps 1 > "$O/${T}_mgpu_rehearsal_${n}rank.log" 2>&1)
  rc=$?; echo "ranks $n rc=$rc"; tail -c 400 "$O/${T}_mgpu_rehearsal_${n}rank.log"; [ $rc -eq 0 ] || exit $rc
done
