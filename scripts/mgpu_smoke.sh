#!/bin/bash
# Multi-rank rehearsal on a single-GPU box: NPROC ranks share GPU 0. RCCL
# refuses duplicate devices, so the image reduce goes over gloo on the host;
# --validate checks the assembled image against a 1-GPU render bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PT_BENCH_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NPROC:-2} --steps 2 --warmup 1 --no-cpu-baseline \
  --width ${WIDTH:-480} --height ${HEIGHT:-270} --dist-backend gloo --validate > gpurun_out/mgpu.log 2>&1
rc=$?; echo "torchrun rc=$rc"; grep -E '^\{' gpurun_out/mgpu.log | tail -1; grep -iE "error|duplicate|invalid" gpurun_out/mgpu.log | head -5
exit 0
