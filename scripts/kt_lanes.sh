#!/bin/bash
# Kernel-trace + stats of the bench workload with one and two pipelines
# (bench.py --pipelines), to separate each kernel's standalone time from its time
# beside the other pipeline.  Outputs gpurun_out/kt_<tag>_l<N>/.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for n in ${LANES:-1 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_${1:-x}_l$n" -o kt \
      --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --pipelines $n ${KT_ARGS:-} \
      > "$R/gpurun_out/kt_${1:-x}_l$n.log" 2>&1
  rc=$?; echo "lanes $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
