#!/bin/bash
# Instruction-cache and issue counters of the pipeline kernels, two pipelines
# (default) vs one (bench.py --pipelines 1).  Each PMC pass is its own short run.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/icache"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lanes in 2 1; do
  i=0
  for p in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
           "SQ_IFETCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $p --kernel-trace -d "$OUT/l${lanes}_pmc$i" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --pipelines $lanes > "$OUT/l${lanes}_pmc${i}.log" 2>&1
    rc=$?; echo "lanes $lanes pass $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
