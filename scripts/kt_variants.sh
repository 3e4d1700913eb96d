#!/bin/bash
# Kernel-trace + stats of the bench workload per variant (env sets separated
# by ';' in KT_VARIANTS), one pipeline by default (standalone kernel times).
# Outputs gpurun_out/kv_<tag>_<i>/ and a summary line per variant.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra VARS <<< "${KT_VARIANTS:-PT_BIN_LANES=1}"
i=0
for v in "${VARS[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kv_${1:-x}_$i" -o kt \
      --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${KT_ARGS:-} \
      > "$R/gpurun_out/kv_${1:-x}_$i.log" 2>&1
  rc=$?; echo "variant $i ($v) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 "$R/scripts/kt_summary.py" "$R/gpurun_out/kv_${1:-x}_$i" | tee -a "$R/gpurun_out/kv_${1:-x}.txt"
done
