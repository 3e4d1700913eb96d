#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, ';'-separated in PMC_PASSES)
# over a short bench run; results in gpurun_out/pmc_<TAG>/p<N>/.  Summarise
# with scripts/pmc_table.py.  Extra bench args: PMC_ARGS.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${PMC_TAG:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra PASSES <<< "$PMC_PASSES"
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $p --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline ${PMC_ARGS:-} > "$OUT/p${i}.log" 2>&1
  rc=$?; echo "pass $i rc=$rc ($p)"
  [ $rc -eq 0 ] || exit $rc
done
