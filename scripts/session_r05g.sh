#!/bin/bash
# Round 5: every BASELINE config on one MI355X (scripts/configs.py) and the
# driver-form bench, on the frozen tree ab/<TREE>.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-r05g}"; T=${TAG:-r05g}
O="$R/gpurun_out"; mkdir -p "$O"
(cd "$D" && timeout -k 10 600 python scripts/configs.py > "$O/${T}_configs.jsonl" 2> "$O/${T}_configs.err")
rc=$?; echo "configs rc=$rc"; cut -c1-160 "$O/${T}_configs.jsonl"; [ $rc -eq 0 ] || exit $rc
(cd "$D" && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$O/${T}_bench.log" 2>&1)
rc=$?; echo "bench rc=$rc"; tail -c 300 "$O/${T}_bench.log"; exit $rc
