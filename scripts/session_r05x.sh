#!/bin/bash
# Round 5: what the shade pass waits on -- PMC passes over
# one one-pipeline bench step of the final tree: vector memory / LDS
# instruction counts and waits, LDS bank conflicts, L2 and vector-L1 hits.
# Each counter is asked for only if this box's rocprofv3 lists it.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
D="$R/ab/${TREE:-final}"; O="$R/gpurun_out/prof_r05x"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > "$O/counters.txt" 2>&1
rc=$?; echo "list rc=$rc $(wc -l < "$O/counters.txt") lines"; [ $rc -eq 0 ] || exit $rc
have() { grep -qw "$1" "$O/counters.txt"; }
i=0
for pass in "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU" \
            "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAVES" \
            "TCC_HIT TCC_MISS" "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ TCP_PENDING_STALL_CYCLES"; do
  sel=""
  for c in $pass; do
    b=${c%_sum}
    if have "$b"; then case "$b" in TCC_*|TCP_*) sel="$sel ${b}_sum";; *) sel="$sel $b";; esac; fi
  done
  i=$((i+1))
  [ -z "$sel" ] && { echo "pass $i: none listed"; continue; }
  timeout -s KILL 240 rocprofv3 --pmc $sel --kernel-trace -d "$O/pmc$i" -o pmc --output-format csv -- \
      python3 "$D/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-tile-check --no-table-kernel --pipelines 1 \
      > "$O/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($sel) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then exit $rc; fi
done
exit 0
