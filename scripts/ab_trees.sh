#!/bin/bash
# A/B of source trees on one box: alternating bench runs of each tree (an
# extracted, built revision such as ab/r03u, or "." for the repo), AB_PAIRS
# rounds.  Results: gpurun_out/ab_trees.log.
#   scripts/ab_trees.sh tree_A tree_B ...      (AB_ARGS: bench flags)
# A tree may carry environment settings for its runs: ab/x@PT_JIT_DEFS=FOO.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
root=$(pwd)
mkdir -p gpurun_out
for p in $(seq 1 ${AB_PAIRS:-2}); do
  for spec in "$@"; do
    t=${spec%%@*}; envs=""
    [ "$t" != "$spec" ] && envs=${spec#*@}
    (cd "$root/$t" && env $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-20} --warmup ${AB_WARMUP:-5} \
        --no-cpu-baseline ${AB_ARGS:-} > "$root/gpurun_out/ab_tree.tmp" 2>&1)
    rc=$?
    echo "pair $p tree $spec rc=$rc $(python scripts/parse_bench.py gpurun_out/ab_tree.tmp 2>/dev/null | cut -c1-160)" \
      | tee -a gpurun_out/ab_trees.log
    if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_tree.tmp; exit $rc; fi
  done
done
