cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${ABL:-BASE PT_EXP_NOTAPS PT_EXP_NOBOUNDS}; do
  if [ $v = BASE ]; then D=""; else D=$v; fi
  PT_BIN_LANES=1 PT_JIT_DEFS=$D timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/abl_$v -o kt --output-format csv -- python3 $R/bench.py --bounces 1 --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/abl_$v.log 2>&1 || exit 1
  echo "$v ok"
done
