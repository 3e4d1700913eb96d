#!/bin/bash
# Host side: run one gpurun call, retrying only while gpurun answers 3 (no
# box or slot free: nothing ran, nothing charged), at most GR_TRIES times,
# GR_WAIT seconds apart.  Any other status (the command ran) is final.
#   scripts/gpurun_retry.sh <timeout s> '<command>'
t=$1; shift
for i in $(seq 1 ${GR_TRIES:-15}); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_retry] no box (try $i), waiting ${GR_WAIT:-90}s" >&2
  sleep ${GR_WAIT:-90}
done
exit 3
