#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the traffic probes (pt_probe.hip), one counter
# per rocprofv3 pass, then the measured / known byte ratios per access shape
# (scripts/calib_table.py -> gpurun_out/calib.json).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 "$R/scripts/traffic_probe.py" > "$R/gpurun_out/calib_plain.log" 2>&1 || exit $?
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -d "$R/gpurun_out/calib_$p" -o calib --output-format csv -- \
      python3 "$R/scripts/traffic_probe.py" > "$R/gpurun_out/calib_$p.log" 2>&1
  rc=$?; echo "calib $p rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 "$R/scripts/calib_table.py" "$R/gpurun_out"
