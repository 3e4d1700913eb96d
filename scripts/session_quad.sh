#!/bin/bash
# Round 4 GPU call: the hit-quad tree's GPU suite + smoke, the A/B bench of
# the pre-quad tree (ab/r04a) against it, and the traffic-probe calibration.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
SKIP_BENCH=1 scripts/frozen_session.sh ab/quad r04q || exit $?
AB_PAIRS=2 scripts/ab_trees.sh ab/r04a ab/quad ab/quad@PT_JIT_DEFS=PT_SHADE_QPREFETCH || exit $?
bash scripts/pmc_calib.sh
