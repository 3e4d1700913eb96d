#!/bin/bash
# Round session: GPU tests + smoke + bench (scripts/gpu_session.sh), then
# the rocprofv3 kernel-trace and PMC passes of the bench (scripts/profile.sh).
#   scripts/gpu_full.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}
scripts/gpu_session.sh "$tag" || exit $?
PROF_TAG=$tag bash scripts/profile.sh pmc
