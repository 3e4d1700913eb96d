#!/bin/bash
# Run a GPU session (scripts/gpu_session.sh) inside a frozen copy of the tree
# (ab/<name>, made by scripts/freeze.sh), so edits made here while a gpurun
# call waits in the queue do not change what it runs.  Outputs go to the
# repo's top-level gpurun_out/ (the only directory gpurun brings back, and
# the one its silence watchdog watches).
#   scripts/frozen_session.sh <ab dir> <tag> [pytest args...]
set -u
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
d="$root/$1"; tag=$2; shift 2
mkdir -p "$root/gpurun_out"
(cd "$d" && GRAFT_REPO_ROOT="$d" GPU_OUT="$root/gpurun_out" bash "$root/scripts/gpu_session.sh" "$tag" "$@")
