#!/bin/bash
# Build the library of a git revision (default HEAD) as an A/B variant:
# compute_path_tracer_amd/lib/variants/libpt_<name>.so (load it with PT_LIB=...).
set -eu
REV="${1:-HEAD}"; NAME="${2:-head}"
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TMP="$(mktemp -d)"
git -C "$ROOT" archive "$REV" | tar -x -C "$TMP"
(cd "$TMP" && python -m compute_path_tracer_amd.build --force > /dev/null)
mkdir -p "$ROOT/compute_path_tracer_amd/lib/variants"
cp "$TMP/compute_path_tracer_amd/lib/libpt.so" "$ROOT/compute_path_tracer_amd/lib/variants/libpt_$NAME.so"
rm -rf "$TMP"
echo "$ROOT/compute_path_tracer_amd/lib/variants/libpt_$NAME.so"
