#!/bin/bash
# Freeze the working tree for a GPU call: ab/<name> = the tracked files as
# they are now (committed or not) plus the built libraries (libpt.so, its
# jitcache, the oracle), so later edits do not reach a queued gpurun call.
#   scripts/freeze.sh <name>
set -eu
cd "$(dirname "$0")/.."
name=$1
rm -rf "ab/$name" && mkdir -p "ab/$name"
git ls-files -z | grep -zv "^profiles/" | xargs -0 tar -cf - | tar -xf - -C "ab/$name"
mkdir -p "ab/$name/profiles" && cp profiles/*_pmc.json "ab/$name/profiles/"
mkdir -p "ab/$name/compute_path_tracer_amd/lib"
cp -r compute_path_tracer_amd/lib/libpt.so compute_path_tracer_amd/lib/jitcache "ab/$name/compute_path_tracer_amd/lib/"
cp oracle/libpt_oracle.so "ab/$name/oracle/"
cp compute_path_tracer_amd/csrc/pt_embed.inc "ab/$name/compute_path_tracer_amd/csrc/"
echo "ab/$name"
