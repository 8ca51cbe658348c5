#!/bin/bash
# Kernel-trace + stats profile of a short bench run (run on the GPU box from the repo root).
# Usage: tools/profile_bench.sh <tag> [bench args...]
set -e
TAG=${1:-run}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --cpu-sample 0 "$@"
