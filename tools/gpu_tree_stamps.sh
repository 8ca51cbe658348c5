#!/bin/bash
# Tree mode per-phase cycle stamps (diagnostic build) for C3 and C4.
# Usage (from the repo root on the GPU box): tools/gpu_tree_stamps.sh <tag>
set -o pipefail
TAG=${1:-ts}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
SL=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so
KSIM_LIB=$SL timeout -k 10 120 python3 bench.py --mode tree --cpu-sample 0 --steps 5 > $OUT/stamps_c3.json 2> $OUT/stamps_c3.err || { echo "stamps failed"; tail $OUT/stamps_c3.err; exit 1; }
grep 'ksim stamps' $OUT/stamps_c3.err | tail -2
KSIM_LIB=$SL timeout -k 10 180 python3 bench.py --mode tree --workload c4 --batch 4096 --cpu-sample 0 --steps 2 > $OUT/stamps_c4.json 2> $OUT/stamps_c4.err || { echo "stamps c4 failed"; tail $OUT/stamps_c4.err; exit 1; }
grep 'ksim stamps' $OUT/stamps_c4.err | tail -2
