#!/bin/bash
# A/B of tree-mode diagnostic variants (stamps builds under lib/stamps_v*/): per-phase cycles at C3 and C4.
# Usage (from the repo root on the GPU box): tools/gpu_tree_ab.sh <tag> <variant>...
set -o pipefail
TAG=${1:-tab}; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  SL=kubernetes-schedule-simulator_amd/lib/$v/libksim.so
  for w in c3 c4; do
    KSIM_LIB=$SL timeout -k 10 180 python3 bench.py --mode tree --workload $w --batch 4096 --cpu-sample 0 --steps 2 --warmup 1 > $OUT/${v}_$w.json 2> $OUT/${v}_$w.err || { echo "$v $w failed"; tail $OUT/${v}_$w.err; exit 1; }
    echo "$v $w: $(grep 'ksim stamps' $OUT/${v}_$w.err | tail -1)"
  done
done
