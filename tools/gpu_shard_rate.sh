#!/bin/bash
# Node-sharded launch form (Phase A): the per-rank rate of the second call for C2 / C2x shapes,
# `world` processes on this box's device(s) (a one-device rehearsal shares one GPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/shard_rate
for W in c2 c2x; do
  for WORLD in 1 2; do
    PORT=$((29500 + RANDOM % 2000))
    PIDS=()
    for ((r = 0; r < WORLD; r++)); do
      timeout -k 10 300 python3 tests/shard_worker.py $r $WORLD $PORT gpurun_out/shard_rate/$W-$WORLD-$r.npz 0 5000 3000 1000 $W > gpurun_out/shard_rate/$W-$WORLD-$r.log 2>&1 &
      PIDS+=($!)
    done
    for p in "${PIDS[@]}"; do wait $p || { echo "rank failed ($W world $WORLD)"; cat gpurun_out/shard_rate/$W-$WORLD-*.log | tail -20; exit 1; }; done
    grep -h "pods/s" gpurun_out/shard_rate/$W-$WORLD-*.log
  done
done
