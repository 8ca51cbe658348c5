#!/bin/bash
# Round-4 refresh after the launch-form changes: the default (C3) bench line and the C2 / C2x lines
# with their per-pod side line through the C++ cache.  Usage: tools/gpu_r4v.sh <tag>
set -o pipefail
TAG=${1:-r4v}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
for W in c2 c2x; do
  timeout -k 10 400 python3 bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { echo "$W bench failed"; tail -20 $OUT/bench_$W.err; exit 1; }
  cut -c1-400 $OUT/bench_$W.json
done
