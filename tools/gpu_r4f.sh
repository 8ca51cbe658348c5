#!/bin/bash
# C2 / C2x bench lines with the per-pod side line through the C++ scheduler cache.
set -o pipefail
TAG=${1:-r4f}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in c2 c2x; do
  timeout -k 10 400 python3 bench.py --workload $W --cpu-sample 0 --steps 5 --warmup 1 > $OUT/$W.json 2> $OUT/$W.err || { tail $OUT/$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', d['value'], d['ms_per_step'], json.dumps(d.get('per_pod')))"
done
