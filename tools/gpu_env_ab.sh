#!/bin/bash
# A/B of environment settings for one workload on one box (each timed twice).
# Usage: tools/gpu_env_ab.sh <tag> <workload> "ENV=V ..." "ENV=V ..." ...   ("-" = no setting)
set -o pipefail
TAG=$1; W=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    if [ "$e" = "-" ]; then envs=(); else read -ra envs <<< "$e"; fi
    env "${envs[@]}" timeout -k 10 120 python3 bench.py --workload $W --cpu-sample 0 > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { echo "bench [$e] failed"; tail -5 $OUT/ab_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], round(1e6/d['value'],3), 'us/pod', d['config'].get('blocks'))" $OUT/ab_$i.json "$e"
  done
done
