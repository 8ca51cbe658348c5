#!/bin/bash
# A/B of an environment switch on the default C3 bench: tools/gpu_ab.sh VAR [bench args]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
V=$1; shift
for rep in 1 2; do
  for on in 0 1; do
    if [ $on = 1 ]; then export $V=1; else unset $V; fi
    timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 30 --warmup 2 "$@" > /tmp/ab.json 2>/dev/null || { echo "bench failed"; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/ab.json')); print('$V=$on', d['value'], d['roofline']['avg_launch_us'])"
  done
done
