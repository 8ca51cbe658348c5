#!/bin/bash
# C3 pods/s of the fast persistent kernel against the workgroup count (KSIM_MAX_GRID).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for g in 256 192 160 128 96 64; do
  KSIM_MAX_GRID=$g timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 20 --warmup 2 > /tmp/b_$g.json 2>/dev/null || { echo "grid $g failed"; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/b_$g.json')); print($g, d['value'], d['config']['blocks'], d['roofline']['avg_launch_us'])"
done
