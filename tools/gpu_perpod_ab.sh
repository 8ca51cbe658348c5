#!/bin/bash
# Per-pod A/B of library builds on one box (the C2 workload's per-pod marks):
#   [WL=c2x] tools/gpu_perpod_ab.sh lib1.so lib2.so ...
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2 3; do
  for L in "$@"; do
    KSIM_LIB=$L timeout -k 10 200 python3 bench.py --workload ${WL:-c2} --cpu-sample 0 --steps 3 --warmup 1 > /tmp/ab.json 2>/dev/null || { echo "bench $L failed"; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('/tmp/ab.json'))
print(sys.argv[1], [(m['us_per_call'], m['p99_us'], m['adapter_pattern']['us_per_pod'], m['adapter_pattern']['p99_us']) for m in d['per_pod']['marks']])" $L
  done
done
