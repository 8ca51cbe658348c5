#!/bin/bash
# A/B of library builds x an environment switch: tools/gpu_libab2.sh VAR lib1.so lib2.so ...
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
V=$1; shift
for rep in 1 2; do
  for L in "$@"; do
    for on in 0 1; do
      if [ $on = 1 ]; then export $V=1; else unset $V; fi
      KSIM_LIB=$L timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 30 --warmup 2 > /tmp/ab.json 2>/dev/null || { echo "bench $L failed"; exit 1; }
      python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], '$V=$on', d['value'], d['roofline']['avg_launch_us'])" $L
    done
  done
done
