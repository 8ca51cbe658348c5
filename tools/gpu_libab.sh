#!/bin/bash
# A/B of library builds on one box: tools/gpu_libab.sh lib1.so lib2.so ... [-- bench args]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; shift
for rep in 1 2 3; do
  for L in "${LIBS[@]}"; do
    KSIM_LIB=$L timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 30 --warmup 2 "$@" > /tmp/ab.json 2>/dev/null || { echo "bench $L failed"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], d['value'], d['roofline']['avg_launch_us'])" $L
  done
done
