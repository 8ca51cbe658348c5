#!/bin/bash
# Quick perf iteration: selected GPU tests (-k), one bench line, the stamps build's phase split.
# Usage: tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args...]
set -o pipefail
TAG=$1; K=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --cpu-sample 0 "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-700 $OUT/bench.json
if [ -f kubernetes-schedule-simulator_amd/lib/stamps/libksim.so ]; then
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 4 "$@" > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
  grep 'ksim stamps' $OUT/stamps.err | tail -3
fi
