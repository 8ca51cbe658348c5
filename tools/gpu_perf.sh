#!/bin/bash
# Perf iteration on the GPU box: parity tests, a short bench, the stamps build's phase split.
# Usage: tools/gpu_perf.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-perf}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --cpu-sample 0 --steps 30 "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -f kubernetes-schedule-simulator_amd/lib/stamps/libksim.so ]; then
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 30 "$@" > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
  grep 'ksim stamps' $OUT/stamps.err | tail -4
fi
