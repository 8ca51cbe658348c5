#!/bin/bash
# C2 iteration on the GPU box: the whole -m gpu suite, the C2 bench line, the stamps build's
# phase split.  Usage: tools/gpu_c2.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-c2}; K=${2:-}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 "${KA[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -22 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --workload c2 --cpu-sample 0 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
cut -c1-600 $OUT/bench_c2.json
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --workload c2 --cpu-sample 0 --steps 3 > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
grep 'ksim stamps' $OUT/stamps.err | tail -4
