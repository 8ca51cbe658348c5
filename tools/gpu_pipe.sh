#!/bin/bash
# Pipelined fast kernel (KSIM_PIPE=1): parity subset, A/B bench against the 1-deep kernel, stamps.
# Usage (GPU box, repo root): tools/gpu_pipe.sh <tag>
set -o pipefail
TAG=${1:-pipe}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
KSIM_PIPE=1 KSIM_PIPE_SPEC=${SPEC:-1} timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "cached_fast or c3_prefix or c3_full or score_boundaries or fast_and_general or hands_over or c1_full" > $OUT/pytest_pipe.log 2>&1 \
  || { echo "pipe tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_pipe.log | head -20; exit 1; }
tail -2 $OUT/pytest_pipe.log
for v in 0 1 2; do
  KSIM_PIPE=$((v > 0)) KSIM_PIPE_SPEC=$((v > 1)) timeout -k 10 200 python3 bench.py --cpu-sample 0 --steps 10 --warmup 1 > $OUT/bench$v.json 2> $OUT/bench$v.err || { tail $OUT/bench$v.err; exit 1; }
  echo "pipe=$((v > 0)) spec=$((v > 1)) $(grep -o '"value": [0-9.]*' $OUT/bench$v.json | head -1)"
done
KSIM_PIPE=1 KSIM_PIPE_SPEC=${SPEC:-1} KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --cpu-sample 0 --steps 2 --warmup 0 > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 1; }
grep "stamps\] pipe" $OUT/st.err | head -3
