#!/bin/bash
# The -m gpu suite (optionally a -k filter) and smoke() on the GPU box; output under gpurun_out/<tag>.
# Usage (from the repo root on the GPU box): tools/gpu_suite.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-suite}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head -30; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -14 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
