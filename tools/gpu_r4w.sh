#!/bin/bash
# Round-4 closing record: the whole -m gpu suite (full-size scale tests included) and smoke()
set -o pipefail
TAG=${1:-r4w}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $OUT/pytest_gpu_full.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu_full.log | head -30; tail -30 $OUT/pytest_gpu_full.log; exit 1; }
tail -18 $OUT/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
