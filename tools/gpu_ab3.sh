#!/bin/bash
# GPU parity suite, then C3 A/B over several libraries and C4 A/B over several libraries.
# Usage: tools/gpu_ab3.sh <tag> "<c3 libs>" "<c4 libs>"
set -o pipefail
TAG=$1; C3L=$2; C4L=$3
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
[ -n "$C3L" ] && { bash tools/gpu_libab.sh $C3L || exit 1; }
[ -n "$C4L" ] && { bash tools/gpu_libab.sh $C4L -- --workload c4 || exit 1; }
exit 0
