#!/bin/bash
# GPU parity suite with the in-tree library, then a library A/B on one workload:
# tools/gpu_test_ab.sh <tag> lib1.so lib2.so ... [-- bench args]
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
exec_ab() { bash tools/gpu_libab.sh "$@"; }
exec_ab "$@"
