#!/bin/bash
# GPU parity suite, then C3 and C4 library A/B (new in-tree vs a variant), then C3 stamps.
# Usage: tools/gpu_ab2.sh <tag> <variant.so>
set -o pipefail
TAG=$1; V=$2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
L=kubernetes-schedule-simulator_amd/lib/libksim.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_libab.sh $L $V || exit 1
bash tools/gpu_libab.sh $L $V -- --workload c4 || exit 1
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
grep "ksim stamps" $OUT/stamps.err | tail -3
