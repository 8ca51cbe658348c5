#!/bin/bash
# Round 4: the per-pod drop-in suites (both cache mirrors, the front end, the plain-C loops) and the
# C3 per-phase stamps of the fast persistent kernel (diagnostic lib, make stamps).
set -o pipefail
TAG=${1:-r4b}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-tree --c4-pods 0 --steps 2 --warmup 0 --pods 200000 > $OUT/st_c3.json 2> $OUT/st_c3.err || { tail $OUT/st_c3.err; exit 1; }
grep stamps $OUT/st_c3.err | head -8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 \
  -k "${2:-test_gpu_cache or k8s or c_abi}" > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest.log | head -40; tail -30 $OUT/pytest.log; exit 1; }
tail -15 $OUT/pytest.log
