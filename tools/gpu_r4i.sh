#!/bin/bash
# per-pod: the profile of the timed window, then the per-pod / cache parity suites
set -o pipefail
TAG=${1:-r4i}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in c2 c2x; do
  KSIM_CACHE_PROFILE=1 KSIM_CACHE_PROFILE_SKIP=1000 timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${2:-test_gpu_cache or k8s or c_abi or schedule_one or per_pod or perpod}" > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
