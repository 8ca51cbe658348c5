#!/bin/bash
# per-pod profile, then the -m gpu suite without the full-size scale tests, then smoke
set -o pipefail
TAG=${1:-r4k}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in c2 c2x; do
  KSIM_CACHE_PROFILE=1 KSIM_CACHE_PROFILE_SKIP=1000 timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
done
bash tools/gpu_suite.sh $TAG "${2:-not test_gpu_scale}"
