#!/bin/bash
# per-pod call A/B: pod descriptor read from mapped host memory vs a device copy
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1; do
for W in c2 c2x; do
  for D in 0; do
    echo -n "KSIM_POD_DEVICE=$D "
    KSIM_CACHE_PROFILE=1 KSIM_CACHE_PROFILE_SKIP=1000 KSIM_POD_DEVICE=$D timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
  done
done
done
