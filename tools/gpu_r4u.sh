#!/bin/bash
# per-pod c2x: cache phase profile and the scan kernel's phase stamps (diagnostic build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4u
for W in c2 c2x; do
  KSIM_CACHE_PROFILE=1 KSIM_CACHE_PROFILE_SKIP=1000 timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 | tee -a gpurun_out/r4u/prof.txt || exit 1
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 | tee -a gpurun_out/r4u/prof.txt || exit 1
done
