#!/bin/bash
# per-pod: kernel-argument placement A/B and the scan stamps
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for W in c2 c2x; do
  for K in 0 1; do
    echo -n "HIP_FORCE_DEV_KERNARG=$K "
    HIP_FORCE_DEV_KERNARG=$K timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
  done
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
done
