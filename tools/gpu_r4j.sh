#!/bin/bash
# per-pod: scan-kernel phase stamps (diagnostic lib)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for W in c2 c2x; do
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 || exit 1
done
