#!/bin/bash
# per-pod latency through the C++ cache after the pass-A / predicate changes (c2, c2x)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4t
for W in c2 c2x; do
  timeout -k 10 300 python3 tools/perpod_prof.py --workload $W 2>&1 | tee -a gpurun_out/r4t/perpod.txt || exit 1
done
