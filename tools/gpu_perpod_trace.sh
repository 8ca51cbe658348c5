#!/bin/bash
# Per-pod path kernel trace (rocprofv3 --kernel-trace --stats) for C2 / C2x through the C++
# scheduler cache (tools/perpod_prof.py).  Usage (GPU box, repo root): tools/gpu_perpod_trace.sh <tag>
set -o pipefail
TAG=${1:-perpod_trace}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in ${WORKLOADS:-c2 c2x}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$W -o run -- python3 tools/perpod_prof.py --workload $W > $OUT/$W.txt 2>&1 || { echo "$W failed"; tail -20 $OUT/$W.txt; exit 1; }
  tail -2 $OUT/$W.txt
  find $OUT/$W -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-160 | head -6
done
