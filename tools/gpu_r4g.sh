#!/bin/bash
# per-pod call: wall-time percentiles and the kernels it launches (rocprofv3 kernel trace)
set -o pipefail
TAG=${1:-r4g}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in c2 c2x; do
  timeout -k 10 300 python3 tools/perpod_prof.py --workload $W > $OUT/$W.txt 2>&1 || { tail $OUT/$W.txt; exit 1; }
  cat $OUT/$W.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$W -o run -- python3 tools/perpod_prof.py --workload $W > $OUT/prof_$W.log 2>&1 || { tail $OUT/prof_$W.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -12 "$f"; done
