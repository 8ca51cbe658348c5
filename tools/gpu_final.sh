#!/bin/bash
# Round-end record, second pass: PMC passes for the C3 and C2 lines, the C2 / C2x per_pod lines,
# the per-pod kernel trace, and the pipelined-kernel A/B.  Usage (GPU box): tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_pmc.sh ${TAG}_pmc_c3 || exit 1
bash tools/gpu_pmc.sh ${TAG}_pmc_c2 --workload c2 || exit 1
for w in c2 c2x; do
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  cut -c1-300 $OUT/bench_$w.json
done
WORKLOADS="c2 c2x" bash tools/gpu_perpod_trace.sh ${TAG}_trace || exit 1
