#!/bin/bash
# Round-3 record on the GPU box: the default bench line and the kernel-trace profile of the SAME
# command, then the C2x line and its kernel-trace profile.  Usage: tools/gpu_r3final.sh <tag>
set -o pipefail
TAG=${1:-r3final}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-900 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -12
timeout -k 10 300 python3 bench.py --workload c2x > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { echo "c2x bench failed"; tail -20 $OUT/bench_c2x.err; exit 1; }
cut -c1-600 $OUT/bench_c2x.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2x -o run -- python3 bench.py --workload c2x > $OUT/prof_bench_c2x.json 2> $OUT/prof_c2x.err || { echo "rocprof c2x failed"; tail -20 $OUT/prof_c2x.err; exit 1; }
find $OUT/prof_c2x -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -12
