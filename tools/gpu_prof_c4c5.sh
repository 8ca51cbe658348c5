#!/bin/bash
# Kernel-trace profiles of the C4 bench (streaming scan + tree mode) and the C5 sweep bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-profc4c5}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- python3 bench.py --workload c4 --cpu-sample 0 > $OUT/bench_c4.json 2> $OUT/c4.err || { echo "c4 prof failed"; tail -20 $OUT/c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
find $OUT/c4 -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o run -- python3 bench.py --workload c5 --cpu-sample 0 > $OUT/bench_c5.json 2> $OUT/c5.err || { echo "c5 prof failed"; tail -20 $OUT/c5.err; exit 1; }
cut -c1-300 $OUT/bench_c5.json
find $OUT/c5 -name '*kernel_stats.csv' -exec cat {} \;
