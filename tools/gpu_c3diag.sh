#!/bin/bash
# C3 diagnostics: per-phase cycle stamps, the grid-size sweep, then the C4 bench line and its
# kernel-trace profile.  Usage: tools/gpu_c3diag.sh <tag>
set -o pipefail
TAG=${1:-diag}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
grep "ksim stamps" $OUT/stamps.err | tail -3
timeout -k 10 600 bash tools/gpu_grid_sweep.sh > $OUT/grid.txt 2>&1 || { echo "grid failed"; cat $OUT/grid.txt; exit 1; }
cat $OUT/grid.txt
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload c4 --cpu-sample 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
