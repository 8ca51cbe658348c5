#!/bin/bash
# C5 scenario sweep on the GPU box: bench line, kernel trace, FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
TAG=${1:-c5}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --workload c5 "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
ARGS="--workload c5 --steps 1 --warmup 0 --cpu-sample 0 --scenarios 1024"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail $OUT/trace.err; exit 1; }
find $OUT/trace -name '*kernel_stats.csv' -exec cat {} \;
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.json 2> $OUT/fetch.err || { echo "fetch failed"; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.json 2> $OUT/write.err || { echo "write failed"; tail $OUT/write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o run -- python3 bench.py $ARGS > $OUT/tcc.json 2> $OUT/tcc.err || { echo "tcc failed"; tail $OUT/tcc.err; exit 1; }
python3 tools/pmc_summary.py $OUT
