#!/bin/bash
# Round-4 record: the default bench line and the kernel-trace profile of the SAME command, the C3
# PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs), then the C2 / C2x (with the per-pod line
# through the C++ cache), C4 and C5 lines.  Usage: tools/gpu_r4final.sh <tag>
set -o pipefail
TAG=${1:-r4final}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-700 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -8
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_c3/fetch -o run -- python3 bench.py --cpu-sample 0 --c4-pods 0 --no-tree > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo "fetch pass failed"; tail $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_c3/write -o run -- python3 bench.py --cpu-sample 0 --c4-pods 0 --no-tree > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo "write pass failed"; tail $OUT/pmc_write.err; exit 1; }
python3 tools/pmc_summary.py $OUT/pmc_c3 --record c3 pfast 5000000000 "bench.py --cpu-sample 0 --c4-pods 0 --no-tree" > $OUT/pmc_c3_record.json || { echo "pmc summary failed"; exit 1; }
head -20 $OUT/pmc_c3_record.json
for W in c2 c2x c4 c5; do
  timeout -k 10 400 python3 bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { echo "$W bench failed"; tail -20 $OUT/bench_$W.err; exit 1; }
  cut -c1-500 $OUT/bench_$W.json
done
