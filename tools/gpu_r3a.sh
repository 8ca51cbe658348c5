#!/bin/bash
# Round-3 GPU pass: the f3 parity suites (affinity, spread, volumes, goldens, C2x; every mode, so
# the general persistent kernel and the launch form), the default bench line (C3 + the C4
# streaming side line), its kernel-trace profile, the C2x line (general persistent kernel and
# launch form), then the PMC passes of the default command.
# Test failures (pytest rc 1) do not stop the pass; a fault, abort or time-out does.
set -o pipefail
TAG=${1:-r3a}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 240 --timeout-method thread \
  -k "affinity or spread or volume or c2x or goldens_f3 or mixed_features" > $OUT/pytest_f3.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_f3.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-3500 $OUT/bench.json
timeout -k 10 300 python3 bench.py --workload c2x > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { echo "c2x bench failed"; tail -20 $OUT/bench_c2x.err; exit 1; }
cut -c1-2500 $OUT/bench_c2x.json
KSIM_NO_PGEN=1 timeout -k 10 300 python3 bench.py --workload c2x --cpu-sample 0 > $OUT/bench_c2x_launch.json 2> $OUT/bench_c2x_launch.err || { echo "c2x launch bench failed"; tail -20 $OUT/bench_c2x_launch.err; exit 1; }
cut -c1-600 $OUT/bench_c2x_launch.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2x -o run -- python3 bench.py --workload c2x > $OUT/prof_bench_c2x.json 2> $OUT/prof_c2x.err || { echo "rocprof c2x failed"; tail -20 $OUT/prof_c2x.err; exit 1; }
find $OUT/prof_c2x -name '*kernel_stats.csv' -exec cat {} \;
bash tools/gpu_pmc_bench.sh $TAG/pmc_c3
