#!/bin/bash
# Round-6 record on one GPU box.  Usage (GPU box, repo root): tools/gpu_r6.sh <tag> suite|measure
#   suite:   the whole -m gpu suite and smoke()
#   measure: the default bench line (C3) and the kernel trace of the same command, the C2 / C2x
#            lines, PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs) for C3 / C2 / C2x
set -o pipefail
TAG=${1:-r6}; WHAT=${2:-measure}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$WHAT" = suite ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1 \
    || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head -30; tail -20 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  exit 0
fi
timeout -k 10 300 python3 bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench failed"; tail $OUT/bench_c3.err; exit 1; }
cut -c1-300 $OUT/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py > $OUT/bench_c3_under_rocprof.json 2> $OUT/prof_c3.err || { echo "rocprof failed"; tail $OUT/prof_c3.err; exit 1; }
for w in c2 c2x; do
  timeout -k 10 300 python3 bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
  cut -c1-200 $OUT/bench_$w.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2x -o run -- python3 bench.py --workload c2x --cpu-sample 0 > $OUT/bench_c2x_under_rocprof.json 2> $OUT/prof_c2x.err || { echo "rocprof c2x failed"; tail $OUT/prof_c2x.err; exit 1; }
for w in c3 c2 c2x; do
  mkdir -p $OUT/pmc_$w
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$w/$ctr -o run -- python3 bench.py --workload $w --cpu-sample 0 --per-pod-calls 0 --steps 5 --warmup 1 \
      > $OUT/pmc_$w/$ctr.json 2> $OUT/pmc_$w/$ctr.err || { echo "pmc $w $ctr failed"; tail $OUT/pmc_$w/$ctr.err; exit 1; }
  done
done
ls -R $OUT | head -60
