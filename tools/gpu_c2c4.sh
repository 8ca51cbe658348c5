set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r1b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "c2_matches or c4_million" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -8 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python -u bench.py --workload c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
