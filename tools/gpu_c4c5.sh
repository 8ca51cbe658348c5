#!/bin/bash
# Streaming (C4) and sweep (C5) checks: their parity tests, then both bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-c4c5}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stream or c4 or sweep or sharded or fast or tiny" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --workload c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -20 $OUT/bench_c4.err; exit 1; }
cut -c1-400 $OUT/bench_c4.json
timeout -k 10 300 python3 bench.py --workload c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench c5 failed"; tail -20 $OUT/bench_c5.err; exit 1; }
cut -c1-400 $OUT/bench_c5.json
