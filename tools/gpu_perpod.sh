#!/bin/bash
# Per-pod path: the cache-event GPU tests, then the C2x and C2 bench lines with their per_pod side
# lines (ksim_schedule_one latency at 1k and 20k cached pods).  Usage: tools/gpu_perpod.sh <tag>
set -o pipefail
TAG=${1:-perpod}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cache.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_cache.log 2>&1 || { echo "cache tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_cache.log | head -30; tail -20 $OUT/pytest_cache.log; exit 1; }
tail -3 $OUT/pytest_cache.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden_priorities or golden_reduce" > $OUT/pytest_golden.log 2>&1 || { echo "golden tests failed"; grep -E "^E |FAILED" $OUT/pytest_golden.log | head -20; exit 1; }
tail -2 $OUT/pytest_golden.log
timeout -k 10 400 python3 -u bench.py --workload c2x --cpu-sample 0 --per-pod-calls 200 > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { echo "c2x bench failed"; tail -20 $OUT/bench_c2x.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench_c2x.json')); print(d['value'], json.dumps(d.get('per_pod')))"
timeout -k 10 400 python3 -u bench.py --workload c2 --cpu-sample 0 --per-pod-calls 200 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "c2 bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench_c2.json')); print(d['value'], json.dumps(d.get('per_pod')))"
