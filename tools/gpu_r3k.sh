#!/bin/bash
# C front end loop + f3 suites + C2x line.
set -o pipefail
TAG=${1:-r3k}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 ./tests/c/build/ksim_k8s_loop 240 1500 > $OUT/k8s_loop.log 2>&1; echo "k8s loop rc=$?"; tail -12 $OUT/k8s_loop.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 240 --timeout-method thread \
  -k "affinity or spread or volume or c2x or goldens_f3 or mixed_features or c_abi" > $OUT/pytest_f3.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_f3.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 bench.py --workload c2x > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { echo "c2x bench failed"; tail -20 $OUT/bench_c2x.err; exit 1; }
cut -c1-500 $OUT/bench_c2x.json; grep -o '"parity": {[^}]*}' $OUT/bench_c2x.json
