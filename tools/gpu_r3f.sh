#!/bin/bash
# f3 GPU suites + the C2x line + the stamps breakdown of the general persistent kernel.
set -o pipefail
TAG=${1:-r3f}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 240 --timeout-method thread \
  -k "affinity or spread or volume or c2x or goldens_f3 or mixed_features" > $OUT/pytest_f3.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_f3.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 bench.py --workload c2x > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { echo "c2x bench failed"; tail -20 $OUT/bench_c2x.err; exit 1; }
cut -c1-700 $OUT/bench_c2x.json; grep -o '"parity": {[^}]*}' $OUT/bench_c2x.json
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --workload c2x --cpu-sample 0 --steps 2 --warmup 0 > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 1; }
grep stamps $OUT/st.err
