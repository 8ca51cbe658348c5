set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3b; mkdir -p $OUT
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --workload c2x --cpu-sample 0 --steps 2 --warmup 0 > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 1; }
grep stamps $OUT/st.err; cut -c1-200 $OUT/st.json
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 240 --timeout-method thread \
  -k "affinity or spread or volume or c2x or goldens_f3 or mixed_features" > $OUT/pytest_f3.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_f3.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python3 bench.py --workload c2x --cpu-sample 0 > $OUT/bench_c2x.json 2> $OUT/bench_c2x.err || { tail $OUT/bench_c2x.err; exit 1; }
cut -c1-400 $OUT/bench_c2x.json
