#!/bin/bash
# Critical-path probe A/B for one workload on one box: the C2 parity subset, then the base
# library and each probe build (tools/probe_libs.sh) timed twice, then the stamps split.
# Usage: tools/gpu_probe_ab.sh <tag> <pytest -k expr> <workload> k1 k2 ...
set -o pipefail
TAG=$1; K=$2; W=$3; shift 3
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
L=kubernetes-schedule-simulator_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for v in base "$@"; do
    lib=$L/libksim.so; [ "$v" != base ] && lib=$L/probe$v/libksim.so
    KSIM_LIB=$lib timeout -k 10 120 python3 bench.py --workload $W --cpu-sample 0 > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { echo "bench $v failed"; tail -5 $OUT/ab_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], round(1e6/d['value'],3), 'us/pod')" $OUT/ab_$v.json $v
  done
done
KSIM_LIB=$L/stamps/libksim.so timeout -k 10 120 python3 bench.py --workload $W --cpu-sample 0 --steps 3 > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
grep 'ksim stamps' $OUT/stamps.err | tail -4
