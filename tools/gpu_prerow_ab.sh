#!/bin/bash
# Tree-mode row-prefetch A/B: tree + sweep parity tests on the default library, then C3 / C4 / C5
# tree bench lines for lib/v0 (a HEAD build of ksim_tree.hip linked beside the other objects) and
# the default library (the variant under test), and the stamps build.
# Usage (from the repo root on the GPU box): tools/gpu_prerow_ab.sh <tag>
set -o pipefail
TAG=${1:-pr}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tree or sweep" > $OUT/pytest_tree.log 2>&1 || { echo "tree tests failed"; tail -30 $OUT/pytest_tree.log; exit 1; }
tail -2 $OUT/pytest_tree.log
for r in 1 2; do
for v in v0 new; do
  if [ $v = v0 ]; then export KSIM_LIB=kubernetes-schedule-simulator_amd/lib/v0/libksim.so; else unset KSIM_LIB; fi
  timeout -k 10 120 python3 bench.py --mode tree --cpu-sample 0 --steps 20 > $OUT/${v}_c3_$r.json 2> $OUT/${v}_c3_$r.err || { echo "$v c3 failed"; tail $OUT/${v}_c3_$r.err; exit 1; }
  timeout -k 10 180 python3 bench.py --mode tree --workload c4 --batch 4096 --cpu-sample 0 --steps 2 --warmup 1 > $OUT/${v}_c4_$r.json 2> $OUT/${v}_c4_$r.err || { echo "$v c4 failed"; tail $OUT/${v}_c4_$r.err; exit 1; }
  python3 -c "import json,sys; [print('$v', f, json.load(open(f))['value']) for f in sys.argv[1:]]" $OUT/${v}_c3_$r.json $OUT/${v}_c4_$r.json
done
done
unset KSIM_LIB
timeout -k 10 300 python3 bench.py --workload c5 --cpu-sample 0 --steps 3 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
python3 -c "import json; print('c5', json.load(open('$OUT/c5.json'))['value'])"
tools/gpu_tree_stamps.sh $TAG
