#!/bin/bash
# Round 4, first GPU pass: the full-size parity tests (whole 1M-pod C3 queue vs the C oracle, the
# 1M-node world-8 shard rehearsal), the exchange floors (tools/xchg_bench*.hip) and the C3 grid sweep.
set -o pipefail
TAG=${1:-r4a}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 ./tools/build_xchg2 > $OUT/xchg2.txt 2>&1; echo "xchg2 rc=$?"; cat $OUT/xchg2.txt
timeout -k 10 60 ./tools/build_xchg > $OUT/xchg.txt 2>&1; echo "xchg rc=$?"; cat $OUT/xchg.txt
for g in 256 192 128 96 64; do
  KSIM_MAX_GRID=$g timeout -k 10 120 python3 bench.py --cpu-sample 0 --no-tree --c4-pods 0 --steps 10 --warmup 1 > $OUT/grid_$g.json 2>$OUT/grid_$g.err || { echo "grid $g failed"; tail -5 $OUT/grid_$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/grid_$g.json')); print($g, d['value'], d['config'].get('blocks'), d['roofline']['avg_launch_us'])"
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 \
  -k "full_queue or c4_shape or multi_process" > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest.log | head -30; tail -30 $OUT/pytest.log; exit 1; }
tail -15 $OUT/pytest.log
