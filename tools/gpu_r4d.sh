#!/bin/bash
# Round 4: the reworked fast persistent kernel (split sweep, local fix, top-list select) —
# exchange floors, C3 rate + stamps, parity, then the per-pod line through the C++ cache.
set -o pipefail
TAG=${1:-r4d}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 tools/build_xchg2 > $OUT/xchg2.txt 2>&1 || { cat $OUT/xchg2.txt; exit 1; }
cat $OUT/xchg2.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; grep -E "^E |FAILED|Timeout" $OUT/parity.log | head -30; tail -20 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-tree --c4-pods 0 --steps 30 --warmup 2 > $OUT/c3.json 2> $OUT/c3.err || { tail $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c3.json')); print('C3', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_us'))"
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-tree --c4-pods 0 --steps 2 --warmup 0 --pods 200000 > $OUT/st_c3.json 2> $OUT/st_c3.err || { tail $OUT/st_c3.err; exit 1; }
grep stamps $OUT/st_c3.err | head -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 500 --timeout-method thread -k "c3_full or c3_saturated or c4_3000" > $OUT/scale.log 2>&1 || { echo "scale failed"; grep -E "^E |FAILED|Timeout" $OUT/scale.log | head -30; exit 1; }
tail -3 $OUT/scale.log
