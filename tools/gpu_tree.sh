#!/bin/bash
# Tree mode (KSIM_MODE_TREE): its parity tests, then C3 / C4 bench lines in tree mode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-tree}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_tree.log 2>&1 || { echo "tree tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest_tree.log | head -30; tail -5 $OUT/pytest_tree.log; exit 1; }
tail -1 $OUT/pytest_tree.log
timeout -k 10 300 python3 bench.py --mode tree --cpu-sample 0 > $OUT/bench_c3_tree.json 2> $OUT/bench_c3_tree.err || { echo "bench c3 tree failed"; tail -20 $OUT/bench_c3_tree.err; exit 1; }
cut -c1-700 $OUT/bench_c3_tree.json
timeout -k 10 300 python3 bench.py --mode tree --workload c4 --cpu-sample 0 --batch 4096 --steps 10 > $OUT/bench_c4_tree.json 2> $OUT/bench_c4_tree.err || { echo "bench c4 tree failed"; tail -20 $OUT/bench_c4_tree.err; exit 1; }
cut -c1-700 $OUT/bench_c4_tree.json
