#!/bin/bash
# Tree-mode iteration: tree + sweep parity tests, then stamps and C3 / C4 / C5 tree bench lines.
# Usage (from the repo root on the GPU box): tools/gpu_tree_iter.sh <tag>
set -o pipefail
TAG=${1:-ti}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tree or sweep" > $OUT/pytest_tree.log 2>&1 || { echo "tree tests failed"; tail -30 $OUT/pytest_tree.log; exit 1; }
tail -2 $OUT/pytest_tree.log
tools/gpu_tree_stamps.sh $TAG || exit 1
timeout -k 10 200 python3 bench.py --mode tree --cpu-sample 0 --steps 20 > $OUT/c3_tree.json 2> $OUT/c3_tree.err || { echo "c3 tree failed"; tail $OUT/c3_tree.err; exit 1; }
cat $OUT/c3_tree.json
timeout -k 10 300 python3 bench.py --workload c5 --cpu-sample 0 --steps 3 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { echo "c5 failed"; tail $OUT/c5.err; exit 1; }
cat $OUT/c5.json
