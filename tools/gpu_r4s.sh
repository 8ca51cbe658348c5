#!/bin/bash
# Round-4 end record: the whole -m gpu suite (full-size scale tests included) + smoke, then a
# one-device 2-rank rehearsal of the N>1 bench path (both ranks on device 0: correctness only).
set -o pipefail
TAG=${1:-r4s}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head -30; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -20 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --cpu-sample 0 --one-device > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo "n2 bench failed"; tail -30 $OUT/bench_n2.err; exit 1; }
cut -c1-400 $OUT/bench_n2.json
