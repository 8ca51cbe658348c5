#!/bin/bash
# One GPU-box pass for the round record: parity tests, the default bench line, the kernel-trace
# profile of the same bench, and a 2-rank node-sharded rehearsal on the one device.
# Usage (from the repo root on the GPU box): tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --cpu-sample 0 --steps 20 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --one-device --steps 10 --shard-steps 10 --cpu-sample 0 > $OUT/bench_2r.json 2> $OUT/bench_2r.err || { echo "2-rank bench failed"; tail -20 $OUT/bench_2r.err; exit 1; }
cat $OUT/bench_2r.json
