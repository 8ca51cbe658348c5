#!/bin/bash
# GPU-box bench pass: the driver's bench command, the rocprofv3 kernel trace of that SAME command
# (summary for profiles/), and a 2-rank node-sharded rehearsal on the one device.
# Usage: tools/gpu_bench.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-bench}
shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
CMD="bench.py --gpus 1 --steps 20 --warmup 5 $*"
timeout -k 10 300 python -u $CMD > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $CMD > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
if [ -z "$NO_2R" ]; then
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --one-device --steps 10 --warmup 2 --cpu-sample 0 --no-tree --pods 200000 $* > $OUT/bench_2r.json 2> $OUT/bench_2r.err || { echo "2-rank bench failed"; tail -20 $OUT/bench_2r.err; exit 1; }
cat $OUT/bench_2r.json
fi
