#!/bin/bash
# One GPU-box pass for the round record: parity tests, the default bench line, the kernel-trace
# profile of the SAME default bench command, the C2 bench line, and a 2-rank node-sharded
# rehearsal on the one device.  Usage (from the repo root on the GPU box): tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_gpu.log | head; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -14 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 python3 bench.py --workload c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "c2 bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
cut -c1-400 $OUT/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --workload c2 > $OUT/prof_bench_c2.json 2> $OUT/prof_c2.err || { echo "rocprof c2 failed"; tail -20 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --one-device --steps 10 --cpu-sample 0 > $OUT/bench_2r.json 2> $OUT/bench_2r.err || { echo "2-rank bench failed"; tail -20 $OUT/bench_2r.err; exit 1; }
cut -c1-600 $OUT/bench_2r.json
