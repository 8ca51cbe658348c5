#!/bin/bash
# C4 streaming PMC passes + 4-rank node-sharded rehearsal on one device.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_pmc.sh pmc_c4 --workload c4 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c4 > /dev/null || exit 1
OUT=gpurun_out/r4; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --one-device --steps 6 --shard-steps 6 --cpu-sample 0 > $OUT/bench_4r.json 2> $OUT/bench_4r.err || { echo "4-rank bench failed"; tail -20 $OUT/bench_4r.err; exit 1; }
cat $OUT/bench_4r.json
