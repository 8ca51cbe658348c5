#!/bin/bash
# PMC passes over the bench command (MI355X_MICROARCH.md HBM section: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc runs, --kernel-trace only beside them), then the per-kernel summary.
# Usage (repo root on the GPU box): tools/gpu_pmc_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "bench args: $*" > $OUT/args.txt
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --cpu-sample 0 "$@" > $OUT/fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --cpu-sample 0 "$@" > $OUT/write.json 2> $OUT/write.err || { echo "write pass failed"; tail $OUT/write.err; exit 1; }
python3 tools/pmc_summary.py $OUT > /dev/null && cat $OUT/pmc_summary.json | head -60
