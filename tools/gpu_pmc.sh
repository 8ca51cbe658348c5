#!/bin/bash
# PMC passes (one counter group per run, MI355X_MICROARCH.md HBM section) over a short bench,
# plus the stamps diagnostic build.  Usage: tools/gpu_pmc.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --cpu-sample 0 --steps 5 --warmup 1 "$@" > $OUT/fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --cpu-sample 0 --steps 5 --warmup 1 "$@" > $OUT/write.json 2> $OUT/write.err || { echo "write pass failed"; tail $OUT/write.err; exit 1; }
if [ -f kubernetes-schedule-simulator_amd/lib/stamps/libksim.so ]; then
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 5 --warmup 1 "$@" > $OUT/stamps.json 2> $OUT/stamps.err || { echo "stamps failed"; tail $OUT/stamps.err; exit 1; }
  grep 'ksim stamps' $OUT/stamps.err | tail -4
fi
ls -R $OUT | head -30
