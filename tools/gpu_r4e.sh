#!/bin/bash
# C3 fast kernel: per-wave barrier stamps (diagnostic lib) and an A/B of library variants.
set -o pipefail
TAG=${1:-r4e}; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-tree --c4-pods 0 --steps 2 --warmup 0 --pods 200000 > $OUT/st_c3.json 2> $OUT/st_c3.err || { tail $OUT/st_c3.err; exit 1; }
grep stamps $OUT/st_c3.err | head -8
[ $# -gt 0 ] && bash tools/gpu_libab.sh "$@" -- --no-tree --c4-pods 0 --pods 200000 --steps 10
exit 0
