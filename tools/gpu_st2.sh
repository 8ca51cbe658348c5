#!/bin/bash
# C2x stamps breakdown of the general persistent kernel only (stamps library).
set -o pipefail
TAG=${1:-st}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 200 python3 bench.py --workload c2x --cpu-sample 0 --steps 2 --warmup 0 > $OUT/st.json 2> $OUT/st.err || { tail $OUT/st.err; exit 1; }
grep stamps $OUT/st.err
