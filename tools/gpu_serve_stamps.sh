#!/bin/bash
# The resident per-pod kernel's phase stamps (make stamps) on the C2 / C2x per_pod lines.
# Usage (GPU box, repo root): tools/gpu_serve_stamps.sh <tag>
set -o pipefail
TAG=${1:-serve_stamps}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for w in ${WORKLOADS:-c2 c2x}; do
  KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 300 python3 bench.py --workload $w --cpu-sample 0 --steps 2 --warmup 1 \
    > $OUT/st_${w}.json 2> $OUT/st_${w}.err || { tail $OUT/st_${w}.err; exit 1; }
  echo "== $w stamps"; grep "stamps\] serve" $OUT/st_${w}.err | sort -t: -k2 | tail -1 || true
done
