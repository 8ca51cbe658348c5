#!/bin/bash
# Per-pod call breakdown (KSIM_CACHE_PROFILE=1): the C2 / C2x per_pod lines, resident form and
# per-pod launches; prints the cache / schedule_one phase profiles.
# Usage (GPU box, repo root): tools/gpu_perpod_prof.sh <tag>
set -o pipefail
TAG=${1:-pprof}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for w in ${WORKLOADS:-c2 c2x}; do
  for v in 1 0; do
    KSIM_SERVE=$v KSIM_CACHE_PROFILE=1 KSIM_SERVE_STATS=1 timeout -k 10 300 python3 bench.py --workload $w --cpu-sample 0 --steps 2 --warmup 1 \
      > $OUT/bench_${w}_$v.json 2> $OUT/bench_${w}_$v.err || { tail $OUT/bench_${w}_$v.err; exit 1; }
    echo "== $w serve=$v"
    grep -E "profile\]|ksim serve" $OUT/bench_${w}_$v.err | tail -6 || true
  done
done
# the resident kernel's phase stamps (make stamps)
if [ -n "$STAMPS" ]; then
  for w in ${WORKLOADS:-c2 c2x}; do
    KSIM_LIB=kubernetes-schedule-simulator_amd/lib/stamps/libksim.so timeout -k 10 300 python3 bench.py --workload $w --cpu-sample 0 --steps 2 --warmup 1 \
      > $OUT/st_${w}.json 2> $OUT/st_${w}.err || { tail $OUT/st_${w}.err; exit 1; }
    echo "== $w stamps"; grep "stamps\] serve" $OUT/st_${w}.err | tail -3 || true
  done
fi
