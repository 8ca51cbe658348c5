#!/bin/bash
# Per-pod pick kernel: the per-pod suites forced through the multi-block path (KSIM_ONE_WG=0; the
# resident form unless KSIM_SERVE=0 is exported), then the C2 / C2x per_pod lines for the resident
# form (serve=1), per-pod launches of the pick kernel (serve=0) and the scan kernel (KSIM_NO_PICK=1).
# Usage (GPU box, repo root): tools/gpu_pick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-pick}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
KSIM_SERVE_STATS=1 KSIM_ONE_WG=0 timeout -k 10 700 python -u -m pytest tests/test_gpu_cache.py tests/test_c_abi.py tests/test_gpu_wide.py \
  tests/test_gpu_affinity.py tests/test_gpu_volumes.py tests/test_gpu_spread.py tests/test_gpu_service_affinity.py \
  -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_pick.log 2>&1 \
  || { echo "pick tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_pick.log | head -20; exit 1; }
tail -2 $OUT/pytest_pick.log
for w in c2 c2x; do
  for v in serve launch scan; do
    KSIM_SERVE=$([ $v = serve ] && echo 1 || echo 0) KSIM_NO_PICK=$([ $v = scan ] && echo 1 || echo 0) KSIM_SERVE_STATS=1 \
      timeout -k 10 300 python3 bench.py --workload $w --cpu-sample 0 --steps 2 --warmup 1 > $OUT/bench_${w}_$v.json 2> $OUT/bench_${w}_$v.err || { tail $OUT/bench_${w}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_${w}_$v.json')); p=d.get('per_pod') or {}; print('$w $v', [(m['cached_pods'], m['us_per_call'], m['p99_us'], m['adapter_pattern']['us_per_pod'], m['adapter_pattern']['p99_us']) for m in p.get('marks', [])])"
    grep "ksim serve" $OUT/bench_${w}_$v.err | tail -2 || true
  done
done
