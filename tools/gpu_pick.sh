#!/bin/bash
# Per-pod pick kernel: the per-pod suites forced through the multi-block path (KSIM_ONE_WG=0),
# then the C2 / C2x per_pod lines with and without it (KSIM_NO_PICK=1).
# Usage (GPU box, repo root): tools/gpu_pick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-pick}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
KSIM_ONE_WG=0 timeout -k 10 700 python -u -m pytest tests/test_gpu_cache.py tests/test_c_abi.py tests/test_gpu_wide.py \
  tests/test_gpu_affinity.py tests/test_gpu_volumes.py tests/test_gpu_spread.py tests/test_gpu_service_affinity.py \
  -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_pick.log 2>&1 \
  || { echo "pick tests failed"; grep -E "^E |FAILED|Timeout" $OUT/pytest_pick.log | head -20; exit 1; }
tail -2 $OUT/pytest_pick.log
for w in c2 c2x; do
  for v in 0 1; do
    KSIM_NO_PICK=$v timeout -k 10 300 python3 bench.py --workload $w --cpu-sample 0 --steps 2 --warmup 1 > $OUT/bench_${w}_$v.json 2> $OUT/bench_${w}_$v.err || { tail $OUT/bench_${w}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_${w}_$v.json')); p=d.get('per_pod') or {}; print('$w no_pick=$v', [(m['cached_pods'], m['us_per_call'], m['p99_us'], m['adapter_pattern']['us_per_pod']) for m in p.get('marks', [])])"
  done
done
