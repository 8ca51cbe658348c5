set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cloop
for v in "KSIM_SERVE=0" "KSIM_SERVE_LIGHT=0" "KSIM_SERVE=1" "KSIM_SERVE=1"; do
  env $v KSIM_SERVE_STATS=1 timeout -k 10 200 python -u -m pytest tests/test_c_abi.py -m gpu -x -q --timeout 150 --timeout-method thread -k schedule_one_loop > gpurun_out/cloop/log 2>&1
  echo "$v rc=$? $(grep -E 'passed|failed' gpurun_out/cloop/log | tail -1) $(grep -m2 'FAIL ksim' gpurun_out/cloop/log | head -2 | tr '\n' ' ')"
done
