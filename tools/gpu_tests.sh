#!/bin/bash
# GPU-box test pass: the given pytest targets (default: the whole -m gpu suite), each step under
# its own time limit; stops at the first failure.  Usage: tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
TAG=${1:-tests}
shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -25 $OUT/pytest.log
exit $rc
