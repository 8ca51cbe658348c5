#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-k8s}; mkdir -p $OUT
timeout -k 10 300 ./tests/c/build/ksim_k8s_loop 240 1500 > $OUT/k8s_loop.log 2>&1; echo "k8s loop rc=$?"; tail -12 $OUT/k8s_loop.log
timeout -k 10 300 ./tests/c/build/ksim_k8s_loop 30 1500 > $OUT/k8s_loop_sat.log 2>&1; echo "k8s loop (saturated) rc=$?"; tail -12 $OUT/k8s_loop_sat.log
