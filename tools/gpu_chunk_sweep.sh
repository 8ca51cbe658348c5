#!/bin/bash
# C2x pods/s of the general persistent kernel at several rows-per-workgroup (KSIM_PGEN_CHUNK).
set -o pipefail
TAG=${1:-chunk}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p $OUT
for CH in 96 128 160 192 256 384; do
  KSIM_PGEN_CHUNK=$CH timeout -k 10 200 python3 bench.py --workload c2x --cpu-sample 0 --per-pod-calls 0 > $OUT/c2x_$CH.json 2> $OUT/c2x_$CH.err || { echo "chunk $CH failed"; tail -5 $OUT/c2x_$CH.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c2x_$CH.json')); print($CH, d['value'], d['config']['blocks'], d['parity'])"
done
