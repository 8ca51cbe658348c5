#!/bin/bash
# Diagnostic: the same short bench against experiment builds of libksim (tools/build_variants).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/variants
for f in kubernetes-schedule-simulator_amd/lib/libksim.so tools/build_variants/*.so; do
  KSIM_LIB=$f timeout -k 10 120 python3 bench.py --cpu-sample 0 --steps 30 > gpurun_out/variants/$(basename $(dirname $f))_$(basename $f).json 2>&1 || { echo "$f failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/variants/$(basename $(dirname $f))_$(basename $f).json $f
done
