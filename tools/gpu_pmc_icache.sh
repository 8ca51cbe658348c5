#!/bin/bash
# instruction-fetch counters of the C2x run (general persistent kernel)
set -o pipefail
TAG=${1:-ic}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -iE "ICACHE|IFETCH|WAIT_INST|INST_LEVEL|SQ_WAVE_CYCLES|SQ_BUSY_CYCLES" $OUT/avail.txt | head -40
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/p1 -o run -- python3 bench.py --workload c2x --cpu-sample 0 --steps 1 --warmup 0 > $OUT/p1.json 2> $OUT/p1.err || { echo "p1 failed"; tail -5 $OUT/p1.err; }
find $OUT/p1 -name '*counter_collection.csv' | head -2
