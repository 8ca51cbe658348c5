#!/bin/bash
# Tree-form sweep: sweep + tree parity tests, then C5 bench in tree and scan forms.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-swt}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tree.py -x -q --timeout 200 --timeout-method thread -k "sweep or tree" > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|Error" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --workload c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench c5 failed"; tail -20 $OUT/bench_c5.err; exit 1; }
cut -c1-400 $OUT/bench_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --workload c5 --cpu-sample 0 > $OUT/prof_c5.json 2> $OUT/prof.err || { echo "prof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
