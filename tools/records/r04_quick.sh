#!/bin/bash
# quick GPU check: selected test files (TESTS), then the bench without the CPU leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04q}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
