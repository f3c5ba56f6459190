#!/bin/bash
# GPU parity suite + the default bench line (one box, each step under its own time limit).
set -o pipefail
OUT=gpurun_out/${1:-gt}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
