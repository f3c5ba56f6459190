#!/bin/bash
# One GPU call: parity tests, smoke, default bench, rocprofv3 trace + FETCH/WRITE PMC passes.
# usage: tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 240 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/prof_pmc.sh $OUT/prof "--steps 20 --warmup 50" FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/prof_summary.py $OUT/prof/trace 20 > $OUT/prof_summary.md && head -20 $OUT/prof_summary.md
