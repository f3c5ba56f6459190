#!/bin/bash
# Round-4 check on one box: the GPU suite, smoke, the default bench line, then a rocprofv3 kernel trace
# and the FETCH_SIZE / WRITE_SIZE passes of the headline alone (each step under its own limit).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -z "$NO_PROF" ]; then
bash tools/prof_pmc.sh $OUT/prof "--steps 20 --warmup 50 --no-c4 --e2e-steps 0" FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/prof_summary.py $OUT/prof/trace 20 > $OUT/prof_summary.md && head -12 $OUT/prof_summary.md
python3 tools/pmc_headline.py $OUT/prof ${1:-r04a} > $OUT/pmc_torus30_a7.json && head -8 $OUT/pmc_torus30_a7.json
fi
