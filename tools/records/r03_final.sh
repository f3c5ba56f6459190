#!/bin/bash
# Round-3 final check on one box: the GPU suite, smoke, the default bench line, rocprofv3 trace +
# FETCH / WRITE passes of the headline alone, the headline / C4 / Sat64 and heavy legs (tree), the
# small cells
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03final; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 240 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/prof_pmc.sh $OUT/prof "--steps 20 --warmup 50 --no-c4" FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/prof_summary.py $OUT/prof/trace 20 > $OUT/prof_summary.md && head -12 $OUT/prof_summary.md
timeout -k 10 600 python tools/ab.py --reps 3 --c4 --sat64 tree > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A2 summary $OUT/ab.txt
timeout -k 10 600 python tools/ab_heavy.py --reps 2 --big tree > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A2 summary $OUT/ab_heavy.txt
timeout -k 10 400 python tools/small_cells.py > $OUT/small_cells.csv 2>&1 || { tail -30 $OUT/small_cells.csv; exit 1; }
echo done
