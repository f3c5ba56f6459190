#!/bin/bash
# Round-3 call t: the GPU suite on the tree (long B rows four stretches per step, fat rows by block
# tickets); the stretch count 8 (lu8) and the old walk (lu1: one stretch, fat rows by stride) on the
# power-law / long-row products incl. the 2^18 C5; the default bench line; rocprofv3 trace + FETCH /
# WRITE passes of the headline alone (--no-c4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 1000 python tools/ab_heavy.py --reps 2 --big tree lu8 lu1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A4 summary $OUT/ab_heavy.txt
timeout -k 10 240 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/prof_pmc.sh $OUT/prof "--steps 20 --warmup 50 --no-c4" FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/prof_summary.py $OUT/prof/trace 20 > $OUT/prof_summary.md && head -16 $OUT/prof_summary.md
echo done
