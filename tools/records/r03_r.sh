#!/bin/bash
# Round-3 call r: the GPU suite on the tree (packed emit sort on, small path <= 2048 rows);
# k_symbolic_short's batch bound (variants sc50 / sc85 against 70 %) on C4; a kernel trace of the
# RG R-MAT 2^16 A^2 products; the reference's two harnesses (repeat: the Sat64 chain; sweep: the
# C3 grid)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 600 python tools/ab.py --reps 3 --c4 tree sc50 sc85 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rg -o rg --output-format csv -- python3 tools/prof_rg.py > $OUT/rg.log 2>&1 || { tail -30 $OUT/rg.log; exit 1; }
tail -4 $OUT/rg.log
timeout -k 10 300 python tools/bench_protocol.py repeat > $OUT/repeat.csv 2> $OUT/repeat.err || { tail -30 $OUT/repeat.err; exit 1; }
cat $OUT/repeat.csv
timeout -k 10 300 python tools/bench_protocol.py sweep > $OUT/sweep.csv 2> $OUT/sweep.err || { tail -30 $OUT/sweep.err; exit 1; }
tail -22 $OUT/sweep.csv
echo done
