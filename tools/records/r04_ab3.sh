#!/bin/bash
# parity of the all-short / early-exit changes, then the current library (k5) against round 3's (r3)
# on the 30^3 chain, Sat64, C4 and the heavy products; then a kernel trace of the C4 and chain legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab3}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 600 python tools/ab.py --reps 2 --steps 100 --chain --sat64 --c4 r3 k5 k5:SLAT_NO_SHORT1=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt | cut -c1-900
timeout -k 10 400 python tools/ab_heavy.py --reps 1 r3 k5 tree > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 4 $OUT/heavy.txt | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ab.py --child --steps 20 --chain --c4 > $OUT/child.json 2> $OUT/child.err || { tail -20 $OUT/child.err; exit 1; }
cat $OUT/child.json
python3 tools/trace_table.py $OUT/trace > $OUT/trace_table.txt && head -30 $OUT/trace_table.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace -o run --output-format csv -- python3 tools/ab_heavy.py --child --legs rg,c5any,c5ord > $OUT/hchild.json 2> $OUT/hchild.err || { tail -20 $OUT/hchild.err; exit 1; }
cat $OUT/hchild.json
python3 tools/trace_table.py $OUT/htrace > $OUT/htrace_table.txt && head -25 $OUT/htrace_table.txt
