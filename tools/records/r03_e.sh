#!/bin/bash
# Round-3 call e: full GPU tests (k_numeric at 3 waves/SIMD, early A-value loads of long rows);
# A/B tree vs late (A values re-read after the bitmap) and the grid knobs on the headline, C4 and
# Sat64; then the C4 kernel trace + FETCH/WRITE and SQ counter passes (tools/prof_c4.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree late tree:SLAT_SYM_BPC=7 tree:SLAT_NUM_OVER=2 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A8 summary $OUT/ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4trace -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4trace.log 2>&1 || { tail $OUT/c4trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $OUT/c4pmc1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1.log 2>&1 || { tail $OUT/c4pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $OUT/c4pmc2 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc2.log 2>&1 || { tail $OUT/c4pmc2.log; exit 1; }
echo done
