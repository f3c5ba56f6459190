#!/bin/bash
# Round-3 call ae: LDS hash probe checks as selects (variant sel: every round consumes all its CAS
# results, so the next round's CASes issue back to back; the CASes keep their per-key branches):
# GPU suite on it, A/B on C4 / the headline and the heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ae; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_sel.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_sel.log 2>&1 || { tail -40 $OUT/tests_sel.log; exit 1; }
tail -n 1 $OUT/tests_sel.log
timeout -k 10 600 python tools/ab.py --reps 4 --c4 tree sel > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
timeout -k 10 600 python tools/ab_heavy.py --reps 2 tree sel > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
echo done
