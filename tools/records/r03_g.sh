#!/bin/bash
# Round-3 call g: per-mode work distribution (tickets for the wide launches' window / hash rows,
# twice the resident blocks for the short-row tiles) and XCD-contiguous tile ranges (noxcd = plain
# stride), the completion word stored by the last kernel (vs a k_signal launch); GPU tests first, then A/B on the headline / C4 / Sat64 and the power-law products, and
# C4's FETCH_SIZE pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree noxcd tree:SLAT_DYN=0 tree:SLAT_NUM_OVER=3 tree:SLAT_NO_FUSED_SIGNAL=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A8 summary $OUT/ab.txt
timeout -k 10 1100 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_DYN=0 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A8 summary $OUT/ab_heavy.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c4pmc1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1.log 2>&1 || { tail $OUT/c4pmc1.log; exit 1; }
SLAT_LIB_PATH=tools/var/libslat_noxcd.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c4pmc1n -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1n.log 2>&1 || { tail $OUT/c4pmc1n.log; exit 1; }
echo done
