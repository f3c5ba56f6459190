#!/bin/bash
# Round-3 call s: packed stored bitmaps (variant spk: only the non-zero words of each touched block
# plus a word mask) on the headline / Sat64; long B rows walked four 64-entry stretches per step
# (variant lu), fat rows by block tickets (ft), both (luft) on the power-law / long-row products;
# the GPU suite on spk and luft first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03s; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_spk.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_spk.log 2>&1 || { tail -40 $OUT/tests_spk.log; exit 1; }
tail -n 1 $OUT/tests_spk.log
SLAT_LIB_PATH=tools/var/libslat_luft.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_luft.log 2>&1 || { tail -40 $OUT/tests_luft.log; exit 1; }
tail -n 1 $OUT/tests_luft.log
timeout -k 10 600 python tools/ab.py --reps 4 --sat64 tree spk > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
timeout -k 10 900 python tools/ab_heavy.py --reps 2 tree lu ft luft > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A5 summary $OUT/ab_heavy.txt
echo done
