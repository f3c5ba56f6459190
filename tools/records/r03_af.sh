#!/bin/bash
# Round-3 call af: the short-row batches' entry -> row marker reads issued together (variant mk):
# targeted tests, A/B on C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03af; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_mk.so timeout -k 10 400 python -u -m pytest tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_mk.log 2>&1 || { tail -40 $OUT/tests_mk.log; exit 1; }
tail -n 1 $OUT/tests_mk.log
timeout -k 10 600 python tools/ab.py --reps 4 --c4 tree mk > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
echo done
