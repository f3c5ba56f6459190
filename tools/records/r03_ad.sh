#!/bin/bash
# Round-3 call ad: k_numeric emit, four 64-slot stretches per step (variant eu); symbolic popcounts of up to eight touched blocks per step (sp8); k_numeric rank lookups of 2 / 4 groups issued together (aq2, aq4):
# targeted tests, A/B on the headline / C4 / Sat64; the default bench line twice (box spread)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ad; mkdir -p $OUT
for v in eu sp8 aq2 aq4; do
SLAT_LIB_PATH=tools/var/libslat_$v.so timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_wide_hash_gpu.py tests/test_graph_gpu.py tests/test_magnus_usize_gpu.py tests/test_real_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { tail -40 $OUT/tests_$v.log; exit 1; }
done
tail -n 1 $OUT/tests_$v.log
timeout -k 10 900 python tools/ab.py --reps 4 --c4 --sat64 tree eu sp8 aq2 aq4 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt
echo done
