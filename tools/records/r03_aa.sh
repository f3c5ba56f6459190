#!/bin/bash
# Round-3 call aa: the LDS hash tables' first probe round branch-free (nb2), and the round-2
# symbolic ballot patch re-applied (ballot: one-window symbolic finds its touched blocks by a ballot
# per bitmap block afterwards, no per-product block mask): tests, then A/B on the headline / C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03aa; mkdir -p $OUT
for v in nb2 ballot; do
SLAT_LIB_PATH=tools/var/libslat_$v.so timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_tiny_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1 || { tail -40 $OUT/tests_$v.log; exit 1; }
tail -n 1 $OUT/tests_$v.log
done
timeout -k 10 900 python tools/ab.py --reps 4 --c4 tree nb2 ballot > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
echo done
