#!/bin/bash
# fold-order fat walk holding only each entry's lane (variant libraries ft, ft24): parity, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05ft}; mkdir -p $OUT
for v in ft ft24; do
SLAT_LIB_PATH=tools/var/libslat_$v.so timeout -k 10 300 python -u -m pytest tests/test_f64_fold_edge_gpu.py tests/test_f64_any_order_gpu.py tests/test_fat_rows_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
echo $v; tail -1 $OUT/pytest_$v.log; done
timeout -k 10 600 python3 tools/ab_heavy.py --reps 2 --big --legs c5big_ord tree ft ft24 > $OUT/ab18.txt 2>&1 || { tail $OUT/ab18.txt; exit 1; }
tail -4 $OUT/ab18.txt
