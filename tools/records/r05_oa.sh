#!/bin/bash
# f64 fold order, window / hash rows: entries whose B loads run ahead (SLAT_ORD_AHEAD 8 in tree; variants 16, 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05oa}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_oa16.so timeout -k 10 300 python -u -m pytest tests/test_f64_fold_edge_gpu.py tests/test_fat_rows_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_oa16.log 2>&1 || { tail -30 $OUT/pytest_oa16.log; exit 1; }
tail -1 $OUT/pytest_oa16.log
timeout -k 10 700 python3 tools/ab_heavy.py --reps 2 --big --legs c5big_ord tree oa16 oa4 > $OUT/ab18.txt 2>&1 || { tail $OUT/ab18.txt; exit 1; }
tail -4 $OUT/ab18.txt
