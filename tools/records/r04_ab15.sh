#!/bin/bash
# the tree (lane look-back split, fold-order walk 16 entries deep, ordered traversal double-buffered):
# parity of the f64 / fat / lane paths, then the ordered traversal single-buffered (odb0) and the
# fold walk 32 deep (fd32) against the tree on the fold-order legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab15}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_tiny_gpu.py tests/test_spgemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 700 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord,c5any odb0 tree fd32 > $OUT/ab_fold.txt 2>&1 || { tail -30 $OUT/ab_fold.txt; exit 1; }
grep -A4 summary $OUT/ab_fold.txt
