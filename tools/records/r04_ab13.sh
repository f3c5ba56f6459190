#!/bin/bash
# f64 fat rows in the reference's fold order: the per-entry walk's B loads four entries ahead (fd4,
# the tree) against one ahead (fd1); wide launches' short-row tiles by row count (the tree) against
# 64-row tiles (pg4: the previous tree); parity first (f64 / fat-row / wide tests)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab13}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_wide_hash_gpu.py tests/test_spgemm_gpu.py -k "f64 or fold or fat or order or wide or hash or short" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 800 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord,c5any fd1 fd4 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 300 python tools/ab.py --reps 2 --steps 50 --c4 pg4 tree > $OUT/ab_c4.txt 2>&1 || { tail -30 $OUT/ab_c4.txt; exit 1; }
grep -A3 summary $OUT/ab_c4.txt | cut -c1-300
timeout -k 10 200 python tools/c4_eighth.py > $OUT/eighth.json 2> $OUT/eighth.err || { tail -20 $OUT/eighth.err; exit 1; }
cat $OUT/eighth.json
