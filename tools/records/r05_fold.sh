#!/bin/bash
# f64 fold order with in-order LDS atomic adds: edge-value and fold-order parity, then the heavy A/B
# against the read-add-write build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05fold}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_f64_fold_edge_gpu.py tests/test_f64_any_order_gpu.py tests/test_fat_rows_gpu.py tests/test_wide_hash_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 500 python3 tools/ab_heavy.py --reps 2 --big --legs c5big_ord tree rmw > $OUT/ab18.txt 2>&1 || { tail $OUT/ab18.txt; exit 1; }
tail -3 $OUT/ab18.txt
timeout -k 10 300 python3 tools/ab_heavy.py --reps 2 --legs c5ord tree rmw > $OUT/ab16.txt 2>&1 || { tail $OUT/ab16.txt; exit 1; }
tail -3 $OUT/ab16.txt
