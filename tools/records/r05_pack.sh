#!/bin/bash
# fold-order fat walk with several entries' parts per wave instruction (variant library pack): parity, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05pack}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_pack.so timeout -k 10 300 python -u -m pytest tests/test_f64_fold_edge_gpu.py tests/test_f64_any_order_gpu.py tests/test_fat_rows_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_pack.log 2>&1 || { tail -30 $OUT/pytest_pack.log; exit 1; }
tail -1 $OUT/pytest_pack.log
timeout -k 10 600 python3 tools/ab_heavy.py --reps 2 --big --legs c5big_ord tree pack > $OUT/ab18.txt 2>&1 || { tail $OUT/ab18.txt; exit 1; }
tail -4 $OUT/ab18.txt
