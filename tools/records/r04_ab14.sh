#!/bin/bash
# lane kernel: the aggregate published before the u32 outputs are staged, the look-back walked after
# (lb2) against the previous tree (pg4); fold-order walk depth 8 / 16 against 4 (fd4); parity first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab14}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_lb2.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_tiny_gpu.py -k "lane or golden or tiny or small" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lb2.log 2>&1 || { tail -40 $OUT/pytest_lb2.log; exit 1; }
tail -n 1 $OUT/pytest_lb2.log
SLAT_LIB_PATH=tools/var/libslat_fd16.so timeout -k 10 300 python -u -m pytest tests/test_fat_rows_gpu.py -k "f64 or fold or order" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_fd16.log 2>&1 || { tail -40 $OUT/pytest_fd16.log; exit 1; }
tail -n 1 $OUT/pytest_fd16.log
timeout -k 10 500 python tools/ab.py --reps 3 --steps 100 --chain pg4 lb2 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt | cut -c1-300
timeout -k 10 600 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord fd4 fd8 fd16 > $OUT/ab_fold.txt 2>&1 || { tail -30 $OUT/ab_fold.txt; exit 1; }
grep -A4 summary $OUT/ab_fold.txt
