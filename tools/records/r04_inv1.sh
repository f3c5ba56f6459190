#!/bin/bash
# the chain's first steps (all rows short): numeric phases and rows per tile; then the flat fat walk
# against a lowered fat threshold on the heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04inv1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_fat_rows_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_ph.so timeout -k 10 120 python tools/phases_chain.py 3 > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt
timeout -k 10 600 python tools/ab.py --reps 2 --steps 100 --chain r3 k6 k6:SLAT_TILE_ROWS=16 k6:SLAT_TILE_ROWS=64 k6:SLAT_SHORT1_ANY=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt | cut -c1-700
timeout -k 10 900 python tools/ab_heavy.py --reps 1 --big --legs rg,c5any,chain,c5big_any k6 k6:SLAT_FAT_MIN=2048 k6:SLAT_FAT_MIN=1024 k6:SLAT_FAT_MIN=512 > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 5 $OUT/heavy.txt | cut -c1-900
