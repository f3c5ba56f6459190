#!/bin/bash
# the flattened fat-row walk: parity of the fat-row / power-law tests, then the heavy products against
# the walk before it (k5), with the fat threshold lowered (SLAT_FAT_MIN) as the flat walk may allow
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab4}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 900 python tools/ab_heavy.py --reps 1 --big ${VARIANTS:-k5 flat flat:SLAT_FAT_MIN=2048 flat:SLAT_FAT_MIN=1024} > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 5 $OUT/heavy.txt | cut -c1-900
