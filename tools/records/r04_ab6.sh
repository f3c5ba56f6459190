#!/bin/bash
# the fold-order flattened fat walk (k8) against the per-entry walks (noflat: -DSLAT_FR_FLAT=0) on the
# heavy products; C4 with B read in CSR form by the short-row batches (SLAT_NO_ELL=1: no ELL image)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab6}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_spgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 400 python tools/ab.py --reps 2 --steps 100 --c4 k8 k8:SLAT_NO_ELL=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt | cut -c1-800
timeout -k 10 900 python tools/ab_heavy.py --reps 1 --big noflat k8 > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 3 $OUT/heavy.txt | cut -c1-900
