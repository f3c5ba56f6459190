#!/bin/bash
# the next row's bounds (and C offsets, stored block mask) loaded ahead in the single-window passes:
# numeric (rpn), symbolic (rps), both (rpb) against the tree; parity first (rpb)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab16}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_rpb.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_reorder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 700 python tools/ab.py --reps 3 --steps 200 --chain --sat64 tree rpn rps rpb > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A5 summary $OUT/ab.txt | cut -c1-400
