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
# the ELL image of a row block built only over the B rows its columns reference (ellr = the tree's
# sources with that change): parity, then one rank's eighth of C4 against the tree's library
SLAT_LIB_PATH=tools/var/libslat_ellr.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_dist_gpu.py tests/test_tiny_gpu.py -k "rowblock or dist or block or gather or cuts" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ellr.log 2>&1 || { tail -40 $OUT/pytest_ellr.log; exit 1; }
tail -n 1 $OUT/pytest_ellr.log
for L in ellr tree ellr tree; do
  if [ $L = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=tools/var/libslat_$L.so; fi
  timeout -k 10 200 python tools/c4_eighth.py > $OUT/eighth_$L.json 2> $OUT/eighth.err || { tail -20 $OUT/eighth.err; exit 1; }
  echo "$L $(cat $OUT/eighth_$L.json)"
done
