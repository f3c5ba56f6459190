#!/bin/bash
# k_numeric / k_numeric_short with the pattern-B shortcut (base = the tree) against without (numuni0):
# the fat walk's version of it measured slower (r04ab19), so the window / hash kernels' one is re-taken
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab20}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_numuni0.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "pattern or golden or narrow" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 700 python tools/ab.py --reps 3 --steps 100 --chain --c4 base numuni0 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt | cut -c1-400
