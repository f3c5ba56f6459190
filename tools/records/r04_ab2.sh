#!/bin/bash
# parity of the short-row category on single-window launches (tiles of T rows, listed long rows by the
# wave kernels), then the A/B against the round-3 path and the workgroup kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab2}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 600 python tools/ab.py --reps 2 --steps 100 --chain --sat64 k4 k4:SLAT_NO_SHORT1=1 k4:SLAT_GROUP=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt | cut -c1-600
