#!/bin/bash
# A/B of the workgroup-per-row kernels and the single-window short rows against the round-3 path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab1}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 600 python tools/ab.py --reps 2 --steps 100 --chain --sat64 knobs knobs:SLAT_NO_GROUP=1 g2 g3 g3:SLAT_GRP_NUM_T=128 g3:SLAT_GRP_SYM_T=256 g3:SLAT_NO_SHORT1=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
