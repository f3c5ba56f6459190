#!/bin/bash
# Round-3 call y: the GPU suite on the tree (fat rows from 8192 products); k_numeric_short with a
# stage's ELL columns loaded before any is hashed (spre; spre4: at 4 waves/SIMD, no spills) on C4;
# the multi-rank path rehearsed on one GPU (dist tests, RCCL at world size 1, 2 gloo ranks)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03y; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 600 python tools/ab.py --reps 3 --c4 tree spre spre4 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
bash tools/r02_dist.sh r03y/dist || exit 1
echo done
