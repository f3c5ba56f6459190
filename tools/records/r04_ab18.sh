#!/bin/bash
# R-MAT 2^16 A^2 (RG) took 4.39 ms at r04ab5 / ab6 and 6.1 ms on the final tree: the same leg on
# libraries built at the commits between (b<commit>) and the tree; the lane-overflow pair cache's test first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab18}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "lane" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 700 python tools/ab_heavy.py --reps 2 --legs rg,c5any bf4ca692 bf53db0a b46e3417 be670ace tree > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt
