#!/bin/bash
# Round-3 call p: the one-kernel small path (regular launch, block look-back) — its tests and the
# small cells against the pipeline; contiguous row runs per wave (variant contig) and the
# rebuilt-bitmap numeric (SLAT_NO_SBM=1) A/B on the headline / C4 / Sat64; C4 phase counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tiny_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 300 python tools/small_cells.py > $OUT/small_cells.csv 2>&1 || { tail -30 $OUT/small_cells.csv; exit 1; }
cat $OUT/small_cells.csv
timeout -k 10 900 python tools/ab.py --reps 3 --c4 --sat64 tree contig tree:SLAT_NO_SBM=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 200 python tools/prof_c4.py > $OUT/phases_c4.txt 2>&1 || { tail -30 $OUT/phases_c4.txt; exit 1; }
tail -6 $OUT/phases_c4.txt
echo done
