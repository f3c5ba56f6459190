#!/bin/bash
# Round-3 call i: the one-kernel small path (slat_tiny.hip) and its tests; ordered f64 fat rows with
# a per-wave-slice split table (SLAT_NO_FAT_SLICES=1: the chunk table + a 64-ary search per A
# entry); env knobs read once and the free-memory query only after the pool changes. GPU tests
# first (the new tiny tests before the rest), then the host split of a call, the C3 sweep (small
# cells), and the A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tiny_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_tiny.log 2>&1 || { tail -40 $OUT/tests_tiny.log; exit 1; }
tail -n 2 $OUT/tests_tiny.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -5 $OUT/host.txt
timeout -k 10 300 python tools/small_cells.py > $OUT/small.csv 2> $OUT/small.err || { tail -30 $OUT/small.err; exit 1; }
cat $OUT/small.csv
timeout -k 10 1100 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord tree tree:SLAT_NO_FAT_SLICES=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A4 summary $OUT/ab_heavy.txt
timeout -k 10 600 python tools/ab.py --reps 2 --c4 --sat64 tree > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
echo done
