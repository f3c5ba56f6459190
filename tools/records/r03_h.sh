#!/bin/bash
# Round-3 call h: ticket queues with a static first round (no ticket for a wave's first item), on
# the wide launches' window / hash rows (default) and the short-row tiles (SLAT_DYN=3); GPU tests
# first, then A/B on the headline / C4 / Sat64 and the power-law products; host split of a call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree tree:SLAT_DYN=0 tree:SLAT_DYN=3 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A8 summary $OUT/ab.txt
timeout -k 10 1100 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_DYN=0 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A8 summary $OUT/ab_heavy.txt
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -20 $OUT/host.txt
echo done
