#!/bin/bash
# Round-3 call m: per-block max row counts from symbolic (reduced by the scan's last tile), tickets
# compiled out of the single-window and short-row instances (registers back to the round's start);
# GPU tests first, then A/B on the headline / C4 / Sat64 / power-law products and the host split
# (first 64 calls not counted)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 3 --c4 --sat64 tree > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
timeout -k 10 900 python tools/ab_heavy.py --reps 1 --big tree > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -4 $OUT/host.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo done
