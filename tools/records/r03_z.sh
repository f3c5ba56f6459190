#!/bin/bash
# Round-3 call z: branch-free LDS hash probe rounds (variant nb: settled keys CAS a per-lane dummy
# word, so a round's CASes issue back to back instead of each behind an lgkmcnt(0) wait): the hash
# categories' tests and the GPU suite on it, then A/B on C4 / the headline / the heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03z; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_nb.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_nb.log 2>&1 || { tail -40 $OUT/tests_nb.log; exit 1; }
tail -n 1 $OUT/tests_nb.log
timeout -k 10 600 python tools/ab.py --reps 4 --c4 tree nb > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
timeout -k 10 600 python tools/ab_heavy.py --reps 2 tree nb > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
echo done
