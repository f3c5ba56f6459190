#!/bin/bash
# round-5 closing check on one box: the GPU suite and the default bench line on the final tree, then
# the A/B of 32 KB fat-row chunks for the atomic semirings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05final2}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 300 $OUT/bench.json; echo
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 500 python3 tools/ab_heavy.py --reps 2 --big --legs c5big_any,c5big_ord tree fr32 > $OUT/ab18.txt 2>&1 || { tail $OUT/ab18.txt; exit 1; }
tail -3 $OUT/ab18.txt
