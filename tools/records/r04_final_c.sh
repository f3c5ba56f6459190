#!/bin/bash
# Round-4 final tree on one box: tools/r04_check.sh (GPU suite, smoke, bench, trace, FETCH / WRITE), then
# one rank's eighth of C4 and a kernel trace of the f64 fold-order C5 2^18 leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04c3}; mkdir -p $OUT
bash tools/r04_check.sh ${1:-r04c3} || exit 1
timeout -k 10 200 python tools/c4_eighth.py > $OUT/c4_eighth.json 2> $OUT/c4_eighth.err || { tail -20 $OUT/c4_eighth.err; exit 1; }
cat $OUT/c4_eighth.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5trace -o c5 --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_ord > $OUT/c5trace.log 2>&1 || { tail $OUT/c5trace.log; exit 1; }
grep -h "c5big_ord" $OUT/c5trace.log | tail -1
