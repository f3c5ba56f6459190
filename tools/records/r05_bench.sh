#!/bin/bash
# the default bench line on the current tree, C4 whole vs eighths, and a kernel trace of C1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05b}; mkdir -p $OUT
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c1trace -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/c1trace.log 2>&1 || { tail $OUT/c1trace.log; exit 1; }
grep "C1" $OUT/c1trace.log | tail -3
