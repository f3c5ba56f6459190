#!/bin/bash
# Round-5 baseline on one box: the default bench line, then a kernel trace of C4 whole vs one eighth
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05base}; mkdir -p $OUT
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c4e --output-format csv -- python3 tools/prof_c4_eighth.py > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep "C4" $OUT/trace.log
