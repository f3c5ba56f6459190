#!/bin/bash
# headline step timeline: kernel trace of a short bench run, the last dispatches with their gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05ht}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o head --output-format csv -- python3 tools/prof_head.py > $OUT/head.log 2>&1 || { tail $OUT/head.log; exit 1; }
cat $OUT/head.log
python3 tools/trace_gaps.py $OUT/trace 20
python3 tools/trace_table.py $OUT/trace 8
