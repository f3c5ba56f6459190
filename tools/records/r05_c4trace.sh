#!/bin/bash
# C4 whole + one eighth (B prepared): kernel trace with per-dispatch gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c4t}; mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c4 --output-format csv -- python3 tools/prof_c4_eighth.py > $OUT/c4.log 2>&1 || { tail $OUT/c4.log; exit 1; }
grep C4 $OUT/c4.log
python3 tools/trace_gaps.py $OUT/trace 40 > $OUT/gaps.txt && cat $OUT/gaps.txt
python3 tools/trace_table.py $OUT/trace 12
