#!/bin/bash
# kernel traces with per-dispatch gaps: the headline step and C4 (whole, then one eighth)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06tr}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
grep headline $OUT/ht.log
python3 tools/trace_table.py $OUT/ht 6
python3 tools/trace_gaps.py $OUT/ht 12
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o c4 --output-format csv -- python3 tools/prof_c4_eighth.py > $OUT/c4.log 2>&1 || { tail $OUT/c4.log; exit 1; }
grep C4 $OUT/c4.log
python3 tools/trace_gaps.py $OUT/c4 12
