#!/bin/bash
# round-6 baseline on one box: headline + C4 A/B line of the tree, headline kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06base}; mkdir -p $OUT
timeout -k 10 300 python3 tools/ab.py --reps 1 --c4 tree > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
cat $OUT/ht.log
python3 tools/trace_table.py $OUT/ht 8
