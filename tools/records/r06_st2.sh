#!/bin/bash
# MODE 4 (stored-bitmap pair) against MODE 0 on the headline, Sat64 and the 30^3 chain (knobs build),
# then the headline kernel trace of the tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06st2}; mkdir -p $OUT
timeout -k 10 400 python3 tools/ab.py --reps 2 --sat64 --chain knobs knobs:SLAT_NO_STORED_MODE=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
tail -3 $OUT/ht.log
python3 tools/trace_table.py $OUT/ht 8
